# Lion K2 majority (all-gather exchange) two chunks per block (variant pm) vs default: kernel tests on the variant, then the roofline bench interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ax
DLION_LIB=variants/_dlion_C_pm.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "prevoted or vote_reduce or vote_apply or majority" --timeout 120 --timeout-method thread > gpurun_out/r3ax/tests_pm.log 2>&1 || { tail -40 gpurun_out/r3ax/tests_pm.log; exit 1; }
tail -1 gpurun_out/r3ax/tests_pm.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "majority or prevoted" --timeout 120 --timeout-method thread > gpurun_out/r3ax/tests_default.log 2>&1 || { tail -40 gpurun_out/r3ax/tests_default.log; exit 1; }
tail -1 gpurun_out/r3ax/tests_default.log
for r in 1 2; do
  for m in gpt2 llama3; do
    echo "== default $m"; timeout -k 10 200 python -u tools/bench_lion.py $m 8 || exit 1
    echo "== pm $m"; DLION_LIB=variants/_dlion_C_pm.so timeout -k 10 200 python -u tools/bench_lion.py $m 8 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | grep -E "==|K2" | tee gpurun_out/r3ax/lion_ab.txt
