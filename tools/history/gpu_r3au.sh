# Lion K2 pre-voted apply two chunks per block + K4 two words per thread (variant lionP) vs default: kernel tests on the variant, then the roofline bench interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3au
DLION_LIB=variants/_dlion_C_lionP.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "prevoted or vote_reduce or vote_apply" --timeout 120 --timeout-method thread > gpurun_out/r3au/tests_lionP.log 2>&1 || { tail -40 gpurun_out/r3au/tests_lionP.log; exit 1; }
tail -1 gpurun_out/r3au/tests_lionP.log
for r in 1 2; do
  for m in gpt2 llama3; do
    echo "== default $m"; timeout -k 10 200 python -u tools/bench_lion.py $m 8 || exit 1
    echo "== lionP $m"; DLION_LIB=variants/_dlion_C_lionP.so timeout -k 10 200 python -u tools/bench_lion.py $m 8 || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3au/lion_ab.txt
