# dQ kernel with 2 key tiles per barrier (NT=2, 194 VGPRs / 2 waves) vs NT=1 (133 / 3 waves): numerics + kernel A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3v
DLION_LIB=$PWD/variants/_dlion_C_nt2.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3v/attn_tests_nt2.log 2>&1 || { tail -30 gpurun_out/r3v/attn_tests_nt2.log; exit 1; }
tail -1 gpurun_out/r3v/attn_tests_nt2.log
for rep in 1 2 3; do
for v in default nt2; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  echo "== $v"
  DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py 20 1024 12 64 0.1 || exit 1
done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3v/ab.txt
