# Backward attention LDS ring depth A/B (2 = double buffering, 3 default, 4); numerics on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3o
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3o/attn_tests.log 2>&1 || { tail -40 gpurun_out/r3o/attn_tests.log; exit 1; }
tail -1 gpurun_out/r3o/attn_tests.log
for rep in 1 2; do
for v in st2 default st4; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  for shape in "20 1024 12 64 0.1" "4 2048 32 128 0.0"; do
    echo "== $v $shape"
    DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py $shape || exit 1
  done
done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3o/ab.txt
