# Attention occupancy A/B: default build (dKV D64 3 waves, dKV D128 2 waves, dQ D64 4 waves)
# vs variants without the hints; attention numerics on the default build first.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3l
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3l/attn_tests.log 2>&1 || { tail -30 gpurun_out/r3l/attn_tests.log; exit 1; }
tail -2 gpurun_out/r3l/attn_tests.log
for rep in 1 2; do
for v in default noocc dq1 dkv128_1; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  for shape in "20 1024 12 64 0.1" "4 2048 32 128 0.0"; do
    echo "== $v $shape"
    DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py $shape || exit 1
  done
done
done 2>&1 | tee gpurun_out/r3l/ab.txt
