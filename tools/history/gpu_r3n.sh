# Dropout keep bits recorded by the forward, read by the backward: attention numerics + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3n
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3n/attn_tests.log 2>&1 || { tail -40 gpurun_out/r3n/attn_tests.log; exit 1; }
tail -2 gpurun_out/r3n/attn_tests.log
for rep in 1 2; do
  for shape in "20 1024 12 64 0.1" "20 1024 12 64 0.0" "4 2048 32 128 0.0"; do
    echo "== $shape"
    DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py $shape || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3n/bench_attn.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/r3n/bench.json 2> gpurun_out/r3n/bench.err || { tail -20 gpurun_out/r3n/bench.err; exit 1; }
cut -c1-400 gpurun_out/r3n/bench.json
