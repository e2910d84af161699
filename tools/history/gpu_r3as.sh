# Embedding-backward id sort moved into the forward on a side stream (default) vs in the backward; embedding / model tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3as
timeout -k 10 500 python -u -m pytest tests/test_embedding_gpu.py tests/test_models_gpu.py tests/test_grad_fusion_gpu.py tests/test_parity_full_gpu.py -q -x --timeout 240 --timeout-method thread > gpurun_out/r3as/tests.log 2>&1 || { tail -40 gpurun_out/r3as/tests.log; exit 1; }
tail -1 gpurun_out/r3as/tests.log
for v in 1 0 1 0 1 0; do
  DLION_EMBED_SORT_AHEAD=$v timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3as/bench_$v.json 2> gpurun_out/r3as/bench_$v.err || { tail -20 gpurun_out/r3as/bench_$v.err; exit 1; }
  echo "sort_ahead=$v $(python -c "import json;d=json.load(open('gpurun_out/r3as/bench_$v.json'));print(d['value'],d['ms_per_step'],d['loss'])")"
done | tee gpurun_out/r3as/bench_ab.txt
