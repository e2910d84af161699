# LM-head weight gradient deferred into the fusion window's TN GEMM (DLION_LM_DEFER=1, default) vs per micro-batch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3aj
timeout -k 10 500 python -u -m pytest tests/test_grad_fusion_gpu.py tests/test_models_gpu.py tests/test_parity_full_gpu.py tests/test_xent_gpu.py -q -x --timeout 240 --timeout-method thread > gpurun_out/r3aj/tests.log 2>&1 || { tail -40 gpurun_out/r3aj/tests.log; exit 1; }
tail -1 gpurun_out/r3aj/tests.log
for v in 1 0 1 0; do
  DLION_LM_DEFER=$v timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3aj/bench_$v.json 2> gpurun_out/r3aj/bench_$v.err || { tail -20 gpurun_out/r3aj/bench_$v.err; exit 1; }
  echo "lm_defer=$v $(python -c "import json;d=json.load(open('gpurun_out/r3aj/bench_$v.json'));print(d['value'],d['ms_per_step'],d['loss'])")"
done | tee gpurun_out/r3aj/bench_ab.txt
