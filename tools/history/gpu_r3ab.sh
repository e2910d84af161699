# Robust GEMM candidate timing (interleaved rounds): GEMM/lt tests + 4 fresh bench processes (run-to-run spread)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ab
timeout -k 10 300 python -u -m pytest tests/test_lt_gemm_gpu.py tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3ab/tests.log 2>&1 || { tail -30 gpurun_out/r3ab/tests.log; exit 1; }
tail -1 gpurun_out/r3ab/tests.log
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ab/bench_$i.json 2> gpurun_out/r3ab/bench_$i.err || { tail -20 gpurun_out/r3ab/bench_$i.err; exit 1; }
  echo "run$i $(python -c "import json;d=json.load(open('gpurun_out/r3ab/bench_$i.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3ab/bench_runs.txt
