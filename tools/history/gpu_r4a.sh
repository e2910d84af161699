# Round-4 start on one MI355X: full GPU suite, driver smoke, driver-form bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4a/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4a/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r4a/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a/smoke.log 2>&1 || { tail -20 gpurun_out/r4a/smoke.log; exit 1; }
tail -2 gpurun_out/r4a/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4a/bench.json 2> gpurun_out/r4a/bench.err || { tail -20 gpurun_out/r4a/bench.err; exit 1; }
cut -c1-400 gpurun_out/r4a/bench.json
