# what the driver runs at round end: GPU suite, smoke, default bench (driver's K/W)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_tests.log | head; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-200 || exit 1
