set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python -m pytest tests -m gpu -q > gpurun_out/gpu_tests.log 2>&1; echo "tests rc=$?"; tail -8 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_native.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench_native.log; exit 1; }
tail -2 gpurun_out/bench_native.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --impl reference > gpurun_out/bench_ref.log 2>&1 || { echo REFBENCH FAIL; tail -30 gpurun_out/bench_ref.log; exit 1; }
tail -2 gpurun_out/bench_ref.log
