# Round-3 first GPU check: new RCCL audit tests, full GPU suite, bench at HEAD (phase breakdown)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3a
timeout -k 10 300 python -u -m pytest tests/test_nccl_gpu.py -x -v --timeout 160 --timeout-method thread > gpurun_out/r3a/nccl.log 2>&1 || { tail -60 gpurun_out/r3a/nccl.log; exit 1; }
tail -3 gpurun_out/r3a/nccl.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r3a/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3a/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3a/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err || { tail -20 gpurun_out/r3a/bench.err; exit 1; }
cat gpurun_out/r3a/bench.json | cut -c1-3000
