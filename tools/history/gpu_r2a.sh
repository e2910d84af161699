set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_grad_fusion_gpu.py > gpurun_out/fusion_tests.log 2>&1 || { echo FUSION FAIL; tail -40 gpurun_out/fusion_tests.log; exit 1; }
tail -3 gpurun_out/fusion_tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo GPUTESTS FAIL; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
