set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lt_gemm_gpu.py > gpurun_out/lt_tests.log 2>&1; rc=$?
tail -25 gpurun_out/lt_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 python -u tools/bench_lt_mlp.py > gpurun_out/lt_bench.log 2>&1; rc2=$?
cat gpurun_out/lt_bench.log | tail -20
exit $rc2
