# smoke + GPU tests + GPT-2 bench + rocprofv3 kernel stats on one MI355X.
# Usage (via gpurun): bash tools/gpu_full.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAIL; tail -20 $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || { echo BENCH FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python3 bench.py --steps 2 --warmup 1 > $OUT/prof_bench.log 2>&1 || { echo PROF FAIL; tail -20 $OUT/prof_bench.log; exit 1; }
echo prof ok
