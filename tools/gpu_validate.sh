# HEAD validation on one MI355X: full GPU suite, smoke, driver-form bench,
# GPT-2 steady rocprof summary.  Usage: bash tools/gpu_validate.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-head}
O=gpurun_out/$TAG; mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
  tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/gpu_tests.log | head -30; exit 1; }
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
bash tools/profile_bench.sh $TAG --steps 8 --warmup 2 > /dev/null 2>&1 || { tail -20 gpurun_out/prof_$TAG/bench.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 80 30 steady > $O/gpt2_summary_steady.txt; head -14 $O/gpt2_summary_steady.txt | cut -c1-150
