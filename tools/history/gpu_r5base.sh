# round-5 first GPU call: ping-pong attention A/B, full GPU suite, bench (default and pp), rocprof summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5base; mkdir -p $O
bash tools/r5/gpu_attn_pp.sh 3 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/gpu_tests.log | head -20; exit 1; }
for v in 0 3; do
  DLION_ATTN_PP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_pp$v.json 2> $O/bench_pp$v.err || { tail -20 $O/bench_pp$v.err; exit 1; }
  echo "pp=$v $(tail -1 $O/bench_pp$v.json | cut -c1-200)"
done
bash tools/profile_bench.sh r5base --steps 8 --warmup 2 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/prof_r5base -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 80 30 steady > $O/summary.txt; head -20 $O/summary.txt | cut -c1-150
