# round-5 baseline on one MI355X: full GPU suite, GPT-2 rocprof summary, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5base; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/gpu_tests.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || exit 1
tail -1 $O/bench.json | cut -c1-300
bash tools/profile_bench.sh r5base --steps 8 --warmup 2 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/prof_r5base -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 80 30 steady > $O/summary.txt; head -20 $O/summary.txt | cut -c1-150
