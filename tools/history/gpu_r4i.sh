# round-end rehearsal at HEAD: the driver's GPU suite, smoke and default bench, then a
# rocprofv3 kernel-trace of bench.py (8 steps) summarised per micro-batch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/gpu_tests.log | head; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null | tail -1 > $O/bench.json || exit 1
cut -c1-400 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o prof -- python3 bench.py --steps 8 --warmup 2 > $O/prof_bench.log 2>&1 || { tail -5 $O/prof_bench.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 tools/prof_summary.py $f 80 30 steady > $O/summary_steady.txt && cat $O/summary_steady.txt
