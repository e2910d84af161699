# HEAD check on one MI355X: full GPU suite, GPT-2 rocprof summary, 8-rank gloo rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_tests.log | head -20; exit 1; }
bash tools/profile_bench.sh gpt2 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/prof_gpt2 -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 24 30 > gpurun_out/prof_gpt2/summary.txt; head -16 gpurun_out/prof_gpt2/summary.txt | cut -c1-150
tail -1 gpurun_out/prof_gpt2/bench.log | cut -c1-200
bash tools/gpu_w8_gloo.sh
