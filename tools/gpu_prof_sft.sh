set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 280 --timeout-method thread -k bench_contract > gpurun_out/bench_contract.log 2>&1 || { tail -30 gpurun_out/bench_contract.log; exit 1; }
tail -2 gpurun_out/bench_contract.log
bash tools/profile_bench.sh sft --task sft > /dev/null 2>&1 || exit 1
bash tools/profile_bench.sh sft4 --task sft --load_in_4bit > /dev/null 2>&1 || exit 1
for t in sft sft4; do f=$(find gpurun_out/prof_$t -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 6 40 > gpurun_out/prof_$t/summary.txt; head -25 gpurun_out/prof_$t/summary.txt | cut -c1-160; done
