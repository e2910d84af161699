# rocprofv3 kernel summary of the Llama-3-8B full-parameter preset (3 steps of 1 micro-batch, incl. init)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_bench.sh llama3 --task llama3 > /dev/null 2>&1 || { tail -20 gpurun_out/prof_llama3/bench.log; exit 1; }
f=$(find gpurun_out/prof_llama3 -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 3 40 > gpurun_out/prof_llama3/summary.txt; head -40 gpurun_out/prof_llama3/summary.txt | cut -c1-170
tail -1 gpurun_out/prof_llama3/bench.log | cut -c1-300
