# HEAD profile: rocprof kernel stats of the GPT-2 bench (7 steps = 56 micro-batches) + driver-form bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3al
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3al/bench.json 2> gpurun_out/r3al/bench.err || { tail -20 gpurun_out/r3al/bench.err; exit 1; }
cut -c1-300 gpurun_out/r3al/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3al/prof -o prof -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r3al/prof_bench.log 2>&1 || { tail -20 gpurun_out/r3al/prof_bench.log; exit 1; }
f=$(find gpurun_out/r3al/prof -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 56 40 > gpurun_out/r3al/gpt2_summary.txt; head -22 gpurun_out/r3al/gpt2_summary.txt | cut -c1-150
