# Session HEAD check: full GPU suite, driver-form bench, rocprof GPT-2 summary (7 steps = 56 micro-batches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3s
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r3s/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3s/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3s/gpu_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3s/bench.json 2> gpurun_out/r3s/bench.err || { tail -20 gpurun_out/r3s/bench.err; exit 1; }
cut -c1-400 gpurun_out/r3s/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3s/prof -o prof -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r3s/prof_bench.log 2>&1 || { tail -20 gpurun_out/r3s/prof_bench.log; exit 1; }
f=$(find gpurun_out/r3s/prof -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 56 45 > gpurun_out/r3s/gpt2_summary.txt; head -30 gpurun_out/r3s/gpt2_summary.txt | cut -c1-160
