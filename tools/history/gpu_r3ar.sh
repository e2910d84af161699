# HEAD check: full GPU suite, smoke, driver-form bench, rocprof summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ar
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r3ar/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3ar/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3ar/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3ar/smoke.log 2>&1 || { tail -20 gpurun_out/r3ar/smoke.log; exit 1; }
tail -1 gpurun_out/r3ar/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3ar/bench.json 2> gpurun_out/r3ar/bench.err || { tail -20 gpurun_out/r3ar/bench.err; exit 1; }
cut -c1-260 gpurun_out/r3ar/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3ar/prof -o prof -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r3ar/prof_bench.log 2>&1 || { tail -20 gpurun_out/r3ar/prof_bench.log; exit 1; }
f=$(find gpurun_out/r3ar/prof -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 56 40 > gpurun_out/r3ar/gpt2_summary.txt; head -14 gpurun_out/r3ar/gpt2_summary.txt | cut -c1-150
