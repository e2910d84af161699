set -o pipefail
cd $GRAFT_REPO_ROOT
STEPS=16 bash tools/gpu_runclm.sh log5 --logging_steps 5 || exit 1
timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_same.log 2>&1 || exit 1
tail -1 gpurun_out/bench_same.log | cut -c1-150
bash tools/gpu_trace_runclm.sh 2>&1 | head -60
