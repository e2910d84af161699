#!/bin/bash
# Llama-3-8B preset: one steady step's kernel summary at HEAD (after the NN / TN picks).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c25; mkdir -p $O
bash tools/profile_bench.sh r5c25 --task llama3 --steps 3 --warmup 2 > /dev/null 2>&1 || { tail -20 gpurun_out/prof_r5c25/bench.log; exit 1; }
f=$(find gpurun_out/prof_r5c25 -name "*kernel_trace.csv" | head -1)
python tools/trace_step_summary.py $f 30 > $O/llama3_step_summary.txt && cut -c1-170 $O/llama3_step_summary.txt
rm -f $f
