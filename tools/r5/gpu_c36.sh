#!/bin/bash
# Llama-2-7B LoRA SFT preset: one steady step's kernel summary at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c36; mkdir -p $O
bash tools/profile_bench.sh r5c36 --task sft --steps 3 --warmup 2 > /dev/null 2>&1 || { tail -20 gpurun_out/prof_r5c36/bench.log; exit 1; }
f=$(find gpurun_out/prof_r5c36 -name "*kernel_trace.csv" | head -1)
python tools/trace_step_summary.py $f 40 > $O/sft_step_summary.txt && cut -c1-170 $O/sft_step_summary.txt
rm -f $f
