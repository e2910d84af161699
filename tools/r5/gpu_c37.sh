#!/bin/bash
# dK/dV D = 128 without dropout: K in registers, two blocks (waves) per CU/SIMD. Tests, Llama-3 step profile, presets.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c37; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_models_gpu.py tests/test_llama_ops_gpu.py tests/test_parity_full_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --task llama3 --steps 8 --warmup 3 > $O/llama3.json 2> $O/llama3.err || { tail -20 $O/llama3.err; exit 1; }
cut -c1-200 $O/llama3.json
timeout -k 10 400 python -u bench.py --task sft --steps 6 --warmup 2 > $O/sft.json 2> $O/sft.err || { tail -20 $O/sft.err; exit 1; }
cut -c1-200 $O/sft.json
bash tools/profile_bench.sh r5c37 --task llama3 --steps 3 --warmup 2 > /dev/null 2>&1 || { tail -20 gpurun_out/prof_r5c37/bench.log; exit 1; }
f=$(find gpurun_out/prof_r5c37 -name "*kernel_trace.csv" | head -1)
python tools/trace_step_summary.py $f 14 > $O/llama3_step_summary.txt && cut -c1-150 $O/llama3_step_summary.txt
rm -f $f
