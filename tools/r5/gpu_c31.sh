#!/bin/bash
# One-copy weight gradients (hipBLASLt NN with a^T / TT with b^T): tests, shapes, Llama-3 preset A/B.
set -o pipefail
O=gpurun_out/r5c31; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lt_gemm_gpu.py tests/test_gemm_tn_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/r5/bench_wgrad_lt.py > $O/wgrad.jsonl 2> $O/wgrad.err || { tail -20 $O/wgrad.err; exit 1; }
cat $O/wgrad.jsonl
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --task llama3 --steps 8 --warmup 3 > $O/llama3_new_$r.json 2> $O/llama3_new_$r.err || { tail -20 $O/llama3_new_$r.err; exit 1; }
  cut -c1-200 $O/llama3_new_$r.json
done
