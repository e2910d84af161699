#!/bin/bash
# Transpose kernel with b128 LDS stores + hardware-transposed reads: tests, throughput, Llama-3 preset.
set -o pipefail
O=gpurun_out/r5c28; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "transpose" tests/test_gemm_tn_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u tools/r5/bench_transpose.py > $O/transpose.jsonl 2> $O/transpose.err || { tail -20 $O/transpose.err; exit 1; }
cat $O/transpose.jsonl
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --task llama3 --steps 8 --warmup 3 > $O/llama3_$r.json 2> $O/llama3_$r.err || { tail -20 $O/llama3_$r.err; exit 1; }
  cut -c1-200 $O/llama3_$r.json
done
