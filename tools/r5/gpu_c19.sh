#!/bin/bash
# (1) Qwen2 / Mistral step throughput after the deferred-operand guard fix;
# (2) hipBLASLt NN input gradient: numerics, Llama-3-8B shape timings, preset A/B.
set -o pipefail
O=gpurun_out/r5c19; mkdir -p $O
timeout -k 10 300 python -u bench.py --task clm --model qwen2-0.5b --micro_batch 16 --steps 10 --warmup 3 > $O/qwen2.json 2> $O/qwen2.err || { tail -20 $O/qwen2.err; exit 1; }
cut -c1-400 $O/qwen2.json
timeout -k 10 400 python -u bench.py --task llama3 --model mistral-7b --steps 6 --warmup 2 > $O/mistral.json 2> $O/mistral.err || { tail -20 $O/mistral.err; exit 1; }
cut -c1-400 $O/mistral.json
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_lt_gemm_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
MODEL=llama3 TOKENS=8192 timeout -k 10 300 python -u tools/bench_gemm_llama.py > $O/shapes.jsonl 2> $O/shapes.err || { tail -20 $O/shapes.err; exit 1; }
cat $O/shapes.jsonl
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --task llama3 --steps 8 --warmup 3 > $O/llama3_lt_$r.json 2> $O/llama3_lt_$r.err || { tail -20 $O/llama3_lt_$r.err; exit 1; }
  cut -c1-200 $O/llama3_lt_$r.json
  DLION_LT_NN=0 timeout -k 10 400 python -u bench.py --task llama3 --steps 8 --warmup 3 > $O/llama3_base_$r.json 2> $O/llama3_base_$r.err || { tail -20 $O/llama3_base_$r.err; exit 1; }
  cut -c1-200 $O/llama3_base_$r.json
done
