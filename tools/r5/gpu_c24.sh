#!/bin/bash
# Sliding-window attention cost at Mistral-7B shapes, and the Mistral-7B step at 8192 tokens (window 4096 active).
set -o pipefail
O=gpurun_out/r5c24; mkdir -p $O
timeout -k 10 300 python -u tools/r5/bench_window.py > $O/window.jsonl 2> $O/window.err || { tail -20 $O/window.err; exit 1; }
cat $O/window.jsonl
timeout -k 10 400 python -u bench.py --task llama3 --model mistral-7b --micro_batch 1 --seq_len 8192 --steps 6 --warmup 2 > $O/mistral8k.json 2> $O/mistral8k.err || { tail -20 $O/mistral8k.err; exit 1; }
cut -c1-300 $O/mistral8k.json
