#!/bin/bash
# Transpose kernel A/B (transposed-read path vs per-element LDS path), interleaved, same box.
set -o pipefail
O=gpurun_out/r5c29; mkdir -p $O
timeout -k 10 200 python -u tools/r5/bench_transpose.py > $O/transpose.jsonl 2> $O/transpose.err || { tail -20 $O/transpose.err; exit 1; }
cat $O/transpose.jsonl
