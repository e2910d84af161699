#!/bin/bash
# r6 call 1: on-box GEMM anchor + HEAD bench
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python3 -u tools/gemm_anchor.py > gpurun_out/r6/gemm_anchor.txt 2>&1 && \
timeout -k 10 180 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6/bench_head.json 2> gpurun_out/r6/bench_head.err
