#!/bin/bash
# Mistral / Qwen2 native families on the GPU: HF parity tests + step throughput.
set -o pipefail
O=gpurun_out/r5c17; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench.py --task clm --model qwen2-0.5b --micro_batch 16 --steps 10 --warmup 3 > $O/qwen2.json 2> $O/qwen2.err || { tail -20 $O/qwen2.err; exit 1; }
cat $O/qwen2.json
timeout -k 10 400 python -u bench.py --task llama3 --model mistral-7b --steps 6 --warmup 2 > $O/mistral.json 2> $O/mistral.err || { tail -20 $O/mistral.err; exit 1; }
cat $O/mistral.json
