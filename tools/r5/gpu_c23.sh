#!/bin/bash
# Sliding-window attention (D = 128): kernel tests vs fp32, Mistral model vs HF, attention + models suites.
set -o pipefail
O=gpurun_out/r5c23; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_models_gpu.py tests/test_llama_ops_gpu.py > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
