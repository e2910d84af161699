#!/bin/bash
# SwiGLU forward + backward writing h^T, dgu^T for the transposed-copy gate/up weight gradient: tests + Llama-3 preset A/B.
set -o pipefail
O=gpurun_out/r5c34; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_llama_ops_gpu.py tests/test_gemm_tn_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --task llama3 --steps 8 --warmup 3 > $O/llama3_prod_$r.json 2> $O/llama3_prod_$r.err || { tail -20 $O/llama3_prod_$r.err; exit 1; }
  cut -c1-200 $O/llama3_prod_$r.json
  DLION_TT_PRODUCER=0 timeout -k 10 400 python -u bench.py --task llama3 --steps 8 --warmup 3 > $O/llama3_base_$r.json 2> $O/llama3_base_$r.err || { tail -20 $O/llama3_base_$r.err; exit 1; }
  cut -c1-200 $O/llama3_base_$r.json
done
