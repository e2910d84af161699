# Llama parity diagnostic + Lion kernel fast paths (tests + roofline bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 300 python tools/diag_llama_parity.py > gpurun_out/r3c/diag.log 2>&1; cat gpurun_out/r3c/diag.log | grep "layers="
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_multirank_gpu.py tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3c/tests.log 2>&1 || { tail -30 gpurun_out/r3c/tests.log; exit 1; }
tail -2 gpurun_out/r3c/tests.log
timeout -k 10 200 python tools/bench_lion.py gpt2 8 > gpurun_out/r3c/lion_gpt2.txt 2>&1 && timeout -k 10 300 python tools/bench_lion.py llama3 8 > gpurun_out/r3c/lion_llama3.txt 2>&1
cat gpurun_out/r3c/lion_gpt2.txt gpurun_out/r3c/lion_llama3.txt
