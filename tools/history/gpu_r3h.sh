# Llama attention stage diag, kernel/attention tests, Lion roofline, attention SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
timeout -k 10 300 python tools/diag_llama_ops.py > gpurun_out/r3h/diag.log 2>&1; grep "^hidden" gpurun_out/r3h/diag.log || tail -20 gpurun_out/r3h/diag.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_gpu.py tests/test_grad_fusion_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3h/tests.log 2>&1 || { tail -30 gpurun_out/r3h/tests.log; exit 1; }
tail -2 gpurun_out/r3h/tests.log
timeout -k 10 200 python tools/bench_lion.py gpt2 8 > gpurun_out/r3h/lion_gpt2.txt 2>&1 && timeout -k 10 300 python tools/bench_lion.py llama3 8 > gpurun_out/r3h/lion_llama3.txt 2>&1 || exit 1
cat gpurun_out/r3h/lion_gpt2.txt gpurun_out/r3h/lion_llama3.txt
bash tools/pmc_attn_sq.sh 20 1024 12 64 0.1 > gpurun_out/r3h/pmc.txt 2>&1; tail -45 gpurun_out/r3h/pmc.txt
