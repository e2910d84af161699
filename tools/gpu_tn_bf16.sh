# unsplit bf16 wgrad output: TN tests + Llama-3-8B full-parameter bench (+ GPT-2 sanity)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_tn_gpu.py tests/test_grad_fusion_gpu.py tests/test_llama_ops_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/tn_tests.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/tn_tests.log | head -30; tail -30 gpurun_out/tn_tests.log; exit 1; }
tail -2 gpurun_out/tn_tests.log
timeout -k 10 400 python bench.py --task llama3 --steps 4 --warmup 2 > gpurun_out/bench_l3.log 2>&1 || { tail -30 gpurun_out/bench_l3.log; exit 1; }
tail -1 gpurun_out/bench_l3.log | cut -c1-260
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/bench_gpt2.log 2>&1 || { tail -30 gpurun_out/bench_gpt2.log; exit 1; }
tail -1 gpurun_out/bench_gpt2.log | cut -c1-200
