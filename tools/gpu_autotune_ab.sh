# per-shape GEMM autotune: tests + same-box A/B on the Llama presets (SFT, Llama-3) and GPT-2 sanity
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gemm_tn_gpu.py tests/test_lora_gpu.py tests/test_llama_ops_gpu.py tests/test_quant_gpu.py tests/test_models_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/at_tests.log 2>&1; rc=$?; tail -2 gpurun_out/at_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/at_tests.log | head; exit 1; }
bash tools/ab_bench.sh "DLION_GEMM_AUTOTUNE=0" "" 1 --task sft --steps 4 --warmup 2 || exit 1
bash tools/ab_bench.sh "DLION_GEMM_AUTOTUNE=0" "" 1 --task llama3 --steps 3 --warmup 2 || exit 1
bash tools/ab_bench.sh "DLION_GEMM_AUTOTUNE=0" "" 1 --task sft --steps 4 --warmup 2 || exit 1
