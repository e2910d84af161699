# attention tests + per-kernel times at HEAD, then the HF-path SFT / DPO timing (tools/gpu_hf_sft_dpo.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4d
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4d/tests.log 2>&1 || { tail -40 gpurun_out/r4d/tests.log; exit 1; }
tail -1 gpurun_out/r4d/tests.log
bash tools/gpu_attn_p.sh head=default:0.1 || exit 1
bash tools/gpu_hf_sft_dpo.sh
