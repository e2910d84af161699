# r6 call 2: attention backward diet A/B (GPT-2 and Llama D=128 shapes), then HEAD validation
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_attention.sh gpurun_out/r6c2/attn64 3 base=variants/_dlion_C_base.so new=default || exit 1
bash tools/ab_attention.sh gpurun_out/r6c2/attn128 2 base=variants/_dlion_C_base.so new=default -- 1 8192 32 128 0.0 || exit 1
bash tools/gpu_validate.sh r6c2
