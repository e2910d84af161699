set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_hf_sft_dpo.sh
