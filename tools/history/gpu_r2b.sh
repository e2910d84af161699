set -o pipefail
cd $GRAFT_REPO_ROOT
DLION_HF_FUSION=0 bash tools/gpu_runclm.sh nofusion && bash tools/gpu_runclm.sh fusion
