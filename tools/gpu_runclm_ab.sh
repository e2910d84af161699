# run_clm A/B: batch prefetch on/off, SDMA copies on/off (same box, back to back)
set -o pipefail
cd $GRAFT_REPO_ROOT
DLION_HF_PREFETCH=0 STEPS=16 bash tools/gpu_runclm.sh noprefetch --logging_steps 5 | grep median || exit 1
STEPS=16 bash tools/gpu_runclm.sh prefetch --logging_steps 5 | grep median || exit 1
HSA_ENABLE_SDMA=0 DLION_HF_PREFETCH=0 STEPS=16 bash tools/gpu_runclm.sh nosdma --logging_steps 5 | grep median || exit 1
DLION_HF_PREFETCH=0 STEPS=16 bash tools/gpu_runclm.sh noprefetch2 --logging_steps 5 | grep median || exit 1
STEPS=16 bash tools/gpu_runclm.sh prefetch2 --logging_steps 5 | grep median || exit 1
