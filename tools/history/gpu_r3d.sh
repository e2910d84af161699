set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
timeout -k 10 400 python tools/diag_llama_parity.py > gpurun_out/r3d/diag.log 2>&1; grep "^L=" gpurun_out/r3d/diag.log || tail -20 gpurun_out/r3d/diag.log
