set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3e
timeout -k 10 400 python tools/diag_llama_bf16.py > gpurun_out/r3e/diag.log 2>&1; grep -v "Writing\|Loading\|amdgpu.ids" gpurun_out/r3e/diag.log | tail -20
