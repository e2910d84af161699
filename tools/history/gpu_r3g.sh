set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3g
timeout -k 10 300 python tools/diag_llama_ops.py > gpurun_out/r3g/diag.log 2>&1; grep "^hidden" gpurun_out/r3g/diag.log || tail -20 gpurun_out/r3g/diag.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3g/tests.log 2>&1; tail -3 gpurun_out/r3g/tests.log
