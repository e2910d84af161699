# HEAD check: full GPU suite, then every preset (GPT-2 native / reference, Llama-2-7B SFT / QLoRA / DPO, Llama-3-8B, run_clm)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ac
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r3ac/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3ac/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3ac/gpu_tests.log
bash tools/gpu_presets.sh 2>&1 | tail -12 | tee gpurun_out/r3ac/presets.txt
cp gpurun_out/presets.jsonl gpurun_out/r3ac/presets.jsonl
