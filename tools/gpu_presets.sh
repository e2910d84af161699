# Every BASELINE preset of bench.py on one GPU (+ the HF run_clm path), one JSON line each,
# into gpurun_out/presets.jsonl.  usage: bash tools/gpu_presets.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/presets.jsonl
: > $OUT
run() { timeout -k 10 600 python bench.py "$@" 2>gpurun_out/preset_err.log | tail -1 >> $OUT || { tail -20 gpurun_out/preset_err.log; exit 1; }; }
run --steps 8 --warmup 2
run --impl reference --steps 3 --warmup 1
run --task sft --steps 4 --warmup 2
run --task dpo --steps 3 --warmup 1
run --task llama3 --steps 4 --warmup 2
STEPS=12 bash tools/gpu_runclm.sh presets --logging_steps 5 || exit 1
