# Every BASELINE preset of bench.py on one GPU (+ QLoRA and the HF run_clm path), one JSON line each,
# into gpurun_out/presets.jsonl.  usage: bash tools/gpu_presets.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/presets.jsonl
: > $OUT
run() { timeout -k 10 600 python bench.py "$@" 2>gpurun_out/preset_err.log | tail -1 >> $OUT || { tail -20 gpurun_out/preset_err.log; exit 1; }; }
run --steps 8 --warmup 2
run --impl reference --steps 3 --warmup 1
run --task sft --steps 4 --warmup 2
run --task sft --load_in_4bit --steps 4 --warmup 2
run --task dpo --steps 3 --warmup 1
run --task dpo --checkpointing_policy reference --steps 3 --warmup 1
run --task llama3 --steps 4 --warmup 2
STEPS=12 bash tools/gpu_runclm.sh presets --logging_steps 5 || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/presets.jsonl"):
    d = json.loads(l)
    c = d["config"]
    print(f'{c["task"]:6s} {c.get("impl",""):9s} {c.get("base_weights",""):20s} ckpt={c.get("gradient_checkpointing")} {d["value"]:>12,.1f} tok/s  {d["ms_per_step"]} ms/step')
PY
