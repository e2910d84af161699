# BASELINE configs on one MI355X: reference algorithm A/B, Llama-2-7B LoRA SFT / DPO, Llama-3-8B full-param
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/presets
out=gpurun_out/presets/presets.jsonl
: > $out
timeout -k 10 300 python bench.py --impl reference --steps 3 --warmup 1 2>/dev/null | tail -1 >> $out || exit 1
for t in sft dpo llama3; do
  timeout -k 10 400 python bench.py --task $t --steps 4 --warmup 2 2>/dev/null | tail -1 >> $out || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/presets/presets.jsonl"):
    d = json.loads(l)
    print(f"{d['config']['task']:7s} {d['config']['impl']:9s} {d['config']['model']:28s} {d['value']:>12,.1f} tok/s  {d['ms_per_step']:9.1f} ms/step")
PY
