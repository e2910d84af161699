# run_clm (HF Trainer + AsyncTrainer + Lion) with the reference README's GPT-2 config, synthetic data.
# usage: bash tools/gpu_runclm.sh <tag> [extra run_clm args]; env STEPS (default 12)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-default}; shift
mkdir -p gpurun_out/runclm_$TAG
OUT=/tmp/runclm_$TAG
rm -rf $OUT
timeout -k 10 500 python -u run_clm.py --config_name gpt2 --synthetic_data --synthetic_samples 4000 \
  --per_device_train_batch_size 20 --do_train --output_dir $OUT --report_to none \
  --torch_dtype bfloat16 --gradient_accumulation_steps 8 --max_steps ${STEPS:-12} --warmup_steps 2 --lion \
  --learning_rate 1e-4 --weight_decay 0.1 --async_grad --logging_steps 1 --save_strategy no "$@" \
  > gpurun_out/runclm_$TAG/log.txt 2>&1 || { tail -30 gpurun_out/runclm_$TAG/log.txt; exit 1; }
cp $OUT/metrics.jsonl gpurun_out/runclm_$TAG/
python - "$TAG" <<'PY'
import json, sys
tag = sys.argv[1]
recs = [json.loads(l) for l in open(f"gpurun_out/runclm_{tag}/metrics.jsonl")]
tps = [r["tokens_per_s"] for r in recs if "tokens_per_s" in r]
tail = sorted(tps[len(tps) // 2:])
print(tag, "tokens/s per step:", [round(t) for t in tps])
print(tag, "median of last half:", round(tail[len(tail) // 2]), "loss:", [round(r["loss"], 3) for r in recs if "loss" in r][-3:])
PY
