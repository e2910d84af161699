# HF-path SFT and DPO entrypoints (AsyncSFTTrainer / AsyncDPOTrainer + Lion) on one MI355X next to
# the native-loop bench presets of the same configs.  Reference configs: README.md:40-72 (SFT),
# dpo_llama2.py defaults (DPO).  Synthetic data, random-init Llama-2-7B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/hf_sft_dpo; mkdir -p $OUT
rm -rf /tmp/hf_sft /tmp/hf_dpo
timeout -k 10 600 python -u sft_llama2.py --model_name llama-2-7b --output_dir /tmp/hf_sft --max_steps 12 \
  --logging_steps 1 --save_strategy no --per_device_train_batch_size 4 --per_device_eval_batch_size 1 \
  --gradient_accumulation_steps 2 --gradient_checkpointing False --learning_rate 1e-4 \
  --lr_scheduler_type cosine --warmup_steps 2 --weight_decay 0.05 --bf16 True --remove_unused_columns False \
  --report_to none --lion --async_grad --final_save false --synthetic_data --synthetic_samples 4000 > $OUT/sft.log 2>&1 || { tail -30 $OUT/sft.log; exit 1; }
cp /tmp/hf_sft/metrics.jsonl $OUT/sft_metrics.jsonl
timeout -k 10 600 python -u dpo_llama2.py --model_name_or_path llama-2-7b --output_dir /tmp/hf_dpo --max_steps 8 \
  --logging_steps 1 --eval_steps 0 --warmup_steps 2 --lion --async_grad --final_save false \
  --synthetic_data --synthetic_samples 400 --synthetic_chars 1000 > $OUT/dpo.log 2>&1 || { tail -30 $OUT/dpo.log; exit 1; }
cp /tmp/hf_dpo/metrics.jsonl $OUT/dpo_metrics.jsonl
timeout -k 10 600 python bench.py --task sft --steps 6 --warmup 2 2>/dev/null | tail -1 > $OUT/bench_sft.json || exit 1
timeout -k 10 600 python bench.py --task dpo --steps 4 --warmup 1 2>/dev/null | tail -1 > $OUT/bench_dpo.json || exit 1
python - <<'PY'
import json
o = "gpurun_out/hf_sft_dpo"
for name in ("sft", "dpo"):
    recs = [json.loads(l) for l in open(f"{o}/{name}_metrics.jsonl")]
    tps = [r["tokens_per_s"] for r in recs if "tokens_per_s" in r]
    tail = sorted(tps[len(tps) // 2:])
    b = json.loads(open(f"{o}/bench_{name}.json").read())
    med = tail[len(tail) // 2]
    print(f"{name}: HF path median(last half) {med:,.0f} tok/s  per step {[round(t) for t in tps]}  "
          f"bench {b['value']:,.0f} tok/s  ratio {med / b['value']:.3f}")
PY
