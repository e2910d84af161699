# round-5 GPU call 15: run_clm on a local text file, map-style vs --streaming (GPT-2 bench config, byte tokenizer)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c15; mkdir -p $O
python3 - <<'PY'
import random
random.seed(0)
words = ["".join(random.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(random.randint(2, 9))) for _ in range(5000)]
with open("/tmp/corpus.txt", "w") as f:
    for i in range(400000):
        f.write(" ".join(random.choice(words) for _ in range(12)) + "\n")
PY
for mode in map stream; do
  extra=""; [ $mode = stream ] && extra="--streaming"
  rm -rf /tmp/clm_$mode
  timeout -k 10 500 python -u run_clm.py --config_name gpt2 --train_file /tmp/corpus.txt $extra \
    --per_device_train_batch_size 20 --block_size 1024 --do_train --output_dir /tmp/clm_$mode --report_to none \
    --torch_dtype bfloat16 --gradient_accumulation_steps 8 --max_steps 12 --warmup_steps 2 --lion \
    --learning_rate 1e-4 --weight_decay 0.1 --async_grad --logging_steps 1 --save_strategy no \
    > $O/log_$mode.txt 2>&1 || { tail -30 $O/log_$mode.txt; exit 1; }
  cp /tmp/clm_$mode/metrics.jsonl $O/metrics_$mode.jsonl
  python3 - $mode <<'PY'
import json, sys
m = sys.argv[1]
recs = [json.loads(l) for l in open(f"gpurun_out/r5c15/metrics_{m}.jsonl")]
tps = [r["tokens_per_s"] for r in recs if "tokens_per_s" in r]
tail = sorted(tps[len(tps) // 2:])
loss = [round(r["loss"], 3) for r in recs if "loss" in r]
print(m, "tok/s per step:", [round(t) for t in tps], "median of the last half:", tail[len(tail) // 2] if tail else None,
      "loss", loss[:2], "->", loss[-2:])
PY
done
