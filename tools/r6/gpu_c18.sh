# r6 call 18: 50-step learning curves at HEAD on the learnable Markov corpus, native engine vs the
# reference algorithm (--impl reference: HF GPT2LMHeadModel + per-tensor int64 all-gather Lion),
# same initial weights; W = 1 (RCCL-free) and W = 2 (two gloo ranks sharing the GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c18; mkdir -p $O
for impl in native reference; do
  timeout -k 10 300 python3 bench.py --data markov --steps 50 --warmup 0 --loss_log $O/curve_${impl}_w1.jsonl \
    --impl $impl > $O/${impl}_w1.log 2>&1 || { tail -20 $O/${impl}_w1.log; exit 1; }
  timeout -k 10 400 python3 bench.py --gpus 2 --backend gloo --data markov --steps 50 --warmup 0 \
    --loss_log $O/curve_${impl}_w2.jsonl --impl $impl > $O/${impl}_w2.log 2>&1 || { tail -20 $O/${impl}_w2.log; exit 1; }
done
python3 tools/curve_summary.py native_w1=$O/curve_native_w1.jsonl reference_w1=$O/curve_reference_w1.jsonl \
  native_w2=$O/curve_native_w2.jsonl reference_w2=$O/curve_reference_w2.jsonl | tee $O/summary.txt
