# round-5 GPU call 12: inverse RoPE fused into the attention backward stores: tests + Llama-3-8B A/B + GPT-2 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c12; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_llama_ops_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for f in 1 0; do
    DLION_ROPE_BWD_FUSED=$f timeout -k 10 400 python bench.py --task llama3 --steps 4 --warmup 2 > $O/l3_f$f.$i.json 2> $O/l3_f$f.$i.err || { tail -20 $O/l3_f$f.$i.err; exit 1; }
    echo "rope_bwd_fused=$f $(tail -1 $O/l3_f$f.$i.json | cut -c120-260)"
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
