# round-5 GPU call 9: concurrent attention backward (delta pre-pass, dQ || dK/dV): tests, kernel A/B, GPT-2 bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c9; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
PYTHONPATH=. timeout -k 10 300 python tools/r5/bench_attn_conc.py > $O/bench_attn_conc.txt 2>&1 || { tail -20 $O/bench_attn_conc.txt; exit 1; }
grep -v amdgpu.ids $O/bench_attn_conc.txt
for i in 1 2; do
  for c in 1 0; do
    DLION_ATTN_BWD_CONCURRENT=$c timeout -k 10 300 python bench.py --steps 12 --warmup 3 > $O/gpt2_c$c.$i.json 2> $O/gpt2_c$c.$i.err || { tail -20 $O/gpt2_c$c.$i.err; exit 1; }
    echo "concurrent=$c $(tail -1 $O/gpt2_c$c.$i.json | cut -c1-160)"
  done
done
