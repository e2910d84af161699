#!/bin/bash
# dK/dV D = 128 K-in-registers vs K-in-LDS, interleaved in one process; attention tests; SFT preset A/B.
set -o pipefail
O=gpurun_out/r5c38; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/r5/bench_dkv_kreg.py > $O/dkv.jsonl 2> $O/dkv.err || { tail -20 $O/dkv.err; exit 1; }
cat $O/dkv.jsonl
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --task sft --steps 6 --warmup 2 > $O/sft_kreg_$r.json 2> $O/sft_kreg_$r.err || { tail -20 $O/sft_kreg_$r.err; exit 1; }
  cut -c1-150 $O/sft_kreg_$r.json
  DLION_DKV_KREG128=0 timeout -k 10 300 python -u bench.py --task sft --steps 6 --warmup 2 > $O/sft_lds_$r.json 2> $O/sft_lds_$r.err || { tail -20 $O/sft_lds_$r.err; exit 1; }
  cut -c1-150 $O/sft_lds_$r.json
done
