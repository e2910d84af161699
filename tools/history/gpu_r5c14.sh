# round-5 GPU call 14: dQ attention kernel at 4 waves/SIMD (128 VGPRs, 3 dwords spilled outside the loop) vs 3:
# per-kernel rocprofv3 times at the GPT-2 shape, then the GPT-2 bench, 2 interleaved rounds each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c14; mkdir -p $O
DLION_LIB=$PWD/variants/_dlion_C_dq4.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in dq4 head; do
    lib=""; [ $v = dq4 ] && lib=$PWD/variants/_dlion_C_dq4.so
    DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v}_$i -o p -- python3 tools/bench_attention.py 20 1024 12 64 0.1 > $O/log_${v}_$i.txt 2>&1 || { tail -20 $O/log_${v}_$i.txt; exit 1; }
    f=$(find $O/prof_${v}_$i -name "*kernel_stats.csv" | head -1)
    echo "$v $i: $(python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'attn_' in n: print(n.split('(')[0].split('::')[-1][:28], round(float(r['AverageNs'])/1e3,1), end='  ')
")"
  done
done
for i in 1 2; do
  for v in dq4 head; do
    lib=""; [ $v = dq4 ] && lib=$PWD/variants/_dlion_C_dq4.so
    DLION_LIB=$lib timeout -k 10 300 python bench.py --steps 12 --warmup 3 > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail -20 $O/bench_${v}_$i.err; exit 1; }
    echo "$v $i $(tail -1 $O/bench_${v}_$i.json | cut -c80-160)"
  done
done
