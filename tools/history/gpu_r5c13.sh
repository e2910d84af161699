# round-5 GPU call 13: dK/dV hash bases computed per wave (its own key tile) vs on one wave (variant lib):
# attention tests, then per-kernel times (rocprofv3 --kernel-trace --stats) of the GPT-2-shape attention bench, 2 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c13; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in new old; do
    lib=""; [ $v = old ] && lib=$PWD/variants/_dlion_C_hashw1.so
    DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v}_$i -o p -- python3 tools/bench_attention.py 20 1024 12 64 0.1 > $O/log_${v}_$i.txt 2>&1 || { tail -20 $O/log_${v}_$i.txt; exit 1; }
    f=$(find $O/prof_${v}_$i -name "*kernel_stats.csv" | head -1)
    echo "$v $i: $(python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name']
    if 'attn_' in n: print(n.split('(')[0].split('::')[-1][:28], round(float(r['AverageNs'])/1e3,1), end='  ')
")"
  done
done
