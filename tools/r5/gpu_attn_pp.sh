# ping-pong attention backward A/B: numerics vs fp32 with the pp kernels on, then
# per-kernel rocprof times and fwd+bwd wall time, old (0) vs pp (mask), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5pp; mkdir -p $O
MASK=${1:-3}
DLION_ATTN_PP=$MASK timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 0 $MASK; do
  DLION_ATTN_PP=$v DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$v -o p -- python3 tools/bench_attention.py > $O/prof$v.log 2>&1 || { tail -20 $O/prof$v.log; exit 1; }
done
for v in 0 $MASK; do python tools/attn_kernel_times.py pp$v=$(find $O/prof$v -name "*kernel_stats.csv" | head -1); done
for r in 1 2; do for v in 0 $MASK; do
  DLION_ATTN_PP=$v DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py > $O/bench_${v}_$r.txt 2>&1 || exit 1
  echo "pp=$v $(grep ours_fb $O/bench_${v}_$r.txt)"
done; done
