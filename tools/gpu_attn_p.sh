# attention per-kernel times at dropout p = 0 vs 0.1 (GPT-2 shape), default build and given variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/attn_p; rm -rf $OUT; mkdir -p $OUT
for r in 1 2; do
  for v in "$@"; do
    label=${v%%=*}; rest=${v#*=}; lib=${rest%%:*}; p=${rest#*:}
    if [ "$lib" = "default" ]; then unset DLION_LIB; else export DLION_LIB=$lib; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$label$r -o p -- python3 tools/bench_attention.py --ours-only 20 1024 12 64 $p > $OUT/$label$r.log 2>&1 || { tail -5 $OUT/$label$r.log; exit 1; }
    f=$(find $OUT/$label$r -name "*kernel_stats.csv" | head -1)
    python3 tools/attn_kernel_times.py "$label=$f"
  done
done | tee $OUT/summary.txt
