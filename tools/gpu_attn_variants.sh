# attention kernel variants: per-kernel times under rocprofv3 (2 interleaved rounds), GPT-2 shape
# usage: bash tools/gpu_attn_variants.sh label=lib.so ...   (label=default uses the in-tree build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/attn_var; rm -rf $OUT; mkdir -p $OUT
for r in 1 2; do
  for v in "$@"; do
    label=${v%%=*}; lib=${v#*=}
    if [ "$lib" = "default" ]; then unset DLION_LIB; else export DLION_LIB=$lib; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$label$r -o p -- python3 tools/bench_attention.py --ours-only > $OUT/$label$r.log 2>&1 || { tail -5 $OUT/$label$r.log; exit 1; }
    f=$(find $OUT/$label$r -name "*kernel_stats.csv" | head -1)
    python3 tools/attn_kernel_times.py "$label=$f"
  done
done | tee $OUT/summary.txt
