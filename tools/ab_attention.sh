# Attention kernel A/B across builds: per-kernel mean times from rocprofv3 of
# tools/bench_attention.py (our kernels only), alternating the builds for R rounds.
# Usage: bash tools/ab_attention.sh <out_dir> <rounds> <label=lib.so|default> ... [-- B T H D p]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1; R=$2; shift 2
mkdir -p $O
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
for r in $(seq 1 $R); do
  for lv in "${LIBS[@]}"; do
    label=${lv%%=*}; lib=${lv#*=}
    d=$O/${label}_r$r
    if [ "$lib" == "default" ]; then
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o prof -- python3 tools/bench_attention.py --ours-only "$@" > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    else
      DLION_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o prof -- python3 tools/bench_attention.py --ours-only "$@" > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    fi
    f=$(find $d -name "*kernel_stats.csv" | head -1)
    python3 tools/attn_kernel_times.py "${label}_r$r=$f" | tee -a $O/summary.txt
  done
done
