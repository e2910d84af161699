# SQ counters of the attention kernels, 4-wave (pp=0) vs ping-pong (pp=3)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 3; do
  DLION_ATTN_PP=$v bash tools/pmc_attn_sq.sh > /dev/null 2>&1 || { echo "pmc pp=$v failed"; exit 1; }
  mkdir -p gpurun_out/r5pmc && cp gpurun_out/pmc_attn_sq/summary.txt gpurun_out/r5pmc/summary_pp$v.txt
done
cat gpurun_out/r5pmc/summary_pp3.txt
