# Attention SQ counters at the GPT-2 shape (NB=2 tree) + dQ 4-wave floor A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3u
bash tools/pmc_attn_sq.sh 20 1024 12 64 0.1 > gpurun_out/r3u/pmc_sq.txt 2>&1 || { tail -20 gpurun_out/r3u/pmc_sq.txt; exit 1; }
cp gpurun_out/pmc_attn_sq/summary.txt gpurun_out/r3u/pmc_sq_summary.txt; cat gpurun_out/r3u/pmc_sq_summary.txt
for rep in 1 2 3; do
for v in default dq4; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  echo "== $v"
  DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py 20 1024 12 64 0.1 || exit 1
done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3u/dq4_ab.txt
