# attention start stagger (DLION_ATTN_STAGGER = sleep units of 64 cycles per co-resident block lag)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4k; mkdir -p $O
bash tools/gpu_attn_p.sh head=default:0.1 stag10=variants/_dlion_C_stag10.so:0.1 stag20=variants/_dlion_C_stag20.so:0.1 || exit 1
cp gpurun_out/attn_p/summary.txt $O/attn_summary.txt
