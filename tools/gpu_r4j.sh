# dK/dV with the wave's K fragments in registers (DLION_DKV_KREG=1) and the attention start
# stagger (DLION_ATTN_STAGGER = sleep units of 64 cycles per co-resident block lag): tests of the
# kreg build, then per-kernel times of head / kreg / stag10 / stag20
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4j; mkdir -p $O
DLION_LIB=variants/_dlion_C_kreg.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_attn_p.sh head=default:0.1 kreg=variants/_dlion_C_kreg.so:0.1 stag10=variants/_dlion_C_stag10.so:0.1 stag20=variants/_dlion_C_stag20.so:0.1 || exit 1
cp gpurun_out/attn_p/summary.txt $O/attn_summary.txt
