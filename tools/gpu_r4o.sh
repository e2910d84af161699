# dK/dV with K straight from global into registers (DLION_DKV_KREG=2, no LDS copy of K) and with
# that LDS spent on a 4-deep Q / dO ring (DLION_DKV_STAGES=4, 3 blocks per CU): tests + per-kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4o; mkdir -p $O
for v in k2 k2nb4; do
  DLION_LIB=variants/_dlion_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -40 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
bash tools/gpu_attn_p.sh head=default:0.1 k2=variants/_dlion_C_k2.so:0.1 k2nb4=variants/_dlion_C_k2nb4.so:0.1 || exit 1
cp gpurun_out/attn_p/summary.txt $O/attn_summary.txt
