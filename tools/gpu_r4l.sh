# dQ with dO (ops1) / Q and dO (ops3) read from LDS per tile (DLION_DQ_OPS_LDS): tests + per-kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4l; mkdir -p $O
for v in ops1 ops3; do
  DLION_LIB=variants/_dlion_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -40 $O/tests_$v.log; exit 1; }
  tail -1 $O/tests_$v.log
done
bash tools/gpu_attn_p.sh head=default:0.1 ops1=variants/_dlion_C_ops1.so:0.1 ops3=variants/_dlion_C_ops3.so:0.1 || exit 1
cp gpurun_out/attn_p/summary.txt $O/attn_summary.txt
