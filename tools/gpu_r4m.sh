# dQ with two key tiles per barrier (DLION_DQ_NT64=2: 161 VGPRs, 3 waves): tests + per-kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4m; mkdir -p $O
DLION_LIB=variants/_dlion_C_dqnt2.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_attn_p.sh head=default:0.1 dqnt2=variants/_dlion_C_dqnt2.so:0.1 || exit 1
cp gpurun_out/attn_p/summary.txt $O/attn_summary.txt
