# dK/dV one-hash-per-row-pair dropout (DPP swap): attention tests, per-kernel times vs the
# previous build (variants/_dlion_C_persist.so has the old attention), then the 3-rank
# Llama-3-8B dropout rehearsal (regroup time after the death-notice fix).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_attn_p.sh new=default:0.1 old=variants/_dlion_C_persist.so:0.1 dq4=variants/_dlion_C_dq4.so:0.1 || exit 1
cp gpurun_out/attn_p/summary.txt $O/attn_summary.txt
bash tools/gpu_stress_8b.sh > $O/stress8b.txt 2>&1; rc=$?; tail -12 $O/stress8b.txt; cp -r gpurun_out/stress8b $O/ 2>/dev/null; exit $rc
