# Round-4: GPU suite, smoke, bench A/B vs round-3 attention, attention SQ counters, counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4c
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4c/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4c/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r4c/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4c/smoke.log 2>&1 || { tail -20 gpurun_out/r4c/smoke.log; exit 1; }
tail -1 gpurun_out/r4c/smoke.log
for r in 1 2; do
  echo "== r3 bench $r"; DLION_LIB=variants/_dlion_C_r3.so timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 2>/dev/null | cut -c1-120 || exit 1
  echo "== new bench $r"; timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 2>/dev/null | cut -c1-120 || exit 1
done 2>&1 | tee gpurun_out/r4c/bench_ab.txt
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r4c/counters.txt 2>&1 || true
bash tools/pmc_attn_sq.sh > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
cp gpurun_out/pmc_attn_sq/summary.txt gpurun_out/r4c/pmc_attn_sq_summary.txt
cat gpurun_out/r4c/pmc_attn_sq_summary.txt | grep -E "attn|wait_any|VALU/MFMA|mfma_busy"
