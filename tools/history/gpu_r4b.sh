# Attention dropout v2 (packed keep masks): kernel tests, old/new attention A/B, full GPU suite, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/attn_tests.log 2>&1 || { tail -40 gpurun_out/r4b/attn_tests.log; exit 1; }
tail -1 gpurun_out/r4b/attn_tests.log
for r in 1 2 3; do
  echo "== r3 round $r"; DLION_LIB=variants/_dlion_C_r3.so DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py || exit 1
  echo "== new round $r"; DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r4b/attn_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/r4b/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r4b/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/r4b/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4b/smoke.log 2>&1 || { tail -20 gpurun_out/r4b/smoke.log; exit 1; }
tail -1 gpurun_out/r4b/smoke.log
for r in 1 2; do
  echo "== r3 bench $r"; DLION_LIB=variants/_dlion_C_r3.so timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 2>/dev/null | cut -c1-120 || exit 1
  echo "== new bench $r"; timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 2>/dev/null | cut -c1-120 || exit 1
done 2>&1 | tee gpurun_out/r4b/bench_ab.txt
