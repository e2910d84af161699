# round-5 GPU call 6: TN per-XCD rotated k walk A/B (tests + Llama shapes, padded / unpadded)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tn_tests.log 2>&1 || { tail -30 $O/tn_tests.log; exit 1; }
tail -1 $O/tn_tests.log
PYTHONPATH=. timeout -k 10 400 python tools/r5/bench_tn_rot.py > $O/bench_tn_rot.txt 2>&1 || { tail -20 $O/bench_tn_rot.txt; exit 1; }
grep -v amdgpu.ids $O/bench_tn_rot.txt
