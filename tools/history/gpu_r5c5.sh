# round-5 GPU call 5: TN kernel without the per-pair pointer-table load; operand row-stride padding sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tn_tests.log 2>&1 || { tail -30 $O/tn_tests.log; exit 1; }
tail -1 $O/tn_tests.log
PYTHONPATH=. timeout -k 10 300 python tools/r5/bench_tn_llama.py > $O/bench_tn_llama.txt 2>&1 || { tail -20 $O/bench_tn_llama.txt; exit 1; }
grep -v amdgpu.ids $O/bench_tn_llama.txt
PYTHONPATH=. timeout -k 10 300 python tools/r5/bench_tn_pad.py > $O/bench_tn_pad.txt 2>&1 || { tail -20 $O/bench_tn_pad.txt; exit 1; }
grep -v amdgpu.ids $O/bench_tn_pad.txt
