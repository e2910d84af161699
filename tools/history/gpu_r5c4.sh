# round-5 GPU call 4: TN weight-gradient kernel at the Llama-3-8B shapes (bench + PMC vs NT)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tn_tests.log 2>&1 || { tail -30 $O/tn_tests.log; exit 1; }
tail -2 $O/tn_tests.log
PYTHONPATH=. timeout -k 10 300 python tools/r5/bench_tn_llama.py > $O/bench_tn_llama.txt 2>&1 || { tail -20 $O/bench_tn_llama.txt; exit 1; }
grep -v amdgpu.ids $O/bench_tn_llama.txt
bash tools/pmc_gemm_tn.sh || exit 1
