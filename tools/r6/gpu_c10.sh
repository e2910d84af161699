# r6 call 10: branch-free K loops in the own NT and TN GEMM kernels -- GEMM/fusion/parity
# tests on the new build, then a bench and per-kernel A/B against the previous build
# (variants/_dlion_C_head.so), alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c10; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_gemm_tn_gpu.py tests/test_grad_fusion_gpu.py tests/test_dgelu_gpu.py \
  tests/test_parity_full_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # label lib round
  if [ "$2" == "default" ]; then L=""; else L="DLION_LIB=$2"; fi
  env $L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 2> $O/err_$1_$3.log | tail -1 \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'])"
}
for r in 1 2 3; do run head variants/_dlion_C_head.so $r || exit 1; run new default $r || exit 1; done | tee $O/bench_ab.txt
DLION_LIB=variants/_dlion_C_head.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_head -o prof \
  -- python3 bench.py --steps 10 --warmup 3 > $O/prof_head.log 2>&1 || { tail -5 $O/prof_head.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o prof \
  -- python3 bench.py --steps 10 --warmup 3 > $O/prof_new.log 2>&1 || { tail -5 $O/prof_new.log; exit 1; }
echo done
