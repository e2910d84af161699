# r6 call 12: GEMM K-loop address work -- TN fragment reads with the constant address part in
# the ds offset field (TN loop VALU 89 -> 32), then both 8-phase kernels staging through the
# saddr form of the LDS-DMA load with a scalar wave index (TN loop VALU -> 0, NT 63 -> 8).
# Tests on the new build, then bench and per-kernel A/B: prev (HEAD), off (TN offsets only), new.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c12; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_gemm_tn_gpu.py tests/test_grad_fusion_gpu.py tests/test_dgelu_gpu.py \
  tests/test_parity_full_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # label lib round
  if [ "$2" == "default" ]; then L=""; else L="DLION_LIB=$2"; fi
  env $L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 2> $O/err_$1_$3.log | tail -1 \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'])"
}
for r in 1 2; do run prev variants/_dlion_C_bf.so $r || exit 1; run off variants/_dlion_C_off.so $r || exit 1; run new default $r || exit 1; done | tee $O/bench_ab.txt
prof() {  # label lib round
  if [ "$2" == "default" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1$3 -o prof \
      -- python3 bench.py --steps 6 --warmup 2 > $O/prof_$1$3.log 2>&1
  else
    DLION_LIB=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1$3 -o prof \
      -- python3 bench.py --steps 6 --warmup 2 > $O/prof_$1$3.log 2>&1
  fi
}
for r in 1 2; do prof prev variants/_dlion_C_bf.so $r && prof off variants/_dlion_C_off.so $r && prof new default $r || exit 1; done
echo ab-done
