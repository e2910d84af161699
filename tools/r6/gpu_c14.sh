# r6 call 14: persistent own NT GEMM (grid = min(tiles, CUs); a block walks its tiles, the next
# tile's prologue DMA issued right after its park region is drained) vs HEAD (variants/_dlion_C_h2.so).
# GEMM tests on the new build, then bench and per-kernel A/B, builds alternated.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c14; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_dgelu_gpu.py tests/test_grad_fusion_gpu.py tests/test_parity_full_gpu.py \
  tests/test_llama_ops_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # label lib round
  if [ "$2" == "default" ]; then L=""; else L="DLION_LIB=$2"; fi
  env $L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 2> $O/err_$1_$3.log | tail -1 \
    | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'])"
}
for r in 1 2 3; do run prev variants/_dlion_C_h2.so $r || exit 1; run new default $r || exit 1; done | tee $O/bench_ab.txt
prof() {  # label lib round
  if [ "$2" == "default" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1$3 -o prof \
      -- python3 bench.py --steps 6 --warmup 2 > $O/prof_$1$3.log 2>&1
  else
    DLION_LIB=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$1$3 -o prof \
      -- python3 bench.py --steps 6 --warmup 2 > $O/prof_$1$3.log 2>&1
  fi
}
for r in 1 2; do prof prev variants/_dlion_C_h2.so $r && prof new default $r || exit 1; done
echo ab-done
