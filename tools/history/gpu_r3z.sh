# Non-temporal dlogits stores (xent), nt operand DMA loads in the TN wgrad and the NT GEMM; GEMM tests on the default
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3z
timeout -k 10 300 python -u -m pytest tests/test_xent_gpu.py tests/test_gemm_tn_gpu.py tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3z/tests.log 2>&1 || { tail -30 gpurun_out/r3z/tests.log; exit 1; }
tail -1 gpurun_out/r3z/tests.log
for v in default xentnt tnnt ntload default xentnt tnnt ntload; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3z/bench_$v.json 2> gpurun_out/r3z/bench_$v.err || { tail -20 gpurun_out/r3z/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3z/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3z/bench_ab.txt
