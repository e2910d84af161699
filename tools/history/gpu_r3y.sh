# Non-temporal stores beyond the NT GEMM (now default): norm rows, attention O/dQ/dK/dV; GEMM tests on the new default
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3y
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_dgelu_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3y/tests.log 2>&1 || { tail -30 gpurun_out/r3y/tests.log; exit 1; }
tail -1 gpurun_out/r3y/tests.log
for v in default ntnorm ntattn ntboth default ntnorm ntattn ntboth; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3y/bench_$v.json 2> gpurun_out/r3y/bench_$v.err || { tail -20 gpurun_out/r3y/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3y/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3y/bench_ab.txt
