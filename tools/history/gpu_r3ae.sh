# GELU in sigmoid form (8 VALU + 2 transcendental per element vs ~17 + 2): epilogue bench + end to end vs oldgelu; kernel tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ae
timeout -k 10 300 python -u -m pytest tests/test_dgelu_gpu.py tests/test_gemm_gpu.py tests/test_xent_gpu.py tests/test_norm_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3ae/tests.log 2>&1 || { tail -30 gpurun_out/r3ae/tests.log; exit 1; }
tail -1 gpurun_out/r3ae/tests.log
for v in default oldgelu default oldgelu; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  echo "== $v"; DLION_LIB=$lib timeout -k 10 120 python tools/bench_gemm_epi.py 2>&1 | grep -v amdgpu.ids | grep "EPI[268]" || exit 1
done | tee gpurun_out/r3ae/gemm_epi.txt
for v in default oldgelu default oldgelu; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ae/bench_$v.json 2> gpurun_out/r3ae/bench_$v.err || { tail -20 gpurun_out/r3ae/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3ae/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3ae/bench_ab.txt
