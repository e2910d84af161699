# Residual+norm kernels: batched row loads + DPP/permlane wave sums vs the old (serial chunk loads, ds_bpermute sums)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ad
timeout -k 10 300 python -u -m pytest tests/test_norm_gpu.py tests/test_models_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3ad/tests.log 2>&1 || { tail -30 gpurun_out/r3ad/tests.log; exit 1; }
tail -1 gpurun_out/r3ad/tests.log
for v in default oldnorm default oldnorm; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 120 python tools/bench_norm.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1
done | tee gpurun_out/r3ad/norm_bench.txt
for v in default oldnorm default oldnorm; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ad/bench_$v.json 2> gpurun_out/r3ad/bench_$v.err || { tail -20 gpurun_out/r3ad/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3ad/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3ad/bench_ab.txt
