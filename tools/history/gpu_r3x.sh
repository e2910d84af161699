# NT GEMM epilogue with non-temporal aux / C stores (bench_gemm_epi per variant) + end-to-end A/B incl. the pipelined forward
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3x
for rep in 1 2; do
for v in default ntaux ntall; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  echo "== $v"
  DLION_LIB=$lib timeout -k 10 120 python tools/bench_gemm_epi.py || exit 1
done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3x/gemm_epi_ab.txt
for v in default fpipe ntaux ntall default fpipe ntaux ntall; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3x/bench_$v.json 2> gpurun_out/r3x/bench_$v.err || { tail -20 gpurun_out/r3x/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3x/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3x/bench_ab.txt
