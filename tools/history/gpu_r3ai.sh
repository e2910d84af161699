# Non-temporal row loads in the residual+norm kernels (read-once streams) vs plain loads
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ai
for v in default normntld default normntld; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ai/bench_$v.json 2> gpurun_out/r3ai/bench_$v.err || { tail -20 gpurun_out/r3ai/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3ai/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3ai/bench_ab.txt
