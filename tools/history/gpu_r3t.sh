# Attention backward regression hunt: LDS ring depth (3 vs 2) x dK/dV occupancy floor (3 vs none), kernel + end-to-end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3t
for rep in 1 2; do
for v in default st2 w1 st2w1; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  echo "== $v"
  DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py 20 1024 12 64 0.1 || exit 1
done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3t/attn_ab.txt
for v in default st2w1 w1 st2; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3t/bench_$v.json 2> gpurun_out/r3t/bench_$v.err || { tail -20 gpurun_out/r3t/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3t/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3t/bench_ab.txt
