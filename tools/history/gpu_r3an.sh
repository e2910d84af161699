# Plain-epilogue (EPI 0/1) outputs with normal stores (default now) vs non-temporal (ntplain); auto GEMM choice vs pinned tuned hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3an
for rep in 1 2 3; do
for v in auto ntplain lt; do
  lib=""; f=""
  [ $v = ntplain ] && lib=$PWD/variants/_dlion_C_ntplain.so
  [ $v = lt ] && f=lt
  DLION_LIB=$lib DLION_GEMM_FORCE=$f timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3an/bench_$v.json 2> gpurun_out/r3an/bench_$v.err || { tail -20 gpurun_out/r3an/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3an/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done
done | tee gpurun_out/r3an/bench_ab.txt
