# Per-shape GEMM choice vs pinning one candidate everywhere (own NT with non-temporal stores / tuned hipBLASLt / ATen)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ah
for v in auto own lt aten auto own; do
  f=$v; [ $v = auto ] && f=""
  DLION_GEMM_FORCE=$f timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ah/bench_$v.json 2> gpurun_out/r3ah/bench_$v.err || { tail -20 gpurun_out/r3ah/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3ah/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3ah/bench_ab.txt
