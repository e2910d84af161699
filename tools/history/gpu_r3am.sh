# Per-shape GEMM choice (auto: now picks the own NT kernel for the N = 768 input gradients) vs pinned tuned hipBLASLt / ATen, 3 interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3am
for rep in 1 2 3; do
for v in auto lt aten; do
  f=$v; [ $v = auto ] && f=""
  DLION_GEMM_FORCE=$f timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3am/bench_$v.json 2> gpurun_out/r3am/bench_$v.err || { tail -20 gpurun_out/r3am/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3am/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done
done | tee gpurun_out/r3am/bench_ab.txt
