# hipBLASLt exhaustive algorithm search (DLION_LT_ALL=1) vs heuristic top-12: per-shape log, then GPT-2 bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3at
DLION_LT_ALL=1 DLION_LT_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > gpurun_out/r3at/verbose.json 2> gpurun_out/r3at/verbose.err || { tail -30 gpurun_out/r3at/verbose.err; exit 1; }
grep lt_gemm gpurun_out/r3at/verbose.err || true
for v in 1 0 1 0 1 0; do
  DLION_LT_ALL=$v timeout -k 10 300 python bench.py --steps 12 --warmup 3 > gpurun_out/r3at/bench_$v.json 2> gpurun_out/r3at/bench_$v.err || { tail -20 gpurun_out/r3at/bench_$v.err; exit 1; }
  echo "lt_all=$v $(python -c "import json;d=json.load(open('gpurun_out/r3at/bench_$v.json'));print(d['value'],d['ms_per_step'],d['loss'])")"
done | tee gpurun_out/r3at/bench_ab.txt
