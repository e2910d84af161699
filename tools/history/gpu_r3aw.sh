# hipBLASLt search with slow-algorithm early drop: per-shape log + wall time of a short bench, then interleaved A/B vs heuristic-only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3aw
s=$(date +%s.%N)
DLION_LT_VERBOSE=1 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > gpurun_out/r3aw/verbose.json 2> gpurun_out/r3aw/verbose.err || { tail -30 gpurun_out/r3aw/verbose.err; exit 1; }
e=$(date +%s.%N); echo "wall (search on, steps 4 warmup 2): $(python -c "print(round($e-$s,1))") s"
grep lt_gemm gpurun_out/r3aw/verbose.err || true
s=$(date +%s.%N)
DLION_LT_ALL=0 timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > /dev/null 2>&1 || exit 1
e=$(date +%s.%N); echo "wall (search off, steps 4 warmup 2): $(python -c "print(round($e-$s,1))") s"
for v in 1 0 1 0; do
  DLION_LT_ALL=$v timeout -k 10 300 python bench.py --steps 12 --warmup 3 > gpurun_out/r3aw/bench_$v.json 2> gpurun_out/r3aw/bench_$v.err || { tail -20 gpurun_out/r3aw/bench_$v.err; exit 1; }
  echo "lt_all=$v $(python -c "import json;d=json.load(open('gpurun_out/r3aw/bench_$v.json'));print(d['value'],d['ms_per_step'],d['loss'])")"
done
