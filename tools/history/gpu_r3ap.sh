# Outlier check: 4 fresh bench processes with the 5 % own-kernel margin (default), per-run JSON kept
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ap
for i in 1 2 3 4; do
  timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ap/bench_$i.json 2> gpurun_out/r3ap/bench_$i.err || { tail -20 gpurun_out/r3ap/bench_$i.err; exit 1; }
  echo "run$i $(python -c "import json;d=json.load(open('gpurun_out/r3ap/bench_$i.json'));print(d['value'],d['ms_per_step'],d['phase_ms_per_step'])")"
done | tee gpurun_out/r3ap/bench_runs.txt
