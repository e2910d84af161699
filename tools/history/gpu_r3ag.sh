# LM-head logits GEMM on the own NT kernel (non-temporal C stores) vs the autotuned choice (hipBLASLt)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ag
for v in 0 1 0 1; do
  DLION_LM_FWD_OWN=$v timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ag/bench_$v.json 2> gpurun_out/r3ag/bench_$v.err || { tail -20 gpurun_out/r3ag/bench_$v.err; exit 1; }
  echo "lm_fwd_own=$v $(python -c "import json;d=json.load(open('gpurun_out/r3ag/bench_$v.json'));print(d['value'],d['ms_per_step'],d['loss'])")"
done | tee gpurun_out/r3ag/bench_ab.txt
