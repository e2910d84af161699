# Llama-3-8B preset with the LM-head weight gradient deferred into the window (default) vs per micro-batch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ak
for v in 1 0; do
  DLION_LM_DEFER=$v timeout -k 10 500 python bench.py --task llama3 --steps 4 --warmup 2 > gpurun_out/r3ak/llama3_$v.json 2> gpurun_out/r3ak/llama3_$v.err || { tail -20 gpurun_out/r3ak/llama3_$v.err; exit 1; }
  echo "llama3 lm_defer=$v $(python -c "import json;d=json.load(open('gpurun_out/r3ak/llama3_$v.json'));print(d['value'],d['ms_per_step'],d['loss'])")"
done | tee gpurun_out/r3ak/bench_ab.txt
