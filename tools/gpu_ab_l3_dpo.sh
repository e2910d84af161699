# A/B: Llama-3-8B wgrad on the own TN kernel vs hipBLASLt; DPO with / without activation checkpointing
set -o pipefail
cd $GRAFT_REPO_ROOT
for env in "DLION_TN_GEMM=1" "DLION_TN_GEMM=0" "DLION_TN_GEMM=1"; do
  env $env timeout -k 10 400 python bench.py --task llama3 --steps 4 --warmup 2 > gpurun_out/ab_l3.log 2>&1 || { tail -20 gpurun_out/ab_l3.log; exit 1; }
  echo "$env $(tail -1 gpurun_out/ab_l3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 500 python bench.py --task dpo --no_gradient_checkpointing --steps 3 --warmup 1 > gpurun_out/dpo_nockpt.log 2>&1 || { tail -20 gpurun_out/dpo_nockpt.log; exit 1; }
tail -1 gpurun_out/dpo_nockpt.log | cut -c1-200
