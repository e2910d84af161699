# DPO preset: auto checkpointing policy (activations kept in HBM) vs the reference setting, bf16 and 4-bit bases
set -o pipefail
cd $GRAFT_REPO_ROOT
: > gpurun_out/dpo_policy.jsonl
for extra in "" "--checkpointing_policy reference" "--load_in_4bit"; do
  timeout -k 10 500 python bench.py --task dpo --steps 3 --warmup 1 $extra > gpurun_out/dpo_p.log 2>&1 || { tail -20 gpurun_out/dpo_p.log; exit 1; }
  tail -1 gpurun_out/dpo_p.log >> gpurun_out/dpo_policy.jsonl
  tail -1 gpurun_out/dpo_p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["gradient_checkpointing"], d["config"]["base_weights"])'
done
