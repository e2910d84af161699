# BASELINE config #5 rehearsal on ONE MI355X: Llama-3-8B full-parameter bf16 Distributed Lion, 3 rank
# processes sharing the GPU (gloo collectives), rank 1 SIGKILLed after issuing step 4's vote all-to-all;
# the survivors regroup, re-vote step 4 and finish with bit-identical replicas.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stress8b
timeout -k 10 900 python -m distributed_lion_pytorch_amd.launch --nproc 3 --max_failures 1 \
  --report gpurun_out/stress8b/launch.json dropout_stress.py --model llama-3-8b --backend gloo --device cuda \
  --micro_batch 1 --seq_len 2048 --steps 8 --drop_rank 1 --drop_step 4 --drop_phase after_launch \
  --elastic_timeout 120 > gpurun_out/stress8b/out.jsonl 2> gpurun_out/stress8b/err.log
rc=$?
echo "rc=$rc"; grep -v '"steps"' gpurun_out/stress8b/out.jsonl | cut -c1-300; grep '"metric"' gpurun_out/stress8b/out.jsonl | cut -c1-900
tail -5 gpurun_out/stress8b/err.log
exit $rc
