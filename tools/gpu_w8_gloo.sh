# Rehearse the 8-rank distributed path on a 1-GPU box: 8 ranks share the GPU,
# collectives over gloo (RCCL refuses two ranks per device); HIP kernels,
# 1-bit a2a vote exchange and Lion update as in the real run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ex in a2a allgather; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --micro_batch 2 --grad_accum 2 --exchange $ex \
  > gpurun_out/w8_gloo_$ex.log 2>&1 || { tail -30 gpurun_out/w8_gloo_$ex.log; exit 1; }
tail -1 gpurun_out/w8_gloo_$ex.log | cut -c1-600
done
