# Round 3: full-size parity vs HF fp32, learning-curve A/B (native vs reference, W=1 and W=2 gloo on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests/test_parity_full_gpu.py tests/test_embedding_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r3b/parity.log 2>&1; rc=$?
tail -5 gpurun_out/r3b/parity.log; [ $rc -eq 0 ] || grep -E "assert|Error" gpurun_out/r3b/parity.log | head -20
COMMON="--steps 50 --data markov --seq_len 1024"
timeout -k 10 300 python bench.py $COMMON --loss_log gpurun_out/r3b/curve_native_w1.jsonl > gpurun_out/r3b/c1.log 2>&1 || exit 1
timeout -k 10 400 python bench.py $COMMON --impl reference --loss_log gpurun_out/r3b/curve_reference_w1.jsonl > gpurun_out/r3b/c2.log 2>&1 || exit 1
P=$(python -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --backend gloo $COMMON --loss_log gpurun_out/r3b/curve_native_w2.jsonl > gpurun_out/r3b/c3.log 2>&1 || exit 1
P=$(python -c "import socket;s=socket.socket();s.bind(('127.0.0.1',0));print(s.getsockname()[1])")
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --backend gloo $COMMON --impl reference --loss_log gpurun_out/r3b/curve_reference_w2.jsonl > gpurun_out/r3b/c4.log 2>&1 || exit 1
python - <<'PY'
import json
for w in (1, 2):
    a = [json.loads(l)["loss"] for l in open(f"gpurun_out/r3b/curve_native_w{w}.jsonl")]
    b = [json.loads(l)["loss"] for l in open(f"gpurun_out/r3b/curve_reference_w{w}.jsonl")]
    print(f"W={w} native  ", [round(x, 3) for x in a[::5]], a[-1])
    print(f"W={w} reference", [round(x, 3) for x in b[::5]], b[-1])
    print(f"W={w} max |diff| {max(abs(x-y) for x,y in zip(a,b)):.4f}")
PY
exit $rc
