set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/acc
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_grad_fusion_gpu.py tests/test_llama_ops_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
DLION_SPLITK_ACC=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/off$i.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/on$i.log 2>&1 || exit 1
echo off$i $(tail -1 $O/off$i.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
echo on$i $(tail -1 $O/on$i.log | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
done
