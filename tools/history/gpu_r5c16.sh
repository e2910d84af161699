# round-5 GPU call 16: grouped weight-gradient launch at the fusion window's exit: tests + GPT-2 bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c16; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_tn_gpu.py tests/test_grad_fusion_gpu.py tests/test_xent_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for gr in 1 0; do
    DLION_TN_GROUP=$gr timeout -k 10 300 python bench.py --steps 12 --warmup 3 > $O/bench_g$gr.$i.json 2> $O/bench_g$gr.$i.err || { tail -20 $O/bench_g$gr.$i.err; exit 1; }
    echo "group=$gr $i $(tail -1 $O/bench_g$gr.$i.json | cut -c80-160)"
  done
done
