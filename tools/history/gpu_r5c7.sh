# round-5 GPU call 7: LM-head weight gradient unsplit in the backward (tests + Llama-3-8B preset A/B + bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c7; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_xent_gpu.py tests/test_gemm_tn_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for late in 1 0; do
    DLION_LM_LATE=$late timeout -k 10 400 python bench.py --task llama3 --steps 4 --warmup 2 > $O/l3_late$late.$i.json 2> $O/l3_late$late.$i.err || { tail -20 $O/l3_late$late.$i.err; exit 1; }
    echo "late=$late $(tail -1 $O/l3_late$late.$i.json | cut -c1-200)"
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
