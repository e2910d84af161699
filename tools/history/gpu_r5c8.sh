# round-5 GPU call 8: zero-copy fused projection weights (pack_projections): tests + Llama-3-8B A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_tn_gpu.py tests/test_llama_ops_gpu.py tests/test_grad_fusion_gpu.py tests/test_xent_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for pk in 1 0; do
    DLION_PACK_PROJ=$pk timeout -k 10 400 python bench.py --task llama3 --steps 4 --warmup 2 > $O/l3_pack$pk.$i.json 2> $O/l3_pack$pk.$i.err || { tail -20 $O/l3_pack$pk.$i.err; exit 1; }
    echo "pack=$pk $(tail -1 $O/l3_pack$pk.$i.json | cut -c1-200)"
  done
done
