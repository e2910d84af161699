# r6 call 17: dK/dV step instantiated per LDS buffer at D = 64 (immediate LDS offsets; 5 / 2 SGPRs
# spilled outside the loop) vs HEAD (variants/_dlion_C_h2.so): attention tests, then per-kernel A/B
# at the GPT-2 shape and the D = 128 shape (whose code moved through the same lambda)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c17; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attention_gpu.py \
  > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_attention.sh $O/gpt2 3 prev=variants/_dlion_C_h2.so new=default -- 20 1024 12 64 0.1 || exit 1
bash tools/ab_attention.sh $O/d128 2 prev=variants/_dlion_C_h2.so new=default -- 1 8192 32 128 0.0 || exit 1
echo ab-done
