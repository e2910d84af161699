# persistent NT GEMM: bit-identity tests, per-epilogue timing at the GPT-2 shapes,
# then same-box bench.py A/B (default build vs -D DLION_GEMM_PERSIST=1), and the
# HF-path DPO timing with the checkpointing decision fixed.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_dgelu_gpu.py tests/test_kernels_gpu.py tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
DLION_LIB=variants/_dlion_C_persist.so timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_dgelu_gpu.py tests/test_grad_fusion_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests_p.log 2>&1 || { tail -40 $O/tests_p.log; exit 1; }
tail -1 $O/tests_p.log
for shp in "20480 3072 768" "20480 768 3072" "20480 2304 768" "20480 768 768"; do
  timeout -k 10 120 python -u tools/bench_gemm_epi.py $shp >> $O/epi.txt 2>&1 || exit 1
done
cat $O/epi.txt
bash tools/ab_bench.sh "" "DLION_LIB=variants/_dlion_C_persist.so" 3 --steps 10 --warmup 3 | tee $O/ab.txt || exit 1
rm -rf /tmp/hf_dpo
timeout -k 10 600 python -u dpo_llama2.py --model_name_or_path llama-2-7b --output_dir /tmp/hf_dpo --max_steps 8 \
  --logging_steps 1 --eval_steps 0 --warmup_steps 2 --lion --async_grad --final_save false \
  --synthetic_samples 400 --synthetic_chars 1000 > $O/dpo.log 2>&1 || { tail -30 $O/dpo.log; exit 1; }
cp /tmp/hf_dpo/metrics.jsonl $O/dpo_metrics.jsonl
grep -h "checkpointing" $O/dpo.log || true
python -c "
import json
t=[json.loads(l).get('tokens_per_s') for l in open('$O/dpo_metrics.jsonl')]
print('dpo HF tok/s', [round(x) for x in t if x])"
