# r6 call 13: GEMM tables after the K-loop address diet -- on-box anchor, TN layout rows, the GPT-2
# and Llama-3-8B GEMM roles (for tools/gemm_vs_anchor.py), then every bench preset at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c13; mkdir -p $O
timeout -k 10 300 python3 -u tools/gemm_anchor.py --tn > $O/anchor_tn.txt 2>&1 || { tail $O/anchor_tn.txt; exit 1; }
timeout -k 10 300 python3 -u tools/gemm_shape_table.py > $O/gpt2_shapes.txt 2>&1 || { tail $O/gpt2_shapes.txt; exit 1; }
MODEL=llama3 timeout -k 10 300 python3 -u tools/bench_gemm_llama.py > $O/llama_shapes.jsonl 2>&1 || { tail $O/llama_shapes.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/r5/bench_wgrad_lt.py > $O/llama_wgrad.jsonl 2>&1 || { tail $O/llama_wgrad.jsonl; exit 1; }
python3 tools/gemm_vs_anchor.py $O/anchor_tn.txt $O/gpt2_shapes.txt $O/llama_shapes.jsonl $O/llama_wgrad.jsonl > $O/gemm_vs_anchor.txt 2>&1
tail -12 $O/gemm_vs_anchor.txt
bash tools/gpu_presets.sh > $O/presets.txt 2>&1; rc=$?; cp gpurun_out/presets.jsonl $O/ 2>/dev/null; tail -12 $O/presets.txt; exit $rc
