# r6 call 3: GEMM roles vs the on-box anchor (same box), then every preset at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6c3; mkdir -p $O
timeout -k 10 200 python3 -u tools/gemm_anchor.py --square > $O/anchor.txt 2>&1 || { tail $O/anchor.txt; exit 1; }
timeout -k 10 300 python3 -u tools/gemm_shape_table.py > $O/gpt2_shapes.txt 2>&1 || { tail $O/gpt2_shapes.txt; exit 1; }
MODEL=llama3 timeout -k 10 300 python3 -u tools/bench_gemm_llama.py > $O/llama_shapes.jsonl 2>&1 || { tail $O/llama_shapes.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/r5/bench_wgrad_lt.py > $O/llama_wgrad.jsonl 2>&1 || { tail $O/llama_wgrad.jsonl; exit 1; }
bash tools/gpu_presets.sh > $O/presets.txt 2>&1; rc=$?; cp gpurun_out/presets.jsonl $O/ 2>/dev/null; cat $O/presets.txt | tail -12; exit $rc
