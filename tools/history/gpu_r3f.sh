# Round 3 checkpoint: Llama bf16 diagnostic, full GPU suite, Lion roofline, bench + rocprof summary
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3f
timeout -k 10 300 python tools/diag_llama_bf16.py > gpurun_out/r3f/diag.log 2>&1; grep -v "Writing\|Loading\|amdgpu.ids" gpurun_out/r3f/diag.log | tail -16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread --deselect tests/test_parity_full_gpu.py::test_llama_7b_width_two_layers_vs_hf_fp32 > gpurun_out/r3f/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3f/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3f/gpu_tests.log
timeout -k 10 200 python tools/bench_lion.py gpt2 8 > gpurun_out/r3f/lion_gpt2.txt 2>&1 && timeout -k 10 300 python tools/bench_lion.py llama3 8 > gpurun_out/r3f/lion_llama3.txt 2>&1 || exit 1
cat gpurun_out/r3f/lion_gpt2.txt gpurun_out/r3f/lion_llama3.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3f/bench.json 2> gpurun_out/r3f/bench.err || { tail -20 gpurun_out/r3f/bench.err; exit 1; }
cut -c1-400 gpurun_out/r3f/bench.json
bash tools/profile_bench.sh r3 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/prof_r3 -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 24 40 > gpurun_out/r3f/gpt2_summary.txt; head -24 gpurun_out/r3f/gpt2_summary.txt | cut -c1-160
