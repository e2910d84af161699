# 4-bit (QLoRA) path on one MI355X: kernel tests, expansion bandwidth, SFT/DPO benches with --load_in_4bit
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py tests/test_lora_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/quant_tests.log 2>&1 || { tail -40 gpurun_out/quant_tests.log; exit 1; }
tail -3 gpurun_out/quant_tests.log
timeout -k 10 120 python tools/bench_quant.py > gpurun_out/bench_quant.jsonl 2>gpurun_out/bench_quant.err || { tail -20 gpurun_out/bench_quant.err; exit 1; }
cat gpurun_out/bench_quant.jsonl
timeout -k 10 400 python bench.py --task sft --load_in_4bit --steps 4 --warmup 2 > gpurun_out/bench_sft4.log 2>&1 || { tail -30 gpurun_out/bench_sft4.log; exit 1; }
tail -1 gpurun_out/bench_sft4.log
timeout -k 10 400 python bench.py --task dpo --load_in_4bit --steps 3 --warmup 1 > gpurun_out/bench_dpo4.log 2>&1 || { tail -30 gpurun_out/bench_dpo4.log; exit 1; }
tail -1 gpurun_out/bench_dpo4.log
