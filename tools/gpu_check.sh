# GPU validation round: tests, run_clm / sft on the GPU, bench.
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/gpu_tests.log | head -20; exit 1; }
rm -rf /tmp/clm && timeout -k 10 300 python run_clm.py --config_name gpt2 --synthetic_data --synthetic_samples 2000 \
  --per_device_train_batch_size 20 --gradient_accumulation_steps 2 --max_steps 6 --warmup_steps 1 --bf16 \
  --torch_dtype bfloat16 --lion --async_grad --do_train --output_dir /tmp/clm --logging_steps 2 --report_to none \
  --save_steps 6 > gpurun_out/run_clm_gpu.log 2>&1 || { tail -30 gpurun_out/run_clm_gpu.log; exit 1; }
grep -E "train_loss|train_samples_per_second" gpurun_out/run_clm_gpu.log | tail -2; tail -1 /tmp/clm/metrics.jsonl | cut -c1-300
rm -rf /tmp/sft && timeout -k 10 400 python sft_llama2.py --model_name llama-2-7b --synthetic_data --synthetic_samples 2000 --seq_length 1024 \
  --output_dir /tmp/sft --max_steps 3 --per_device_train_batch_size 4 --gradient_accumulation_steps 1 \
  --learning_rate 1e-4 --lion --async_grad --report_to none --logging_steps 1 --bf16 --save_strategy no \
  > gpurun_out/sft_gpu.log 2>&1 || { tail -30 gpurun_out/sft_gpu.log; exit 1; }
grep -E "trainable|train_runtime|'loss'" gpurun_out/sft_gpu.log | tail -3
