set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python tools/trace_runclm.py /tmp/rc_trace.json --config_name gpt2 --synthetic_data --synthetic_samples 2000 \
  --per_device_train_batch_size 20 --do_train --output_dir /tmp/rc_tr --report_to none \
  --torch_dtype bfloat16 --gradient_accumulation_steps 8 --max_steps 5 --warmup_steps 2 --lion \
  --learning_rate 1e-4 --weight_decay 0.1 --async_grad --logging_steps 5 --save_strategy no > gpurun_out/trace_runclm.log 2>&1 || { tail -20 gpurun_out/trace_runclm.log; exit 1; }
python tools/trace_gaps.py /tmp/rc_trace.json 80 0.4 > gpurun_out/trace_runclm_gaps.txt; tail -120 gpurun_out/trace_runclm_gaps.txt
