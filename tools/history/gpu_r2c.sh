set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=25 bash tools/gpu_runclm.sh nb_log5 --logging_steps 5 || exit 1
mkdir -p gpurun_out/prof_runclm
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_runclm -o prof -- python3 run_clm.py --config_name gpt2 --synthetic_data --synthetic_samples 4000 \
  --per_device_train_batch_size 20 --do_train --output_dir /tmp/rc_prof --report_to none \
  --torch_dtype bfloat16 --gradient_accumulation_steps 8 --max_steps 6 --warmup_steps 2 --lion \
  --learning_rate 1e-4 --weight_decay 0.1 --async_grad --logging_steps 5 --save_strategy no > gpurun_out/prof_runclm/log.txt 2>&1 || { tail -20 gpurun_out/prof_runclm/log.txt; exit 1; }
f=$(find /tmp/prof_runclm -name "*kernel_trace.csv" | head -1)
python tools/prof_gaps.py $f 0.4 | tee gpurun_out/prof_runclm/gaps.txt
mkdir -p gpurun_out/prof_bench
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_bench -o prof -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_bench/log.txt 2>&1 || { tail -20 gpurun_out/prof_bench/log.txt; exit 1; }
f=$(find /tmp/prof_bench -name "*kernel_trace.csv" | head -1)
python tools/prof_gaps.py $f 0.4 | tee gpurun_out/prof_bench/gaps.txt
