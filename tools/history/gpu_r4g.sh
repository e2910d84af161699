# (1) [separate call: tools/gpu_stress_8b.sh]
# (2) no-failure cost of elastic mode: GPT-2, 2 gloo ranks on one GPU, with vs without --elastic_timeout,
# (3) vote bucket sweep on the 8-rank gloo rehearsal (exposed exchange ms per step),
# (4) Lion kernel roofline at HEAD (K1 dword stores), (0) EPI 6 cost split (DLION_EPI_DIAG builds).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g; mkdir -p $O
for lib in distributed_lion_pytorch_amd/_dlion_C.so variants/_dlion_C_diag1.so variants/_dlion_C_diag2.so; do
  echo "== $lib" >> $O/epi_diag.txt
  DLION_LIB=$lib timeout -k 10 120 python -u tools/bench_gemm_epi.py 20480 3072 768 >> $O/epi_diag.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/epi_diag.txt
timeout -k 10 120 python tools/bench_lion.py gpt2 8 > $O/lion_gpt2.txt 2>&1 || { tail -20 $O/lion_gpt2.txt; exit 1; }
timeout -k 10 300 python tools/bench_lion.py llama3 8 > $O/lion_llama3.txt 2>&1 || { tail -20 $O/lion_llama3.txt; exit 1; }
cat $O/lion_gpt2.txt $O/lion_llama3.txt
for el in "" "--elastic_timeout 120"; do
  for i in 1 2; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
      bench.py --gpus 2 --backend gloo --steps 4 --warmup 2 $el > $O/el.log 2>&1 || { tail -30 $O/el.log; exit 1; }
    tail -1 $O/el.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('elastic=[$el]', d['ms_per_step'], d['phase_ms_per_step'])" | tee -a $O/elastic_cost.txt
  done
done
for mb in 1 4 32 auto; do
  arg=$([ $mb = auto ] && echo "" || echo "--bucket_mb $mb")
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 8 --backend gloo --steps 3 --warmup 1 --micro_batch 2 --grad_accum 2 $arg > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 1; }
  tail -1 $O/sweep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bucket_mb=$mb', 'buckets', d['optimizer_stats'].get('n_buckets'), 'ms/step', d['ms_per_step'], d['phase_ms_per_step'])" | tee -a $O/bucket_sweep.txt
done
