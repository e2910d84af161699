# GEMM choice with a 5 % margin for the own kernel (default now) vs no margin vs pinned tuned hipBLASLt; Llama SFT must keep its own-kernel picks
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ao
for rep in 1 2 3; do
for v in margin nomargin lt; do
  m=0.05; f=""
  [ $v = nomargin ] && m=0
  [ $v = lt ] && f=lt
  DLION_GEMM_OWN_MARGIN=$m DLION_GEMM_FORCE=$f timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3ao/bench_$v.json 2> gpurun_out/r3ao/bench_$v.err || { tail -20 gpurun_out/r3ao/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3ao/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done
done | tee gpurun_out/r3ao/bench_ab.txt
for v in margin nomargin; do
  m=0.05; [ $v = nomargin ] && m=0
  DLION_GEMM_OWN_MARGIN=$m timeout -k 10 400 python bench.py --task sft --steps 4 --warmup 2 > gpurun_out/r3ao/sft_$v.json 2> gpurun_out/r3ao/sft_$v.err || { tail -20 gpurun_out/r3ao/sft_$v.err; exit 1; }
  echo "sft $v $(python -c "import json;d=json.load(open('gpurun_out/r3ao/sft_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee -a gpurun_out/r3ao/bench_ab.txt
