# GEMM epilogue costs (fc shape) + attention LDS ring depth 4 (no spill, 3 tiles in flight) and the software-pipelined dQ loop vs default: kernels and end to end
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3w
timeout -k 10 200 python tools/bench_gemm_epi.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3w/gemm_epi.txt
for v in st4 pipe fpipe kpipe; do
  DLION_LIB=$PWD/variants/_dlion_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3w/attn_tests_$v.log 2>&1 || { tail -30 gpurun_out/r3w/attn_tests_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r3w/attn_tests_$v.log)"
done
for rep in 1 2 3; do
for v in default st4 pipe fpipe kpipe; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  echo "== $v"
  DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py 20 1024 12 64 0.1 || exit 1
done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3w/attn_ab.txt
for v in default st4 pipe fpipe kpipe default st4 pipe fpipe kpipe; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3w/bench_$v.json 2> gpurun_out/r3w/bench_$v.err || { tail -20 gpurun_out/r3w/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3w/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3w/bench_ab.txt
