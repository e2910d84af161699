# Fewer attention-backward barriers: dQ with 2 key tiles per barrier processed sequentially (dqseq2, 150 VGPR) and dK/dV with 2 query steps per barrier (dkvsq2, 168 VGPR + 4 spill) , forward with 3 key tiles per barrier (fnt3, 168 VGPR, 3 waves) vs the defaults
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3af
for v in dqseq2 dkvsq2 fnt3; do DLION_LIB=$PWD/variants/_dlion_C_$v.so timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r3af/tests_$v.log 2>&1 || { tail -30 gpurun_out/r3af/tests_$v.log; exit 1; }; echo "$v $(tail -1 gpurun_out/r3af/tests_$v.log)"; done
for rep in 1 2 3; do
for v in default dqseq2 dkvsq2 fnt3; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  echo "== $v"; DLION_LIB=$lib DLION_BENCH_OURS_ONLY=1 timeout -k 10 120 python tools/bench_attention.py 20 1024 12 64 0.1 2>&1 | grep -v amdgpu.ids || exit 1
done
done | tee gpurun_out/r3af/attn_ab.txt
for v in default dqseq2 dkvsq2 fnt3 default dqseq2 dkvsq2 fnt3; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 200 python bench.py --steps 12 --warmup 3 > gpurun_out/r3af/bench_$v.json 2> gpurun_out/r3af/bench_$v.err || { tail -20 gpurun_out/r3af/bench_$v.err; exit 1; }
  echo "$v $(python -c "import json;d=json.load(open('gpurun_out/r3af/bench_$v.json'));print(d['value'],d['ms_per_step'])")"
done | tee gpurun_out/r3af/bench_ab.txt
