# Lion kernel A/B: default build vs variant B (K2 non-temporal p stores, K4 grid cap 65536); bf16 copy reference
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3m
for rep in 1 2; do
for v in default lionB; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  for m in gpt2 llama3; do
    echo "== $v $m"
    DLION_LIB=$lib timeout -k 10 300 python tools/bench_lion.py $m 8 || exit 1
  done
done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r3m/lion_ab.txt
