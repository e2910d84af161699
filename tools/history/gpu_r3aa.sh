# rocprof kernel stats of the GPT-2 bench: default (NT GEMM epilogue stores) vs ntoff -- which kernels the hints speed up
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aa
for v in default ntoff; do
  lib=""; [ $v != default ] && lib=$PWD/variants/_dlion_C_$v.so
  DLION_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3aa/prof_$v -o prof -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/r3aa/bench_$v.log 2>&1 || { tail -20 gpurun_out/r3aa/bench_$v.log; exit 1; }
  f=$(find gpurun_out/r3aa/prof_$v -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 56 40 > gpurun_out/r3aa/summary_$v.txt
  head -16 gpurun_out/r3aa/summary_$v.txt | cut -c1-150
done
