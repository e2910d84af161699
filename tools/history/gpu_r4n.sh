# Lion K2 paired apply with 4 chunks per block (DLION_K2_CPB=4) vs 2: kernel tests of the variant,
# then the roofline tool on both builds, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4n; mkdir -p $O
DLION_LIB=variants/_dlion_C_cpb4.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for lib in distributed_lion_pytorch_amd/_dlion_C.so variants/_dlion_C_cpb4.so; do
    echo "== $lib" >> $O/lion_ab.txt
    DLION_LIB=$lib timeout -k 10 120 python tools/bench_lion.py gpt2 8 2>&1 | grep -v amdgpu.ids >> $O/lion_ab.txt || exit 1
  done
done
cat $O/lion_ab.txt
