# MLP aux stream stored with sc1 (DLION_GEMM_AUX_SC1=1: the line leaves L2): GEMM tests of the
# variant, epilogue timing at the up-projection shape, same-box bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4r; mkdir -p $O
DLION_LIB=variants/_dlion_C_sc1.so timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_dgelu_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in distributed_lion_pytorch_amd/_dlion_C.so variants/_dlion_C_sc1.so; do
  echo "== $lib" >> $O/epi.txt
  DLION_LIB=$lib timeout -k 10 120 python -u tools/bench_gemm_epi.py 20480 3072 768 2>&1 | grep -v amdgpu.ids | grep -v "^    P " >> $O/epi.txt || exit 1
done
cat $O/epi.txt
bash tools/ab_bench.sh "" "DLION_LIB=variants/_dlion_C_sc1.so" 3 --steps 10 --warmup 3 | tee $O/ab.txt || exit 1
