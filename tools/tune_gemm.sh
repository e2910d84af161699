# PyTorch TunableOp sweep of every hipBLASLt/rocBLAS GEMM solution for the bench's
# GEMM shapes; writes the winners to distributed_lion_pytorch_amd/tuned/ (shipped in-tree).
# Usage: bash tools/tune_gemm.sh [bench args]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tune
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tune/tunableop_results.csv
timeout -k 10 900 python bench.py --steps 2 --warmup 1 "$@" > gpurun_out/tune/tune.log 2>&1 || { echo TUNE FAIL; tail -30 gpurun_out/tune/tune.log; exit 1; }
tail -1 gpurun_out/tune/tune.log
ls -la gpurun_out/tune/
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
f=$(ls gpurun_out/tune/tunableop_results*.csv | head -1)
export PYTORCH_TUNABLEOP_FILENAME=$f
timeout -k 10 400 python bench.py --steps 5 --warmup 2 "$@" > gpurun_out/tune/bench_tuned.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/tune/bench_tuned.log; exit 1; }
tail -1 gpurun_out/tune/bench_tuned.log
