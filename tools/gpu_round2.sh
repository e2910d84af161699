# full GPU tests + GPT-2 bench + Llama-2-7B SFT bench on one MI355X
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_native.log 2>&1 || { echo BENCH FAIL; tail -30 gpurun_out/bench_native.log; exit 1; }
tail -1 gpurun_out/bench_native.log
timeout -k 10 600 python bench.py --task sft --steps 4 --warmup 2 > gpurun_out/bench_sft.log 2>&1 || { echo SFT FAIL; tail -30 gpurun_out/bench_sft.log; exit 1; }
tail -1 gpurun_out/bench_sft.log
