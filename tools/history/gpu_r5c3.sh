# round-5 GPU call 3: full GPU suite (incl. the torchrun 2-rank run_clm test), bench, elastic
# steady-cost A/B on the 2-rank rehearsal, Llama-3-8B rocprof summary
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5c3; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/gpu_tests.log | head -30; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-240
timeout -k 10 900 python tools/r5/elastic_ab.py 3 $O/elastic_ab.jsonl || exit 1
bash tools/gpu_prof_llama3.sh || exit 1
timeout -k 10 300 python tools/r5/bench_gemm_stagger.py > $O/gemm_stagger.txt 2>&1 || { tail -20 $O/gemm_stagger.txt; exit 1; }
cat $O/gemm_stagger.txt
