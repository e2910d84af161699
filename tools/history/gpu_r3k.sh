# Round-3 checkpoint: full GPU suite (incl. full-size parity), Lion roofline, bench, rocprof summary, 8B dropout rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3k
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > gpurun_out/r3k/gpu_tests.log 2>&1; rc=$?
tail -4 gpurun_out/r3k/gpu_tests.log; [ $rc -eq 0 ] || grep -E "^FAILED|^ERROR" gpurun_out/r3k/gpu_tests.log | head -20
grep -q "Timeout\|Fatal Python" gpurun_out/r3k/gpu_tests.log && exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/parity_full.json"))
for k, v in d.items():
    print(k, "max_loss_diff", round(v["max_loss_diff"], 5), "worst_grad_rel", round(v["worst_grad_rel"], 4))
PY
timeout -k 10 200 python tools/bench_lion.py gpt2 8 > gpurun_out/r3k/lion_gpt2.txt 2>&1 && timeout -k 10 300 python tools/bench_lion.py llama3 8 > gpurun_out/r3k/lion_llama3.txt 2>&1 || exit 1
cat gpurun_out/r3k/lion_gpt2.txt gpurun_out/r3k/lion_llama3.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r3k/bench.json 2> gpurun_out/r3k/bench.err || { tail -20 gpurun_out/r3k/bench.err; exit 1; }
cut -c1-300 gpurun_out/r3k/bench.json
bash tools/profile_bench.sh r3 > /dev/null 2>&1 || exit 1
f=$(find gpurun_out/prof_r3 -name "*kernel_stats.csv" | head -1); python tools/prof_summary.py $f 24 40 > gpurun_out/r3k/gpt2_summary.txt; head -12 gpurun_out/r3k/gpt2_summary.txt | cut -c1-150
bash tools/gpu_stress_8b.sh
