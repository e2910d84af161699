# PMC counters for the attention fwd kernel (rocprofv3 --pmc, kernel-trace only).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_attn
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o pmc1 \
  --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -- python3 tools/bench_attention.py > gpurun_out/pmc_attn/log1.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o pmc2 \
  --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
  -- python3 tools/bench_attention.py > gpurun_out/pmc_attn/log2.txt 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_attn/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"][:60]
        if "attn" not in k and "bwd" not in k: continue
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[k] += 1
    print(f)
    for k, d in agg.items():
        print(" ", k, {c: f"{v:.3g}" for c, v in d.items()})
PY
