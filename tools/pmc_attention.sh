# PMC counters for the attention kernels (rocprofv3 --pmc with kernel-trace only;
# one counter group per run).  Summary -> gpurun_out/pmc_attn/summary.txt
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
rm -rf gpurun_out/pmc_attn; mkdir -p gpurun_out/pmc_attn
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_attn -o pmc$i --pmc $grp \
    -- python3 tools/bench_attention.py > gpurun_out/pmc_attn/log$i.txt 2>&1 || exit 1
done
python3 - > gpurun_out/pmc_attn/summary.txt <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in sorted(glob.glob("gpurun_out/pmc_attn/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "dlion::attn" not in k:
            continue
        k = k.split("(")[0].replace("void ", "")
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        calls[k].add((f, row.get("Dispatch_Id", "")))
for k, d in agg.items():
    n = max(1, len([c for c in calls[k] if "pmc1" in c[0]]))
    print(k, "dispatches/pass", n)
    for c in sorted(d):
        print(f"   {c:28s} {d[c] / n:14.4g}")
    if d.get("SQ_INSTS_MFMA"):
        print(f"   VALU/MFMA = {d['SQ_INSTS_VALU'] / d['SQ_INSTS_MFMA']:.1f}")
PY
cat gpurun_out/pmc_attn/summary.txt
