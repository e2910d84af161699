# LDS bank conflicts / MFMA busy for the attention kernels at the Llama (D=128)
# and GPT-2 (D=64) shapes.  One counter pass per run (rocprofv3 --pmc, kernel trace only).
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
out=gpurun_out/pmc_attn_lds; rm -rf $out; mkdir -p $out
C="${PMC_COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA}"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $out -o llama --pmc $C \
  -- python3 tools/bench_attention.py 4 2048 32 128 0.0 > $out/llama.txt 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $out -o gpt2 --pmc $C \
  -- python3 tools/bench_attention.py 20 1024 12 64 0.1 > $out/gpt2.txt 2>&1 || exit 1
python3 - <<'PY' > $out/summary.txt
import csv, glob, collections
for tag in ("llama", "gpt2"):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"gpurun_out/pmc_attn_lds/**/{tag}*counter_collection.csv", recursive=True):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if "dlion::attn" not in k:
                continue
            per[(k.split("(")[0].replace("void ", ""), row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        for (k, _), d in per.items():
            for c, v in d.items():
                agg[k][c].append(v)
    print("==", tag)
    for k, d in agg.items():
        print(k)
        for c in sorted(d):
            v = sorted(d[c]); print(f"   {c:28s} {v[len(v)//2]:14.4g}")
        m = {c: sorted(v)[len(v)//2] for c, v in d.items()}
        if m.get("SQ_INSTS_LDS"):
            print(f"   bank-conflict cycles / LDS-active cycles = {m['SQ_LDS_BANK_CONFLICT'] / max(1, m['SQ_LDS_IDX_ACTIVE']):.3f}")
PY
cat $out/summary.txt
