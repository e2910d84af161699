# SQ counters of the attention kernels at the GPT-2 shape (one 8-counter pass + one instruction-mix pass)
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
OUT=gpurun_out/pmc_attn_sq; rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT -o pmc$i --pmc $grp -- python3 tools/bench_attention.py --ours-only "$@" > $OUT/log$i.txt 2>&1 || exit 1
done
python3 - "$OUT" > $OUT/summary.txt <<'PY'
import csv, glob, collections, sys
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(lambda: collections.defaultdict(int))
for f in sorted(glob.glob(out + "/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "dlion::attn" not in k:
            continue
        k = k.split("(")[0].replace("void ", "")
        c = row["Counter_Name"]
        agg[k][c] += float(row["Counter_Value"])
        n[k][c] += 1
for k, d in agg.items():
    print(k)
    avg = {c: d[c] / max(1, n[k][c]) for c in d}
    for c in sorted(avg):
        print(f"   {c:28s} {avg[c]:14.4g}")
    if avg.get("SQ_WAVE_CYCLES"):
        w = avg["SQ_WAVE_CYCLES"]
        print(f"   wait_any/wave_cycles {avg.get('SQ_WAIT_ANY', 0) / w:.3f}  wait_inst/wave {avg.get('SQ_WAIT_INST_ANY', 0) / w:.3f}"
              f"  active_inst/wave {avg.get('SQ_ACTIVE_INST_ANY', 0) / w:.3f}")
    if avg.get("SQ_BUSY_CYCLES"):
        print(f"   mfma_busy/busy {avg.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / avg['SQ_BUSY_CYCLES']:.3f}")
    if avg.get("SQ_INSTS_MFMA"):
        print(f"   VALU/MFMA insts = {avg.get('SQ_INSTS_VALU', 0) / avg['SQ_INSTS_MFMA']:.1f}")
PY
cat $OUT/summary.txt
