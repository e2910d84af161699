# PMC counters of the own TN vs NT GEMM kernels (kernel-trace only, one group per pass).
# Summary -> gpurun_out/pmc_gemm/summary.txt
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
rm -rf gpurun_out/pmc_gemm; mkdir -p gpurun_out/pmc_gemm
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  PYTHONPATH=. timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_gemm -o pmc$i --pmc $grp \
    -- python3 tools/gemm_pmc_driver.py > gpurun_out/pmc_gemm/log$i.txt 2>&1 || { tail -5 gpurun_out/pmc_gemm/log$i.txt; exit 1; }
done
python3 - > gpurun_out/pmc_gemm/summary.txt <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmc_gemm/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "gemm_tn_kernel" in k: k = "TN"
        elif "gemm_nt_kernel" in k: k = "NT"
        else: continue
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"   {c:28s} {sum(v) / len(v):14.4g}  (n={len(v)})")
PY
cat gpurun_out/pmc_gemm/summary.txt
