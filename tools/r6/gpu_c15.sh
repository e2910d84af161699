# r6 call 15: HBM fetch of the own TN kernel at the GPT-2 window shapes (is the LM-head
# weight gradient re-reading its output-gradient slab per column tile?)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c15; mkdir -p $O
PYTHONPATH=. timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O -o fetch --pmc FETCH_SIZE \
  -- python3 tools/tn_fetch_driver.py > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
PYTHONPATH=. timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O -o hits --pmc TCC_HIT_sum TCC_MISS_sum \
  -- python3 tools/tn_fetch_driver.py > $O/log2.txt 2>&1 || { tail -5 $O/log2.txt; exit 1; }
python3 - <<'PY' | tee $O/summary.txt
import csv, glob
for f in sorted(glob.glob("gpurun_out/r6c15/**/*counter_collection.csv", recursive=True)):
    print("#", f.split("/")[-1])
    for row in csv.DictReader(open(f)):
        if "gemm_tn_kernel" in row["Kernel_Name"]:
            print(f"  dispatch {row['Dispatch_Id']:>4s} grid {row.get('Grid_Size','?'):>8s} {row['Counter_Name']:14s} {float(row['Counter_Value']):16.4g}")
PY
grep -h "ideal" $O/log.txt
