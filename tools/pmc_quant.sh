# HBM traffic of the 4-bit expansion kernels (plain and transposed) at the Llama-2-7B gate/up shape:
# TCC FETCH_SIZE / WRITE_SIZE (KB) and time per call, kernel-trace only.  -> gpurun_out/pmc_quant/summary.txt
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
rm -rf gpurun_out/pmc_quant; mkdir -p gpurun_out/pmc_quant
cat > gpurun_out/pmc_quant/drive.py <<'PY'
import torch
from distributed_lion_pytorch_amd.ops import hip
from distributed_lion_pytorch_amd.ops.quant import code_tensor, quantize_4bit
dev = torch.device("cuda", 0)
code = code_tensor("nf4", dev)
w = torch.randn(22016, 4096, device=dev, dtype=torch.bfloat16)
q, a = quantize_4bit(w, code)
out = torch.empty_like(w)
outt = torch.empty(4096, 22016, device=dev, dtype=torch.bfloat16)
for _ in range(5):
    hip.ops().dequant4_(q, a, code, out)
    hip.ops().dequant4_t_(q, a, code, outt)
torch.cuda.synchronize()
PY
i=0
for grp in FETCH_SIZE WRITE_SIZE; do  # one pass each: FETCH_SIZE uses 3 of the 4 TCC counters, WRITE_SIZE 2
  i=$((i+1))
  PYTHONPATH=. timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_quant -o pmc$i --pmc $grp \
    -- python3 gpurun_out/pmc_quant/drive.py > gpurun_out/pmc_quant/log$i.txt 2>&1 || { tail -5 gpurun_out/pmc_quant/log$i.txt; exit 1; }
done
python3 - > gpurun_out/pmc_quant/summary.txt <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmc_quant/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "dequant4_t" in k: k = "dequant4_t (transposed)"
        elif "dequant4" in k: k = "dequant4"
        else: continue
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
ideal = 22016 * 4096 * (0.5 + 2 + 4 / 64) / 1024
print(f"ideal traffic per call: {ideal / 1024:.1f} MB (0.5 B/param in, 2 B/param out, fp32 absmax)")
for k, c in agg.items():
    print(k, {n: f"{sum(v) / len(v) / 1024:.1f} MB" for n, v in c.items()})
PY
cat gpurun_out/pmc_quant/summary.txt
