"""Per-kernel mean time (us) of the attention kernels from rocprofv3 kernel_stats
CSVs: python tools/attn_kernel_times.py <label>=<stats.csv> ..."""
import csv
import sys

for arg in sys.argv[1:]:
    label, path = arg.split("=", 1)
    rows = {}
    for r in csv.DictReader(open(path)):
        name = r["Name"]
        if "attn_" not in name:
            continue
        short = name.split("(")[0].replace("void dlion::", "")
        rows[short] = float(r["AverageNs"]) / 1000.0
    print(f"{label:10s} " + "  ".join(f"{k} {v:7.1f}" for k, v in sorted(rows.items())))
