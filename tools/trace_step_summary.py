"""Per-kernel summary of ONE steady training step from a rocprofv3 kernel
trace (csv): the kernels between the last two optimizer-step boundaries (the
first kernel of a Lion apply group), so the first step's hipBLASLt solution
search and the init kernels are excluded.

python tools/trace_step_summary.py <kernel_trace.csv> [top] [boundary-substring]
"""
import collections
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
marker = sys.argv[3] if len(sys.argv) > 3 else "lion_local_kernel"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
# boundaries: first marker kernel of each consecutive run of marker kernels
bounds, prev = [], False
for i, r in enumerate(rows):
    m = marker in r["Kernel_Name"]
    if m and not prev:
        bounds.append(i)
    prev = m
if len(bounds) < 2:
    sys.exit(f"need >= 2 step boundaries ({marker}), found {len(bounds)}")
a, b = bounds[-2], bounds[-1]
# the step = kernels after the previous optimizer group up to and incl. this one
while b < len(rows) and marker in rows[b]["Kernel_Name"]:
    b += 1
while a < len(rows) and marker in rows[a]["Kernel_Name"]:
    a += 1
step = rows[a:b]
wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
agg = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[r["Kernel_Name"]][0] += 1
    agg[r["Kernel_Name"]][1] += d
busy = sum(v[1] for v in agg.values()) / 1e3
print(f"one steady step: {len(step)} kernels, wall {wall:.1f} ms, kernel time {busy:.1f} ms "
      f"({100 * busy / wall:.1f} % busy)")
for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{100 * us / 1e3 / busy:6.2f}% {us / 1e3:8.3f}ms calls={n:5d} avg={us / n:9.1f}us  {name[:100]}")
