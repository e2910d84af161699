"""Summarize a rocprofv3 kernel_stats.csv per micro-batch:
python tools/prof_summary.py <csv> [micro_batches] [top] [steady]
steady: drop hipBLASLt rows that ran less than once per micro-batch (the
first step's algorithm search / candidate timing), recompute the total."""
import csv
import sys

path = sys.argv[1]
mb = int(sys.argv[2]) if len(sys.argv) > 2 else 24
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
if len(sys.argv) > 4 and sys.argv[4] == "steady":
    rows = [r for r in rows if not (r["Name"].startswith("Cijk_") and int(r["Calls"]) < 0.95 * mb)]
    t = sum(float(r["TotalDurationNs"]) for r in rows)
    for r in rows:
        r["Percentage"] = str(100.0 * float(r["TotalDurationNs"]) / t)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.1f} ms = {tot / 1e6 / mb:.2f} ms per micro-batch")
for r in rows[:top]:
    print(f"{float(r['Percentage']):6.2f}% {float(r['TotalDurationNs']) / 1e6 / mb:7.3f}ms/mb "
          f"calls/mb={int(r['Calls']) / mb:6.1f} avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:90]}")
