"""GPU idle time from a rocprofv3 kernel trace: wall span of the last N kernels'
window vs the union of kernel intervals, plus the largest gaps.
usage: python tools/prof_gaps.py <kernel_trace.csv> [skip_fraction]"""
import csv
import sys


def main():
    path = sys.argv[1]
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:80]))
    rows.sort()
    rows = rows[int(len(rows) * skip):]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    prev_name = ""
    for s, e, n in rows:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = n
    busy += cur_e - cur_s
    wall = rows[-1][1] - rows[0][0]
    print(f"kernels {len(rows)}  wall {wall / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {100 * (1 - busy / wall):.1f}%")
    gaps.sort(reverse=True)
    tot = sum(g for g, _, _ in gaps)
    print(f"gaps: {len(gaps)}  total {tot / 1e6:.2f} ms  >100us: {sum(1 for g in gaps if g[0] > 1e5)}")
    for g, a, b in gaps[:15]:
        print(f"  {g / 1e3:9.1f} us  after {a[:60]}  before {b[:60]}")


if __name__ == "__main__":
    main()
