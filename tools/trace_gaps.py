"""GPU idle gaps in a torch.profiler chrome trace and what the host was doing
during each: the runtime calls (hipMemcpy*, *Synchronize, ...) and the CPU ops
that overlap the gap.  usage: python tools/trace_gaps.py trace.json [min_gap_us]"""
import json
import sys
from collections import Counter


def main():
    tr = json.load(open(sys.argv[1]))
    min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
    skip = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0  # fraction of kernels to skip (start-up)
    ev = [e for e in tr["traceEvents"] if e.get("ph") == "X"]
    kern = sorted((e["ts"], e["ts"] + e["dur"], e["name"]) for e in ev if e.get("cat") in ("kernel", "gpu_memcpy", "gpu_memset"))
    rt = [(e["ts"], e["ts"] + e["dur"], e["name"]) for e in ev if e.get("cat") == "cuda_runtime"]
    cpu = [(e["ts"], e["ts"] + e["dur"], e["name"]) for e in ev if e.get("cat") in ("cpu_op", "user_annotation", "python_function")]
    kern = kern[int(len(kern) * skip):]
    busy_end = kern[0][1]
    gaps = []
    for s, e, n in kern[1:]:
        if s - busy_end > min_gap:
            gaps.append((busy_end, s, n))
        busy_end = max(busy_end, e)
    wall = kern[-1][1] - kern[0][0]
    tot = sum(b - a for a, b, _ in gaps)
    print(f"wall {wall / 1e3:.1f} ms, {len(gaps)} gaps > {min_gap} us totalling {tot / 1e3:.2f} ms")
    long_rt = Counter()
    for a, b, nxt in sorted(gaps, key=lambda g: g[0] - g[1])[:25]:
        rts = [(n, round(min(e, b) - max(s, a))) for s, e, n in rt if s < b and e > a and (min(e, b) - max(s, a)) > 20]
        ops = [(n, round(e - s)) for s, e, n in cpu if s < b and e > a and e - s > 50][:6]
        print(f"gap {b - a:8.0f} us before {nxt[:50]}")
        for n, d in rts[:5]:
            print(f"     rt  {d:7d} us {n}")
            long_rt[n] += d
        for n, d in ops:
            print(f"     cpu {d:7d} us {n[:90]}")
    print("runtime calls overlapping the top gaps:", long_rt.most_common(8))


if __name__ == "__main__":
    main()
