"""Compare learning curves written by ``bench.py --data markov --loss_log``:
first / last loss, 5-step moving averages and the per-step |difference| of
two runs (native vs --impl reference), per world size.

  python tools/curve_summary.py <label=native.jsonl> <label=reference.jsonl> [...]   (pairs, in order)
"""
import json
import sys


def load(path):
    return [json.loads(ln)["loss"] for ln in open(path) if ln.startswith("{")]


def mavg(xs, i, k=5):
    w = xs[max(0, i - k + 1):i + 1]
    return sum(w) / len(w)


args = sys.argv[1:]
for a, b in zip(args[0::2], args[1::2]):
    la, pa = a.split("=", 1)
    lb, pb = b.split("=", 1)
    xa, xb = load(pa), load(pb)
    n = min(len(xa), len(xb))
    marks = [m for m in (9, 19, 29, 39, n - 1) if m < n]
    d = [abs(xa[i] - xb[i]) for i in range(n)]
    print(f"{la} vs {lb}: steps {n}; loss {xa[0]:.3f} -> {xa[n - 1]:.3f} ({la}) vs {xb[0]:.3f} -> {xb[n - 1]:.3f} ({lb})")
    print(f"    5-step moving average at steps {[m + 1 for m in marks]}: {la} {[round(mavg(xa, m), 3) for m in marks]}")
    print(f"    {'':>{len('5-step moving average at steps ' + str([m + 1 for m in marks]))}}  {lb} {[round(mavg(xb, m), 3) for m in marks]}")
    print(f"    |diff| mean {sum(d) / n:.4f}, max {max(d):.4f}")
