"""Exposed elastic-mode cost on the 2-rank rehearsal (2 gloo ranks sharing
one MI355X, GPT-2 bench config): bench.py with and without --elastic_timeout,
interleaved rounds; prints the slowest rank's exposed `exchange` phase (the
compute stream's wait on the vote exchange + the shard vote), `optimizer` and
the step time.  python tools/r5/elastic_ab.py [rounds] [out.jsonl]"""
import json
import subprocess
import sys

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
out = open(sys.argv[2], "w") if len(sys.argv) > 2 else None
base = [sys.executable, "bench.py", "--gpus", "2", "--backend", "gloo", "--steps", "8", "--warmup", "2"]
for r in range(rounds):
    for arm, extra in (("plain", []), ("elastic", ["--elastic_timeout", "60"])):
        p = subprocess.run(base + extra, capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            print(p.stdout[-2000:], p.stderr[-3000:])
            sys.exit(1)
        d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{"metric"')][-1])
        ph = d.get("phase_ms_per_step", {})
        rec = {"round": r, "arm": arm, "ms_per_step": d["ms_per_step"], "exchange_ms": ph.get("exchange"),
               "optimizer_ms": ph.get("optimizer"), "fwd_bwd_ms": ph.get("fwd_bwd"),
               "commits": d.get("optimizer_stats", {}).get("elastic_commits")}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
