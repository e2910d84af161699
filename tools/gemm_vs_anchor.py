"""GEMM roles of the GPT-2 and Llama-3-8B steps as % of the on-box anchor
(best bf16 GEMM at 8192^3 measured in the same call, tools/gemm_anchor.py):
per role the candidate the step runs (the fastest of the per-shape timed
pick's candidates; the fused MLP epilogues always run the own NT kernel), its
PF/s, % of the anchor, and the time per step lost against the anchor rate.

  python tools/gemm_vs_anchor.py <anchor.txt> <gpt2_shapes.txt> <llama_shapes.jsonl> <llama_wgrad.jsonl>
"""
import json
import re
import sys

anchor_txt, gpt2_txt, llama_js, wgrad_js = sys.argv[1:5]
anchor = float(re.search(r"ANCHOR .*= ([0-9.]+) PF/s", open(anchor_txt).read()).group(1))
rows = []  # (model, role, M, N, K, kernel, pfs, calls per optimizer step)
GA = 8  # GPT-2 bench: 8 micro-batches per step, 12 layers
for ln in open(gpt2_txt):
    if "|" not in ln or ln.startswith("role"):
        continue
    parts = [p.strip() for p in ln.split("|")]
    role, M, N, K = parts[0], int(parts[1]), int(parts[2]), int(parts[3])
    cands = {}
    for c in parts[4:]:
        m = re.match(r"(.+?):\s+([0-9.]+) us\s+([0-9.]+) PF/s", c)
        if m:
            cands[m.group(1)] = (float(m.group(2)), float(m.group(3)))
    if "EPI" in ln:  # the fused epilogue runs the own kernel; hipBLASLt has no such epilogue
        name = [k for k in cands if "EPI" in k][0]
    else:
        name = min(cands, key=lambda k: cands[k][0])
    us, pfs = cands[name]
    window = "window" in role
    per_step = (1 if window else GA) * (1 if "LM head" in role else 12)
    rows.append(("gpt2", role, M, N, K, name, us, pfs, per_step))
for ln in open(llama_js):
    if not ln.startswith("{"):
        continue
    d = json.loads(ln)
    c = {k[:-3]: v for k, v in d.items() if k.endswith("_us") and k != "transpose_us"}
    if d["shape"].endswith("dgrad"):  # the NT forms pay the per-step W^T copy (trainable weight)
        for k in list(c):
            if k.endswith("_nt"):
                c[k] += d["transpose_us"]
    name = min(c, key=c.get)
    fl = 2.0 * d["M"] * d["N"] * d["K"]
    rows.append(("llama3-8b", d["shape"], d["M"], d["N"], d["K"], name, c[name], fl / c[name] / 1e9, 32))
for ln in open(wgrad_js):
    if not ln.startswith("{"):
        continue
    d = json.loads(ln)
    c = {k[:-3]: v for k, v in d.items() if k.endswith("_us")}
    name = min(c, key=c.get)
    fl = 2.0 * d["M"] * d["R"] * d["C"]
    rows.append(("llama3-8b", d["shape"] + "_wgrad", d["M"], d["R"], d["C"], name, c[name], fl / c[name] / 1e9, 32))

print(f"# anchor (best bf16 GEMM at 8192^3 on this box, same call) = {anchor:.3f} PF/s")
print("# lost ms/step = (time - time at the anchor rate) x calls per optimizer step "
      "(GPT-2: 8 micro-batches x 12 layers; Llama-3-8B: 32 layers, M as measured)")
print(f"{'model':9s} {'role':44s} {'M':>6s} {'N':>6s} {'K':>6s}  {'kernel':26s} {'us':>9s} {'PF/s':>5s} "
      f"{'%anchor':>7s} {'lost ms/step':>12s}")
lost = []
for model, role, M, N, K, name, us, pfs, per_step in rows:
    ideal = 2.0 * M * N * K / (anchor * 1e9)
    l_ms = (us - ideal) * per_step / 1e3
    lost.append((l_ms, model, role, pfs / anchor))
    print(f"{model:9s} {role:44s} {M:6d} {N:6d} {K:6d}  {name:26s} {us:9.1f} {pfs:5.2f} {100 * pfs / anchor:6.0f}% "
          f"{l_ms:12.2f}")
print("\n# furthest below the anchor (% of anchor):")
for pct, model, role in sorted((x[3], x[1], x[2]) for x in lost)[:3]:
    print(f"#   {model} {role}: {100 * pct:.0f} %")
print("# largest time lost against the anchor rate (ms per optimizer step):")
for l_ms, model, role, pct in sorted(lost, reverse=True)[:5]:
    print(f"#   {model} {role}: {l_ms:.2f} ms ({100 * pct:.0f} %)")
