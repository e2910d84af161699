"""Instruction mix of a kernel's inner loops from hipcc -S output.
Usage: python tools/isa_loop_stats.py <file.s> <mangled-kernel-name-substring>"""
import collections
import re
import sys

text = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", text, re.M) if sys.argv[2] in m.group(1)]
for name in names:
    i = text.index(name + ":")
    j = text.index(".Lfunc_end", i)
    body = text[i:j].split("\n")
    # blocks annotated as loop members by LLVM
    in_loop = False
    ops = collections.Counter()
    total = collections.Counter()
    for ln in body:
        t = ln.strip()
        if re.match(r"^\.LBB\d+_\d+:", t) or t.startswith("; %bb"):
            in_loop = "Loop" in t
            continue
        if not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        total[op] += 1
        if in_loop:
            ops[op] += 1
    print(name, "static total", sum(total.values()), "in-loop", sum(ops.values()))
    for k, v in ops.most_common(25):
        print(f"   {v:4d} {k}")
