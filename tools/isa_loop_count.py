"""Instruction mix of a kernel's main loop from a hipcc -S listing:
python tools/isa_loop_count.py <file.s> <mangled-name-substring>.  The loop
region is taken from the first block tagged 'in Loop' to the last one."""
import collections
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    s = open(path).read()
    start = next(i for i, l in enumerate(s.split("\n")) if name in l and l.split() and l.split()[0].endswith(":"))
    lines = s.split("\n")[start:]
    lines = lines[:next(i for i, l in enumerate(lines) if l.startswith(".Lfunc_end"))]
    idx = [i for i, l in enumerate(lines) if "in Loop" in l or "Loop Header" in l]
    lo = idx[0]
    # last loop block: find the block after the last 'in Loop' label, stop at next non-loop label
    hi = len(lines)
    for i in range(idx[-1] + 1, len(lines)):
        if lines[i].startswith(".LBB") and "in Loop" not in lines[i] and "Loop Header" not in lines[i]:
            hi = i
            break
    c = collections.Counter()
    for l in lines[lo:hi]:
        t = l.strip().split()
        if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
            c[t[0]] += 1
    valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
    mfma = sum(v for k, v in c.items() if "mfma" in k)
    print(f"loop lines {lo}-{hi}: VALU {valu}  MFMA {mfma}  s_nop {c['s_nop']}")
    for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 25):
        print(f"  {v:4d} {k}")


if __name__ == "__main__":
    main()
