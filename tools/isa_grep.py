"""Print the memory / barrier / MFMA skeleton of one kernel from a hipcc -S
listing: python tools/isa_grep.py <file.s> <mangled-name-substring> [pattern,...]."""
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    pats = sys.argv[3].split(",") if len(sys.argv) > 3 else [
        "global_load", "vmcnt", "s_barrier", "ds_write", "Loop Header", "m0", "v_mfma", "scratch_"]
    s = open(path).read()
    for line in s.split("\n"):
        if name in line and line.split() and line.split()[0].endswith(":") and not line.startswith((".", "\t")):
            start = s.index(line)
            break
    else:
        raise SystemExit(f"{name} not found")
    end = s.index(".Lfunc_end", start)
    body = s[start:end].split("\n")
    print(body[0])
    for k, l in enumerate(body):
        if any(p in l for p in pats):
            print(f"  {k:5d} {l.strip()[:80]}")


if __name__ == "__main__":
    main()
