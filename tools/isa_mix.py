"""Instruction-class mix of a kernel's inner loops (LLVM 'Loop' blocks) from a
hipcc -S listing: python tools/isa_mix.py <file.s> <mangled-name-substring>..."""
import collections
import re
import sys


def loop_mix(text: str, sub: str):
    names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", text, re.M) if sub in m.group(1)]
    out = {}
    for name in names:
        i = text.index(name + ":")
        j = text.index(".Lfunc_end", i)
        c = collections.Counter()
        inloop = False
        for ln in text[i:j].split("\n"):
            t = ln.strip()
            if re.match(r"^\.LBB\d+_\d+:", t) or t.startswith("; %bb"):
                inloop = "Loop" in t
                continue
            if not inloop or not t or t.startswith((".", ";")):
                continue
            op = t.split()[0]
            k = ("mfma" if op.startswith("v_mfma") else "valu" if op.startswith("v_") else
                 "nop" if op.startswith("s_nop") else "wait" if op.startswith("s_waitcnt") else
                 "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else
                 "vmem" if op.startswith(("global", "buffer")) else op)
            c[k] += 1
        out[name] = c
    return out


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    for sub in sys.argv[2:]:
        for name, c in loop_mix(text, sub).items():
            print(name[:70], dict(c), "valu/mfma %.1f" % (c["valu"] / max(1, c["mfma"])))
