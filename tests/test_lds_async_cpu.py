"""Race check for the inline-asm LDS reads (CPU: hipcc cross-compiles).

csrc/gemm_tn.hip issues its ``ds_read_b64_tr_b16`` fragment reads through
inline asm (the builtin made the compiler drain the LDS-DMA pipeline).  The
compiler's wait-count pass does not know that such an asm statement leaves a
load in flight: if a read's destination registers became dead before the
explicit ``s_waitcnt lgkmcnt(0)`` that precedes the MFMAs, the register
allocator could hand them to another value and the late LDS return would
overwrite it.  A round-5 diagnostic build that dropped the MFMAs did exactly
that -- a staging address landed in a pending read's registers and the kernel
faulted with an illegal address.  This test compiles the TN kernel and walks
its ISA: no instruction may write a register of an inline tr read that is
still outstanding (no ``lgkmcnt(0)`` in between)."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

CSRC = Path(__file__).resolve().parent.parent / "distributed_lion_pytorch_amd" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _vregs(tok: str) -> set:
    tok = tok.rstrip(",")
    m = re.match(r"^v\[(\d+):(\d+)\]$", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"^v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def clobbers(asm_text: str, kernel_pattern: str):
    """[(kernel, line, instruction)] writes to registers of outstanding tr reads."""
    found, cur, pending = [], None, {}
    for i, line in enumerate(asm_text.splitlines()):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur, pending = m.group(1), {}
            continue
        if cur is None or not re.search(kernel_pattern, cur):
            continue
        t = line.strip()
        if not t or t.startswith((".", ";")):
            continue
        parts = t.replace(",", " ").split()
        op = parts[0]
        if op == "s_waitcnt" and "lgkmcnt(0)" in t:
            pending = {}
        elif op == "ds_read_b64_tr_b16":
            for r in _vregs(parts[1]):
                pending[r] = i
        elif pending and len(parts) > 1 and op.startswith(("v_", "ds_read", "global_load", "buffer_load")):
            hit = _vregs(parts[1]) & set(pending)
            if hit:
                found.append((cur, i, t))
                for r in hit:
                    pending.pop(r)
    return found


def test_checker_flags_a_dead_tr_read():
    asm = "\n".join([
        "_ZN5dlion6kernelEv:",
        "\tds_read_b64_tr_b16 v[4:5], v1",
        "\tv_lshl_add_u64 v[4:5], v[2:3], 1, s[2:3]",
        "\ts_waitcnt lgkmcnt(0)",
        "\tds_read_b64_tr_b16 v[6:7], v1",
        "\ts_waitcnt lgkmcnt(0)",
        "\tv_mov_b32_e32 v6, 0",
    ])
    bad = clobbers(asm, "kernel")
    assert len(bad) == 1 and "v_lshl_add_u64" in bad[0][2]


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")
def test_tn_kernel_inline_tr_reads_are_never_clobbered(tmp_path):
    out = tmp_path / "gemm_tn.s"
    cmd = [HIPCC, "-O3", "--offload-arch=gfx950", "-std=c++17", f"-I{CSRC}", "--cuda-device-only", "-S",
           str(CSRC / "gemm_tn.hip"), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    text = out.read_text()
    assert text.count("ds_read_b64_tr_b16") >= 96, "the TN main loop's transposed reads are missing"
    bad = clobbers(text, r"gemm_tn_kernel")
    assert not bad, f"registers of in-flight inline LDS reads overwritten: {bad[:5]}"
