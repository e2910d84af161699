"""In-tree build of the gfx950 HIP extension (``_dlion_C.so``).

Explicit ``hipcc`` invocations -- no hipify pass, no CUDA sources, no JIT cache
under ``~/.cache`` -- so that the built shared object lives next to the package
and travels with the repository snapshot to the GPU box.  Incremental: a
source is recompiled when it, any header in ``csrc/`` or the flag set changes.

Usage: ``python -m distributed_lion_pytorch_amd._build [-v] [--force]``.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
CSRC = PKG_DIR / "csrc"
BUILD_DIR = PKG_DIR.parent / "build" / "dlion_C"
LIB_NAME = "_dlion_C.so"
LIB_PATH = PKG_DIR / LIB_NAME
ARCH = os.environ.get("DLION_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cand = Path(rocm) / "bin" / "hipcc"
    if cand.exists():
        return str(cand)
    found = shutil.which("hipcc")
    if not found:
        raise RuntimeError("hipcc not found: the dlion extension needs ROCm (set ROCM_PATH)")
    return found


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    lib = root / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _flags():
    inc, _, abi = _torch_paths()
    common = [
        "-O3",
        "-fPIC",
        "-std=c++17",
        f"--offload-arch={ARCH}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        "-DTORCH_EXTENSION_NAME=_dlion_C",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        f"-I{CSRC}",
        f"-I{sysconfig.get_paths()['include']}",
    ] + [f"-I{p}" for p in inc]
    return common


# per-source extras: the attention kernels keep MFMA accumulators in arch VGPRs
# (no v_accvgpr_read/write round trips around the softmax VALU work; measured
# 48 accvgpr reads + 32 writes + 64 moves per forward tile without it), and are
# built without SLP vectorisation: hipcc packed adjacent fp32 multiplies / FMAs
# of the dS and exponent math into v_pk_mul_f32 / v_pk_fma_f32, which issue
# slower than two plain ops beside MFMAs (dQ 88 -> 86 us at the GPT-2 shape)
EXTRA_FLAGS = {"attention.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form", "-fno-slp-vectorize"]}


def _sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _digest(src: Path, flags) -> str:
    h = hashlib.sha256()
    h.update(" ".join(flags).encode())
    h.update(src.read_bytes())
    for hdr in sorted(CSRC.glob("*.h")):
        h.update(hdr.read_bytes())
    return h.hexdigest()[:16]


def _compile(src: Path, flags, verbose: bool, force: bool, bdir: Path = BUILD_DIR) -> Path:
    obj = bdir / (src.name + ".o")
    stamp = bdir / (src.name + ".sha")
    flags = flags + EXTRA_FLAGS.get(src.name, [])
    dig = _digest(src, flags)
    if not force and obj.exists() and stamp.exists() and stamp.read_text() == dig:
        return obj
    lang = ["-x", "hip"] if src.suffix == ".hip" else []
    cmd = [_hipcc()] + lang + flags + ["-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stdout}\n{r.stderr}")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    stamp.write_text(dig)
    return obj


def build(verbose: bool = False, force: bool = False, defines=(), out: Path | None = None, flags_extra=()) -> Path:
    """Compile every HIP/C++ source in csrc/ for gfx950 and link _dlion_C.so.

    ``defines`` (``NAME=VALUE`` strings), ``flags_extra`` (compiler flags)
    and ``out`` build a variant of the extension (tuning macros, e.g.
    ``DLION_DKV_KREG128=0``) into its own object directory and shared
    object, loadable with ``DLION_LIB=<out>``."""
    out = Path(out) if out else LIB_PATH
    bdir = BUILD_DIR
    flags = _flags() + [f"-D{d}" for d in defines] + list(flags_extra)
    if defines or flags_extra or out != LIB_PATH:
        key = " ".join(list(defines) + list(flags_extra))
        bdir = BUILD_DIR.parent / ("dlion_C-" + hashlib.sha256(key.encode()).hexdigest()[:8])
    bdir.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "8"))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, verbose, force, bdir), srcs))
    _, lib, _ = _torch_paths()
    newest = max(o.stat().st_mtime for o in objs)
    if not force and out.exists() and out.stat().st_mtime >= newest:
        return out
    tmp = out.with_suffix(".so.tmp")
    cmd = (
        [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}"]
        + [str(o) for o in objs]
        + [f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lhipblaslt", f"-Wl,-rpath,{lib}", "-o", str(tmp)]
    )
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--define", "-D", action="append", default=[], help="NAME=VALUE macro for a variant build")
    ap.add_argument("--flag", action="append", default=[], help="extra compiler flag for a variant build")
    ap.add_argument("--out", default=None, help="shared object path for a variant build")
    a = ap.parse_args()
    print(build(verbose=a.v, force=a.force, defines=tuple(a.define), out=a.out, flags_extra=tuple(a.flag)))
