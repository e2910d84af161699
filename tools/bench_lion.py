"""Lion optimizer kernels against the HBM roofline (one MI355X, bf16 params):
K0 local update, K1 encode (momentum + 1-bit pack), K2 vote+apply over W
fake voter planes, K4 shard vote (a2a), over the GPT-2 small and the
Llama-3-8B parameter sets (shapes only, random values).  Bytes per param are
the kernels' compulsory traffic; prints us, GB/s and % of 6.3 TB/s.

  python tools/bench_lion.py [gpt2|llama3] [W]
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from distributed_lion_pytorch_amd.ops import hip  # noqa: E402
from distributed_lion_pytorch_amd.ops import reference as ref  # noqa: E402
from distributed_lion_pytorch_amd.optim.executors import HParams, HipExecutor  # noqa: E402
from distributed_lion_pytorch_amd.optim.plan import FlatPlan  # noqa: E402

HBM = 6.3e12


def shapes(model):
    if model == "gpt2":
        C, L, V = 768, 12, 50257
        per = [(3 * C, C), (3 * C,), (C, C), (C,), (4 * C, C), (4 * C,), (C, 4 * C), (C,), (C,), (C,), (C,), (C,)]
        return [(V, C), (1024, C)] + per * L + [(C,), (C,)]
    C, L, V, F, KV = 4096, 32, 128256, 14336, 1024
    per = [(C, C), (KV, C), (KV, C), (C, C), (F, C), (F, C), (C, F), (C,), (C,)]
    return [(V, C)] + per * L + [(C,), (V, C)]


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "gpt2"
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda")
    ps = [torch.randn(s, device=dev, dtype=torch.bfloat16) for s in shapes(model)]
    gs = [torch.randn_like(p) for p in ps]
    ms = [torch.randn_like(p) * 0.1 for p in ps]
    n = sum(p.numel() for p in ps)
    plan = FlatPlan([(p, 0) for p in ps], world=W, device=dev)
    hx = HipExecutor(plan)
    meta = plan.meta(gs, ms)
    hp = HParams(lr=1e-5, wd=0.1, beta1=0.9, beta2=0.99)
    bits = torch.zeros(plan.total_bytes, dtype=torch.uint8, device=dev)
    planes = torch.randint(0, 256, (W * plan.total_bytes,), dtype=torch.uint8, device=dev)
    alive = torch.ones(W, dtype=torch.uint8, device=dev)
    voted = torch.zeros(plan.total_bytes // W, dtype=torch.uint8, device=dev)

    def local():
        for b in plan.buckets:
            hx.local(meta, b, hp)

    def encode():
        for b in plan.buckets:
            hx.encode(meta, b, bits[b.byte_off:b.byte_off + b.nbytes], hp)

    def apply():
        for b in plan.buckets:
            pl = planes[W * b.byte_off: W * (b.byte_off + b.nbytes)]
            hx.apply(meta, b, pl, b.nbytes, alive, ref.VOTE_MAJORITY, ref.TIE_NEGATIVE, None, hp)

    def apply_prevoted():  # a2a (default exchange): one voted plane after the shard vote + all-gather
        for b in plan.buckets:
            hx.apply(meta, b, planes[b.byte_off: b.byte_off + b.nbytes], b.nbytes, alive, ref.VOTE_PREVOTED,
                     ref.TIE_NEGATIVE, None, hp)

    def vote_reduce():  # a2a: this rank's shard of every bucket, W planes of it
        for b in plan.buckets:
            sh = b.nbytes // W
            hx.vote_reduce(planes[W * b.byte_off: W * b.byte_off + W * sh], sh, alive, ref.TIE_NEGATIVE,
                           voted[b.byte_off // W: b.byte_off // W + sh], None)

    src = torch.empty(n, dtype=torch.bfloat16, device=dev)
    dst = torch.empty_like(src)

    def copy():  # practical roofline of a 50/50 read/write stream (what K2's p traffic is)
        dst.copy_(src)

    # compulsory bytes per param: p r+w, g r, m r+w (local); g r, m r+w, 1 bit (encode);
    # p r+w + W bits (apply); W bits read + 1 bit written per shard param (vote_reduce, 1/W of params)
    cases = {"K0 local": (local, 10.0), "K1 encode": (encode, 6.0 + 1 / 8),
             f"K2 vote+apply W={W}": (apply, 4.0 + W / 8), "K2 prevoted apply": (apply_prevoted, 4.0 + 1 / 8), f"K4 shard vote W={W}": (vote_reduce, (W + 1) / 8 / W),
             "bf16 copy (reference)": (copy, 4.0)}
    print(f"{model}: {n / 1e6:.1f}M params, {len(ps)} tensors, {len(plan.buckets)} buckets", flush=True)
    res = {k: [] for k in cases}
    for _ in range(3):
        for k, (f, _) in cases.items():
            res[k].append(timed(f))
    for k, (f, bpp) in cases.items():
        us = statistics.median(res[k])
        gbs = bpp * n / us / 1e3
        print(f"  {k:22s} {us:9.1f} us  {gbs:7.0f} GB/s  {100 * gbs * 1e9 / HBM:5.1f}% of 6.3 TB/s", flush=True)


if __name__ == "__main__":
    main()
