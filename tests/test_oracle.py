"""CPU tests of the pure-PyTorch oracle: codec layout, vote rules, local Lion,
and bit-parity with the reference implementation when it is mounted."""
import importlib.util
import os
import sys

import pytest
import torch

from distributed_lion_pytorch_amd import Lion
from distributed_lion_pytorch_amd.ops import reference as ref

REF_PATH = "/root/reference/distributed_lion.py"


def load_reference():
    if not os.path.exists(REF_PATH):
        pytest.skip("reference not mounted")
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("_ref_distributed_lion", REF_PATH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("n", [1, 7, 8, 13, 1024, 2049])
def test_pack_roundtrip(n):
    g = torch.Generator().manual_seed(n)
    bits = torch.rand(n, generator=g) > 0.5
    packed = ref.pack_bits(bits)
    assert packed.dtype == torch.uint8 and packed.numel() == (n + 7) // 8
    assert torch.equal(ref.unpack_bits(packed, n), bits)


def test_pack_layout_matches_reference_encoding():
    # reference: view(-1, 8) << arange(8) summed -> element 8q+j is bit j of value q
    bits = torch.rand(64, generator=torch.Generator().manual_seed(1)) > 0.5
    expect = (bits.view(-1, 8).long() << torch.arange(8)).sum(-1)
    assert torch.equal(ref.pack_bits(bits).long(), expect)


def test_majority_tie_negative_like_torch_mode():
    a = torch.tensor([True, False, True, False])
    b = torch.tensor([False, True, True, False])
    mode = torch.mode(torch.stack([a, b]), dim=0).values.bool()
    assert torch.equal(ref.majority_vote([a, b]), mode)
    assert torch.equal(ref.majority_vote([a, b], tie=ref.TIE_POSITIVE), a | b)


def test_vote_delta_rules():
    planes = torch.tensor([[1, 1, 0, 0], [1, 0, 0, 1], [1, 0, 1, 1], [0, 1, 0, 1]], dtype=torch.bool)
    alive = torch.ones(4, dtype=torch.uint8)
    # counts: 3, 2, 1, 3 over W=4
    assert ref.vote_delta(planes, alive).tolist() == [1, -1, -1, 1]
    assert ref.vote_delta(planes, alive, tie=ref.TIE_ZERO).tolist() == [1, 0, -1, 1]
    assert ref.vote_delta(planes, alive, tie=ref.TIE_POSITIVE).tolist() == [1, 1, -1, 1]
    assert ref.vote_delta(planes, alive, mode=ref.VOTE_AVERAGE).tolist() == [0.5, 0.0, -0.5, 0.5]
    # drop rank 3: counts over 3 live voters 3, 1, 1, 2
    alive[3] = 0
    assert ref.vote_delta(planes, alive).tolist() == [1, -1, -1, 1]
    assert ref.vote_delta(planes, torch.zeros(4, dtype=torch.uint8)).tolist() == [0, 0, 0, 0]


def test_vote_reduce_bits_matches_delta():
    g = torch.Generator().manual_seed(3)
    planes = torch.rand(5, 300, generator=g) > 0.5
    alive = torch.tensor([1, 1, 0, 1, 1], dtype=torch.uint8)
    for tie in (ref.TIE_NEGATIVE, ref.TIE_ZERO, ref.TIE_POSITIVE):
        pos, neg = ref.vote_reduce_bits(planes, alive, tie)
        assert torch.equal(ref.prevoted_delta(pos, neg), ref.vote_delta(planes, alive, tie=tie))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_update_fn_bit_parity_with_reference(dtype):
    R = load_reference()
    g = torch.Generator().manual_seed(0)
    for shape in [(7,), (33, 17), (768,)]:
        p0 = torch.randn(shape, generator=g).to(dtype)
        gr = torch.randn(shape, generator=g).to(dtype)
        m0 = torch.randn(shape, generator=g).to(dtype) * 0.1
        a, am = p0.clone(), m0.clone()
        b, bm = p0.clone(), m0.clone()
        R.update_fn(a, gr, am, 1e-3, 0.1, 0.9, 0.99)
        ref.update_fn(b, gr, bm, 1e-3, 0.1, 0.9, 0.99)
        assert torch.equal(a, b) and torch.equal(am, bm)


def test_lion_matches_reference_single_process():
    R = load_reference()
    torch.manual_seed(0)
    net_a = torch.nn.Sequential(torch.nn.Linear(20, 31), torch.nn.Tanh(), torch.nn.Linear(31, 5)).bfloat16()
    net_b = torch.nn.Sequential(torch.nn.Linear(20, 31), torch.nn.Tanh(), torch.nn.Linear(31, 5)).bfloat16()
    net_b.load_state_dict(net_a.state_dict())
    oa = R.Lion(net_a.parameters(), lr=3e-3, weight_decay=0.05)
    ob = Lion(net_b.parameters(), lr=3e-3, weight_decay=0.05)
    for step in range(4):
        x = torch.randn(8, 20).bfloat16()
        for net, opt in ((net_a, oa), (net_b, ob)):
            opt.zero_grad()
            net(x).float().pow(2).mean().backward()
            opt.step()
    for pa, pb in zip(net_a.parameters(), net_b.parameters()):
        assert torch.equal(pa, pb)
    sa, sb = oa.state_dict(), ob.state_dict()
    assert sa["param_groups"][0].keys() == sb["param_groups"][0].keys()
    for k in sa["state"]:
        assert sa["state"][k].keys() == sb["state"][k].keys() == {"exp_avg"}
        assert torch.equal(sa["state"][k]["exp_avg"], sb["state"][k]["exp_avg"])


def test_lion_state_dict_roundtrip_and_groups():
    torch.manual_seed(1)
    net = torch.nn.Linear(10, 10)
    opt = Lion([{"params": [net.weight], "lr": 1e-2}, {"params": [net.bias], "weight_decay": 0.5}], lr=1e-3)
    net(torch.randn(3, 10)).sum().backward()
    opt.step()
    sd = opt.state_dict()
    assert [g["lr"] for g in sd["param_groups"]] == [1e-2, 1e-3]
    assert "max_grad_norm" not in sd["param_groups"][0]
    net2 = torch.nn.Linear(10, 10)
    net2.load_state_dict(net.state_dict())
    opt2 = Lion([{"params": [net2.weight], "lr": 1e-2}, {"params": [net2.bias], "weight_decay": 0.5}], lr=1e-3)
    opt2.load_state_dict(sd)
    g = torch.randn(3, 10)
    for n, o in ((net, opt), (net2, opt2)):
        o.zero_grad()
        n(g).sum().backward()
        o.step()
    assert torch.equal(net.weight, net2.weight) and torch.equal(net.bias, net2.bias)


def test_lion_validates_args():
    p = [torch.nn.Parameter(torch.zeros(3))]
    with pytest.raises(ValueError):
        Lion(p, lr=0.0)
    with pytest.raises(ValueError):
        Lion(p, betas=(1.5, 0.9))
    with pytest.raises(ValueError):
        Lion(p, tie_break="coin")
    with pytest.raises(ValueError):
        Lion(p, exchange="carrier-pigeon")


def test_stochastic_single_process_is_not_a_noop():
    # reference D3: W == 1 with max_grad_norm returned the function, no update
    p = torch.nn.Parameter(torch.ones(16))
    opt = Lion([p], lr=0.1, max_grad_norm=1.0)
    p.grad = torch.ones(16)
    opt.step()
    assert torch.allclose(p.detach(), torch.full((16,), 0.9))


def test_stochastic_bits_probability_clamped():
    # reference D4: bernoulli would throw for |raw| > r
    gr = torch.full((1000,), 100.0)
    m = torch.zeros(1000)
    bits = ref.stochastic_bits(gr, m, 0.9, max_grad_norm=1.0)
    assert bits.all()
    bits = ref.stochastic_bits(-gr, m, 0.9, max_grad_norm=1.0)
    assert not bits.any()


def test_lion_clip_grad_norm_cpu_matches_torch():
    """CPU (torch executor): Lion.clip_grad_norm_ is torch's clip_grad_norm_
    over the optimizer's gradients (in place), then step() as usual."""
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(n)) for n in (5, 300, 64)]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for p, q in zip(ps, qs):
        p.grad = torch.randn_like(p) * 3
        q.grad = p.grad.clone()
    a, b = Lion(ps, lr=1e-2, weight_decay=0.1), Lion(qs, lr=1e-2, weight_decay=0.1)
    na = a.clip_grad_norm_(1.0)
    nb = torch.nn.utils.clip_grad_norm_(qs, 1.0)
    torch.testing.assert_close(na, nb)
    a.step()
    b.step()
    for p, q in zip(ps, qs):
        assert torch.equal(p, q)
