"""Fused Hyena implicit filter (kernels.hyena_filter, csrc/hyena_filter.hip) vs the module path.

The reference computes Filter.filter(L) (hyena.py:190-199) with torch ops under bf16 autocast; the same Filter
module with LCI_FUSED_FILTER=0 runs exactly those ops here and is the parity reference. Both round every Linear
output to bf16, so they differ only by accumulation order (and the hardware sin / cos), which flips an
occasional bf16 rounding: tolerance rel-L2 <= 1e-2 on k and <= 3e-2 on every parameter gradient (the fused
weight / bias gradients are f32, without the bf16 rounding of autocast's GEMM output, as kernels._Linear).
The fused k is no further from an fp32 (no autocast) module run than the autocast module path is.
"""
import pytest
import torch

from golden_util import rel_err

pytestmark = pytest.mark.gpu


def _filter(E, Lmax, w, shift, seed):
    from long_context_biomedical_imaging_amd import hyena
    torch.manual_seed(seed)
    f = hyena.Filter(64, emb_dim=E, order=64, seq_len=Lmax, w=w, shift=shift)
    return f.cuda()


def _run(f, L, G, fused, monkeypatch):
    monkeypatch.setenv("LCI_FUSED_FILTER", "1" if fused else "0")
    f.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        assert f.fused_filter_ok(L) == fused
        k = f.filter_k(L)
    assert k.shape == (64, L) and k.dtype == torch.float32
    (k * G).sum().backward()
    grads = {n: p.grad.detach().clone() for n, p in f.named_parameters() if p.grad is not None}
    return k.detach(), grads


@pytest.mark.parametrize("E,Lmax,L,w,shift", [
    (3, 4096, 4096, 1, 0.0),      # the reference default (emb_dim 3, w = 1)
    (3, 70000, 66001, 1, 0.0),    # ragged length < seq_len (z / t are sliced), several persistent tiles
    (5, 1000, 77, 10, 0.5),       # emb_dim 5, sharper sin, shifted modulation, L < one tile
])
def test_filter_fused_vs_module(E, Lmax, L, w, shift, monkeypatch):
    f = _filter(E, Lmax, w, shift, seed=11 + E)
    G = torch.randn(64, L, device="cuda", generator=torch.Generator("cuda").manual_seed(5))
    k_ref, g_ref = _run(f, L, G, False, monkeypatch)
    k, g = _run(f, L, G, True, monkeypatch)
    assert torch.isfinite(k).all()
    assert rel_err(k, k_ref) < 1e-2
    assert set(g) == set(g_ref)
    for n in g_ref:
        assert g[n].shape == g_ref[n].shape, n
        assert rel_err(g[n], g_ref[n]) < 3e-2, (n, rel_err(g[n], g_ref[n]))
    # positions past L receive no gradient
    if L < Lmax:
        assert g["pos_emb.z"][:, L:].abs().max().item() == 0.0
    # the fused path is no further from the f32 module (no autocast) than the reference's own autocast path
    # (at w = 10 both are ~20% away: bf16-rounded pre-activations times a sharp sin)
    monkeypatch.setenv("LCI_FUSED_FILTER", "0")
    with torch.no_grad():
        k32 = f.filter(L)[0].transpose(0, 1)
    assert rel_err(k, k32) < 1.25 * rel_err(k_ref, k32) + 1e-3
    if w == 1:
        assert rel_err(k, k32) < 2e-2


def test_filter_fused_deterministic(monkeypatch):
    f = _filter(3, 8192, 1, 0.0, seed=3)
    G = torch.randn(64, 8192, device="cuda")
    k1, g1 = _run(f, 8192, G, True, monkeypatch)
    k2, g2 = _run(f, 8192, G, True, monkeypatch)
    assert torch.equal(k1, k2)
    for n in g1:
        assert torch.equal(g1[n], g2[n]), n


def test_hyena_operator_uses_fused_filter(monkeypatch):
    """HyenaOperator under autocast: the fused filter path vs LCI_FUSED_FILTER=0 end to end."""
    from long_context_biomedical_imaging_amd import hyena
    torch.manual_seed(2)
    m = hyena.HyenaOperator(d_model=128, l_max=5000, filter_order=64, num_heads=2, short_filter_order=3).cuda()
    x = torch.randn(2, 5000, 128, device="cuda")
    outs = []
    for fused in (False, True):
        monkeypatch.setenv("LCI_FUSED_FILTER", "1" if fused else "0")
        m.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert m.filter_fn.fused_filter_ok(5000) == fused
            y = m(xi)
        y.float().pow(2).mean().backward()
        outs.append((y.detach().float(), xi.grad.clone(), m.filter_fn.implicit_filter[2].weight.grad.clone()))
    (y0, dx0, dw0), (y1, dx1, dw1) = outs
    assert rel_err(y1, y0) < 1e-2
    assert rel_err(dx1, dx0) < 2e-2
    assert rel_err(dw1, dw0) < 3e-2
