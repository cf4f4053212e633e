"""Split-partial sums on HIP (round 6): lci_sum_splits (the Linear / LayerNorm weight-gradient partials, summed by
torch's reduce kernel before) and lci_conv3_wgrad_sum (the decoder conv weight gradient's partials summed and permuted
to PyTorch's Conv weight layout in one pass). Against float64 sums of the same partials: within f32 rounding of an
in-order sum; two splits bitwise (one addition); one split is the partial itself.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ns,shape", [(1, (384, 384)), (2, (1536, 384)), (16, (1536, 384)), (7, (2, 384)),
                                      (3, (13,)), (40, (96, 8))])
def test_sum_splits(ns, shape):
    from long_context_biomedical_imaging_amd import kernels
    g = torch.Generator(device="cuda").manual_seed(ns)
    part = torch.randn(ns, *shape, device="cuda", generator=g)
    out = kernels.sum_splits(part)
    assert out.shape == shape
    if ns <= 2:
        assert torch.equal(out, part.sum(0))
    ref = part.double().sum(0)
    bound = part.double().abs().sum(0) * ns * 2.0 ** -24 + 1e-30
    assert ((out.double() - ref).abs() <= bound).all()


@pytest.mark.parametrize("ns,T,Cout,Cp,Cin", [(1, 27, 96, 96, 96), (5, 27, 192, 96, 70), (2, 9, 64, 128, 128),
                                               (9, 27, 32, 32, 1)])
def test_conv3_wgrad_sum(ns, T, Cout, Cp, Cin):
    from long_context_biomedical_imaging_amd import _lib
    g = torch.Generator(device="cuda").manual_seed(T + Cout)
    part = torch.randn(ns, T, Cout, Cp, device="cuda", generator=g)
    out = torch.empty(Cout, Cin, T, device="cuda")
    _lib.call("lci_conv3_wgrad_sum", part.data_ptr(), out.data_ptr(), ns, T, Cout, Cp, Cin, _lib.stream_of(part))
    ref = part.double().sum(0)[..., :Cin].permute(1, 2, 0)
    bound = part.double().abs().sum(0)[..., :Cin].permute(1, 2, 0) * ns * 2.0 ** -24 + 1e-30
    assert ((out.double() - ref).abs() <= bound).all()
    if ns <= 2:
        assert torch.equal(out, part.sum(0)[..., :Cin].permute(1, 2, 0))
