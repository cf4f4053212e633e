"""Host checks of the decoder-head convolution plumbing (no GPU): the flat row-shift weight-gradient algebra
of kernels._conv3_wgrad and the GEMM forms of the kernel==stride transposed conv and the 1x1 conv, against
torch's own fp32 convolutions (the MONAI-1.3 get_conv_layer semantics: padding (k - s + 1) // 2)."""
import pytest
import torch
import torch.nn.functional as F

from long_context_biomedical_imaging_amd import decoders, kernels


@pytest.mark.parametrize("B,S,Cin,Cout", [(1, (5, 6, 7), 4, 3), (2, (3, 4, 2), 2, 5), (2, (1, 6, 9), 3, 2)])
def test_conv3_wgrad_row_shift(B, S, Cin, Cout):
    torch.manual_seed(0)
    nd = 3 if S[0] > 1 else 2
    shp = S if nd == 3 else S[1:]
    x = torch.randn(B, Cin, *shp, dtype=torch.float64)
    dy = torch.randn(B, Cout, *shp, dtype=torch.float64)
    ref = (torch.nn.grad.conv3d_weight if nd == 3 else torch.nn.grad.conv2d_weight)(
        x, (Cout, Cin) + (3,) * nd, dy, padding=1)
    x_cl = (x.unsqueeze(2) if nd == 2 else x).permute(0, 2, 3, 4, 1).contiguous()
    dy_cl = (dy.unsqueeze(2) if nd == 2 else dy).permute(0, 2, 3, 4, 1).contiguous()
    dw = kernels._conv3_wgrad(x_cl, dy_cl, 3 if nd == 3 else 1)
    assert dw.shape == ref.shape
    assert torch.allclose(dw.double(), ref, atol=1e-4, rtol=1e-4)


def test_gemm_forms_match_torch_convs():
    torch.manual_seed(0)
    x = torch.randn(2, 8, 3, 4, 5)
    for ct in (torch.nn.ConvTranspose3d(8, 6, 2, 2, bias=True), torch.nn.ConvTranspose3d(8, 6, (1, 2, 2), (1, 2, 2))):
        assert torch.allclose(ct(x), decoders._up_gemm(x, ct.weight, ct.bias, ct.kernel_size), atol=1e-5)
    x2 = torch.randn(2, 8, 5, 7)
    for ct in (torch.nn.ConvTranspose2d(8, 6, 2, 2, bias=False), torch.nn.ConvTranspose2d(8, 6, 1, 1, bias=False)):
        assert torch.allclose(ct(x2), decoders._up_gemm(x2, ct.weight, None, ct.kernel_size), atol=1e-5)
    c = torch.nn.Conv3d(8, 6, 1, 1, bias=True)
    assert torch.allclose(c(x), decoders._pointwise(x, c.weight, c.bias), atol=1e-5)


def test_decoder_conv_selection_keeps_parameters():
    """Same parameter names/shapes/seeded init as the nn.Conv layers they replace (state_dict drop-in)."""
    torch.manual_seed(3)
    w = decoders._conv(3, 96, 96, 3, 1)                                 # MONAI Convolution: the layer under .conv
    assert isinstance(w, decoders.Convolution) and list(w.state_dict().keys()) == ["conv.weight"]
    a = w.conv
    torch.manual_seed(3)
    b = torch.nn.Conv3d(96, 96, 3, 1, padding=1, bias=False)
    assert isinstance(a, decoders.Conv3x3) and a.state_dict().keys() == b.state_dict().keys()
    assert torch.equal(a.weight, b.weight)
    assert isinstance(decoders._conv_layer(3, 192, 96, 1, 1), decoders.Conv1x1)
    assert isinstance(decoders._conv_layer(3, 96, 96, (2, 2, 2), (2, 2, 2), transposed=True), decoders.ConvUp)
    assert isinstance(decoders._conv_layer(2, 64, 32, 3, 1), decoders.Conv3x3_2d)
    assert type(decoders._conv_layer(3, 4, 2, 3, 1)) is torch.nn.Conv3d      # Cout % 32 != 0: torch conv
    with pytest.raises(RuntimeError):
        a(torch.randn(1, 96, 4, 4, 4))                                  # no CPU path for the HIP conv
