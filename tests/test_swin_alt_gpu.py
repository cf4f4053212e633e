"""GPU parity: Swin-tiny stage with Hyena / Mamba inside the windows (WindowAttention's alternates,
backbone_swin.py:315-332 / 361-365; shift forced to 0, :674) — the configuration every reference project
script trains (projects/run_*.sh: Swin tiny, patch 2, window 4 or 8, use_hyena xor use_mamba).

tests/golden/swin_{hyena,mamba}_w{4,7,8}[_2d].npz come from the reference's own BasicLayer (fp32, CPU;
tools/gen_golden.py:swin_alt_layer): dim 96 / 3 heads (Hyena head_dim 32, Mamba Dx 48), depth 2, padded grids
(10^3 -> 14^3 at window 7, ragged pads at windows 4 and 8, 2-D grids), PatchMergingV2 on the window-7 layers.

Tolerances: fp32 modules rel-L2 <= 2e-4 on the output, <= 1e-3 on gradients (f32 FFT / scan / GEMM
reassociation); bf16 autocast (the training configuration) <= 2e-2 on outputs, <= 6e-2 on gradients, the
bounds the single-mixer autocast tests use (tests/test_mamba_gpu.py, tests/test_hyena_gpu.py).
"""
import pytest
import torch
import torch.nn.functional as F

from golden_util import Golden, cotangents, rel_err

pytestmark = pytest.mark.gpu

CASES = ["swin_hyena_w7", "swin_mamba_w7", "swin_hyena_w4", "swin_mamba_w4", "swin_hyena_w8", "swin_mamba_w8",
         "swin_mamba_w4_2d", "swin_hyena_w8_2d"]


def _layer(g):
    from long_context_biomedical_imaging_amd import backbone_swin
    hy = bool(g.scalar("cfg/hyena"))
    ws = tuple(int(v) for v in g.z["cfg/window"])
    down = backbone_swin.PatchMergingV2 if int(g.scalar("cfg/downsample")) else None
    layer = backbone_swin.BasicLayer(hy, not hy, dim=96, depth=2, num_heads=3, window_size=ws, drop_path=[0.0, 0.0],
                                     qkv_bias=True, downsample=down)
    missing, unexpected = layer.load_state_dict(g.sd(), strict=False)
    # only the Hyena positional-embedding buffers / parameter are stored as checksums (deterministic, CPU-checked)
    assert not unexpected and all(k.endswith(("pos_emb.z", "pos_emb.t")) for k in missing), (missing, unexpected)
    return layer.cuda()


def _grad_names(g):
    return [k[5:] for k in g.z.files if k.startswith("grad/") and k != "grad/in0"]


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("amp", [False, True])
def test_swin_alt_layer_vs_reference(name, amp):
    g = Golden(name)
    layer = _layer(g)
    x = g.t("in/x").cuda().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        out = layer(x)
    ref = g.t("out/0")
    assert out.shape == ref.shape
    e = rel_err(out, ref)
    assert e < (2e-2 if amp else 2e-4), f"output rel err {e:.3e}"
    out.float().backward(cotangents([ref])[0].cuda())
    e = rel_err(x.grad, g.t("grad/in0"))
    assert e < (6e-2 if amp else 1e-3), f"dx rel err {e:.3e}"
    params = dict(layer.named_parameters())
    for p in _grad_names(g):
        e = rel_err(params[p].grad, g.t(f"grad/{p}"))
        assert e < (6e-2 if amp else 1e-3), f"{p}: rel err {e:.3e}"


@pytest.mark.parametrize("B,dims,ws,dtype", [(2, (10, 10, 10), (7, 7, 7), torch.bfloat16),
                                             (1, (8, 6, 10), (4, 4, 4), torch.float32),
                                             (2, (5, 9, 40), (5, 7, 7), torch.bfloat16),   # collapsed window axis
                                             (2, (18, 14), (4, 4), torch.float32),
                                             (1, (64, 64, 64), (4, 4, 4), torch.bfloat16)])
def test_window_gather_scatter_bit_exact(B, dims, ws, dtype):
    """lci_window_gather (the Hyena / Mamba window path) against the reference op sequence, bit for bit: F.pad of
    the LayerNorm output with zeros + window_partition (backbone_swin.py:445-465) and window_reverse + crop
    (:469-487); both directions of both autograd ops (each one's adjoint is the other)."""
    from long_context_biomedical_imaging_amd import kernels
    from oracle import window as ow
    C = 96
    g = torch.Generator().manual_seed(B * 7 + sum(dims))
    x = torch.randn(B, *dims, C, generator=g).to(dtype)
    pads = [(w - s % w) % w for s, w in zip(dims, ws)]
    padarg = []
    for p in reversed(pads):
        padarg += [0, p]
    xp = F.pad(x, [0, 0] + padarg)
    ref = ow.window_partition(xp, ws)
    xc = x.cuda().requires_grad_(True)
    win = kernels.window_partition_grid(xc, ws, (0,) * len(ws))
    assert win.shape == ref.shape and torch.equal(win.cpu(), ref)
    back = kernels.window_reverse_grid(win, x.shape, ws, (0,) * len(ws))
    assert torch.equal(back.cpu(), x)
    cot = torch.randn(ref.shape, generator=g).to(dtype)
    rev = ow.window_reverse(cot, ws, [B, *xp.shape[1:-1]])
    crop = rev[tuple([slice(None)] + [slice(0, s) for s in dims])]
    win.backward(cot.cuda())
    assert torch.equal(xc.grad.cpu(), crop)
