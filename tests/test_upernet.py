"""UperNet2D / UperNet3D heads (seg_heads.py:18-277) against golden vectors the reference produced on CPU
(tools/gen_golden.py:upernet: training-mode BatchNorm, PSP dropout set to 0, Swin-like and ViT-like feature
lists, seeded cotangent). CPU: construction gives the reference's state_dict keys, shapes and seeded init.
GPU: forward and input/weight gradients; the 3x3 convs run bf16 MFMA (HIP conv3), the 1x1 convs f32 GEMMs:
rel-L2 <= 3e-2 on the output, <= GRAD_TOL on gradients (bf16 conv operands and outputs, as under the
reference's autocast, propagated through three BatchNorm backward passes)."""
import pytest
import torch

from golden_util import Golden, cotangents, rel_err
from long_context_biomedical_imaging_amd import decoders

GRAD_TOL = 0.12
CASES = [("upernet2d_swin", 2, "Swin", 11), ("upernet2d_vit", 2, "ViT", 12),
         ("upernet3d_swin", 3, "Swin", 13), ("upernet3d_vit", 3, "ViT", 14)]


class _Cfg:
    def __init__(self, encoder_name, S, patch):
        self.encoder_name = encoder_name
        self.time, self.height, self.width = S
        self.ViT = type("V", (), {"patch_size": patch})()


def _build(name, nd, enc, seed):
    g = Golden(name)
    feats = [g.t(f"in/f{i}") for i in range(len([k for k in g.z.files if k.startswith("in/f")]))]
    S = tuple(feats[0].shape[2:])
    if enc == "Swin":
        chans = [f.shape[1] for f in feats]
        patch = None
    else:
        chans = [1] + [feats[1].shape[-1]] * 13
        patch = (2, 4, 4) if nd == 3 else (1, 4, 4)
    torch.manual_seed(seed)
    cls = decoders.UperNet3D if nd == 3 else decoders.UperNet2D
    return g, feats, cls(_Cfg(enc, S, patch), chans, 3)


@pytest.mark.parametrize("name,nd,enc,seed", CASES)
def test_upernet_structure_and_init(name, nd, enc, seed):
    g, _, m = _build(name, nd, enc, seed)
    sd, ref = m.state_dict(), g.sd()
    assert list(sd.keys()) == list(ref.keys())
    for k in sd:
        assert sd[k].shape == ref[k].shape, k
        assert torch.equal(sd[k].float(), ref[k].float()), k      # seed-identical initialisation


def _run(m, feats, idx, cot, hip, amp):
    decoders.HIP_CONV_2D = decoders.HIP_CONV_3D = hip
    try:
        m.zero_grad(set_to_none=True)
        ins = [f.cuda().requires_grad_(i in idx) for i, f in enumerate(feats)]
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = m(list(ins))
        (out.float() * cot.cuda()).sum().backward()
        params = dict(m.named_parameters())
        res = {"out": out.detach().float()}
        res.update({f"f{i}": ins[i].grad for i in idx})
        res.update({p: params[p].grad for p in PARAMS})
        return res
    finally:
        decoders.HIP_CONV_2D = decoders.HIP_CONV_3D = True


PARAMS = ("head.weight", "FPN.conv_fusion.0.weight", "FPN.smooth_conv.0.weight", "PPN.bottleneck.0.weight",
          "PPN.stages.0.1.weight")


@pytest.mark.gpu
@pytest.mark.parametrize("name,nd,enc,seed", CASES)
def test_upernet_vs_reference(name, nd, enc, seed):
    """(a) the module through torch's fp32 convolutions matches the reference's fp32 CPU vectors tightly (pins the
    head's structure: pyramid, shared smoothing conv, padding-1 bottleneck, interpolation modes); (b) the product
    path (HIP bf16 convs under autocast) is within 2x of the error of torch's own bf16 autocast path on the same
    module (the reference trains under autocast), and within 3e-2 on the output. The factor 2 covers the
    noise-dominated quantities: gradients through the pyramid's bin-1 BatchNorm (2 values per channel) carry
    10-30 % bf16 error on either path, so two independent bf16 evaluations differ by that much."""
    g, feats, m = _build(name, nd, enc, seed)
    m.load_state_dict(g.sd())
    m = m.cuda().train()
    m.PPN.bottleneck[3].p = 0.0
    idx = [c % len(feats) for c in m.upernet_feature_channels]
    ref = {"out": g.t("out/0")}
    ref.update({f"f{i}": g.t(f"grad/f{i}") for i in idx})
    ref.update({p: g.t(f"grad/{p}") for p in PARAMS})
    cot = cotangents([ref["out"]])[0]
    fp32 = _run(m, feats, idx, cot, hip=False, amp=False)
    e32 = {k: rel_err(v, ref[k]) for k, v in fp32.items()}
    assert max(e32.values()) < 2e-3, e32
    tbf = {k: rel_err(v, ref[k]) for k, v in _run(m, feats, idx, cot, hip=False, amp=True).items()}
    hip = {k: rel_err(v, ref[k]) for k, v in _run(m, feats, idx, cot, hip=True, amp=True).items()}
    print(name, "torch-bf16", {k: round(v, 4) for k, v in tbf.items()}, "hip", {k: round(v, 4) for k, v in hip.items()})
    assert hip["out"] < 3e-2
    for k in hip:
        # the bin-1 stage's weight gradient runs through a BatchNorm over 2 values per channel: pure bf16 noise on
        # both paths (17-35 % error), where any change of summation order (e.g. the channels-last head) moves it
        factor = 2.5 if k == "PPN.stages.0.1.weight" else 2.0
        assert hip[k] <= max(factor * tbf[k], 2e-2), (k, hip[k], tbf[k])
