#!/usr/bin/env python3
"""Generate tests/golden/*.npz by running the REFERENCE model code (/root/reference) on CPU.

Run only in the build container (the reference does not exist on the GPU box):
    python tools/gen_golden.py
The reference source is imported, never copied; third-party packages absent from this image are
replaced by tools/ref_standins.py (restated MONAI-1.3 / mamba-ssm-1.2.0 behaviour).

Each fixture holds data only: state_dict tensors ("sd/<key>"), inputs ("in/<name>"), outputs
("out/<name>") and gradients of a fixed random cotangent ("grad/<name>"). Large deterministic
buffers (the Hyena positional embedding, l_max=66000) are stored as checksums ("chk/<key>").
"""
from __future__ import annotations

import hashlib
import os
import types
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference/model/models"
OUT = os.path.join(REPO, "tests", "golden")

sys.path.insert(0, HERE)
import ref_standins  # noqa: E402

ref_standins.install()
sys.path.insert(0, REF)
import backbone_swin as rswin  # noqa: E402
import backbone_vit as rvit  # noqa: E402
import class_heads as rcls  # noqa: E402
import enhance_heads as renh  # noqa: E402
import hyena as rhyena  # noqa: E402
import mamba as rmamba  # noqa: E402
import seg_heads as rseg  # noqa: E402

BIG = ("filter_fn.pos_emb.z", "filter_fn.pos_emb.t")


def np32(t):
    t = t.detach()
    return t.numpy().astype(np.float32) if t.is_floating_point() else t.numpy()


def dump(name, module=None, **arrays):
    d = {}
    if module is not None:
        for k, v in module.state_dict().items():
            if any(k.endswith(b) for b in BIG):
                d[f"chk/{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item(),
                                          float(v.numel())])
            else:
                d[f"sd/{k}"] = np32(v)
    for k, v in arrays.items():
        d[k] = np32(v) if isinstance(v, torch.Tensor) else np.asarray(v)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **d)
    print(f"{path}: {os.path.getsize(path) / 1024:.0f} KiB, {len(d)} arrays")


def fwd_bwd(module, *inputs, grads=(), seed=123, **kw):
    """Run forward, then backward of sum(out * cot) with a seeded N(0,1) cotangent."""
    ins = [x.clone().requires_grad_(True) for x in inputs]
    out = module(*ins, **kw)
    outs = out if isinstance(out, (list, tuple)) else [out]
    g = torch.Generator().manual_seed(seed)
    cots = [torch.randn(o.shape, generator=g) for o in outs]
    loss = sum((o * c).sum() for o, c in zip(outs, cots))
    module.zero_grad(set_to_none=True)
    loss.backward()
    res = {}
    for i, o in enumerate(outs):
        res[f"out/{i}"] = o  # cotangent i = seeded randn (tests/golden_util.py:cotangents)
    for i, x in enumerate(ins):
        res[f"grad/in{i}"] = x.grad
    params = dict(module.named_parameters())
    for p in grads:
        res[f"grad/{p}"] = params[p].grad
    return res


# ------------------------------------------------------------------------------------------ fixtures
def sablock(name, hidden, heads, B, L, seed):
    torch.manual_seed(seed)
    m = rvit.SABlock(False, False, hidden, heads).eval()
    x = torch.randn(B, L, hidden)
    r = fwd_bwd(m, x, grads=("qkv.weight", "out_proj.weight", "out_proj.bias"))
    dump(name, m, **{"in/x": x, "cfg/heads": heads}, **r)


def vit_encoder(name, hidden, heads, mlp, layers, img, patch, B, seed, classification=False,
                use_hyena=False, use_mamba=False):
    torch.manual_seed(seed)
    m = rvit.ViT_with_alt_ops(use_hyena, use_mamba, in_channels=1, img_size=img, patch_size=patch,
                              hidden_size=hidden, mlp_dim=mlp, num_layers=layers, num_heads=heads,
                              dropout_rate=0.0, spatial_dims=2, classification=classification).eval()
    x = torch.rand(B, 1, 1, *img)
    gnames = ["patch_embedding.patch_embeddings.weight", "patch_embedding.position_embeddings",
              "blocks.0.norm1.weight"]
    if not use_hyena and not use_mamba:
        gnames.append("blocks.0.attn.qkv.weight")
    r = fwd_bwd(m, x, grads=tuple(gnames))
    r = {k: v for k, v in r.items() if not k.startswith("grad/in")}
    dump(name, m, **{"in/x": x, "cfg/heads": heads, "cfg/layers": layers}, **r)


def hyena_op(seed):
    torch.manual_seed(seed)
    m = rhyena.HyenaOperator(d_model=128, l_max=66000, filter_order=64, num_heads=2, num_blocks=1,
                             short_filter_order=5, bidrectional=True, dropout=0.0, filter_dropout=0.0,
                             activation="id").eval()
    assert m.bidirectional is False
    x = torch.randn(1, 512, 128)
    r = fwd_bwd(m, x, grads=("in_proj.weight", "filter_fn.bias", "short_filter.weight",
                             "filter_fn.implicit_filter.0.weight"))
    k = m.filter_fn.filter(512)[0].transpose(0, 1)
    dump("hyena_op", m, **{"in/x": x, "out/k": k}, **r)
    # kernel-level long conv pin: the reference fftconv_ref on random u, k, D
    g = torch.Generator().manual_seed(seed + 1)
    for L, nb in ((1000, 2), (2048, 1)):
        u = torch.randn(1, nb, 64, 1, L, generator=g)
        kk = torch.randn(64, L, generator=g) * torch.exp(-torch.linspace(0, 6, L))[None]
        D = torch.randn(1, 64, 1, generator=g)
        y = rhyena.fftconv_ref(u, kk, D, dropout_mask=None, gelu=False)
        dump(f"fftconv_L{L}", None, **{"in/u": u[:, :, :, 0], "in/k": kk, "in/D": D.reshape(64),
                                       "out/y": y[:, :, :, 0]})
    # reference behaviour beyond l_max: assert message references a missing attribute
    try:
        m(torch.randn(1, 66001, 128))
        err = "none"
    except AttributeError as e:
        err = "AttributeError:" + str(e)
    except AssertionError as e:
        err = "AssertionError:" + str(e)
    dump("hyena_lmax", None, **{"out/err": np.array(err)})


def mamba_mixer(seed):
    torch.manual_seed(seed)
    m = rmamba.MambaVisionMixer(d_model=128, d_state=8, d_conv=3, expand=1).eval()
    x = torch.randn(2, 256, 128)
    r = fwd_bwd(m, x, grads=("A_log", "D", "dt_proj.bias", "x_proj.weight", "in_proj.weight",
                             "conv1d_x.weight"))
    dump("mamba_mixer", m, **{"in/x": x}, **r)
    # kernel-level scan pin (mamba-ssm selective_scan_ref semantics, as called at mamba.py:125-134)
    g = torch.Generator().manual_seed(seed + 1)
    b, d, n, L = 2, 32, 8, 384
    u = torch.randn(b, d, L, generator=g)
    delta = torch.randn(b, d, L, generator=g) * 0.5
    A = -torch.exp(torch.randn(d, n, generator=g) * 0.5)
    Bm = torch.randn(b, n, L, generator=g)
    Cm = torch.randn(b, n, L, generator=g)
    D = torch.randn(d, generator=g)
    db = torch.randn(d, generator=g) * 0.3
    ins = [t.clone().requires_grad_(True) for t in (u, delta, A, Bm, Cm, D, db)]
    y = ref_standins.selective_scan_fn(ins[0], ins[1], ins[2], ins[3], ins[4], ins[5], z=None,
                                       delta_bias=ins[6], delta_softplus=True)
    cot = torch.randn(y.shape, generator=g)
    (y * cot).sum().backward()
    names = ["u", "delta", "A", "B", "C", "D", "delta_bias"]
    arr = {f"in/{k}": t for k, t in zip(names, (u, delta, A, Bm, Cm, D, db))}
    arr.update({f"grad/{k}": t.grad for k, t in zip(names, ins)})
    dump("selective_scan", None, **arr, **{"out/y": y, "cot/y": cot})  # scan cot kept (own generator)


def window_attention(seed):
    torch.manual_seed(seed)
    ws = (7, 7, 7)
    m = rswin.WindowAttention(False, False, 64, 2, ws, qkv_bias=True).eval()
    mask = rswin.compute_mask([7, 7, 14], ws, (3, 3, 3), "cpu")  # nW = 2
    x = torch.randn(2, 343, 64)
    r = fwd_bwd(m, x, grads=("relative_position_bias_table", "qkv.weight", "qkv.bias"), mask=mask)
    r0 = fwd_bwd(m, x, grads=("relative_position_bias_table",), mask=None)
    extra = {k.replace("out/", "out_nomask/").replace("grad/", "grad_nomask/"): v for k, v in r0.items()}
    dump("window_attn_3d", m, **{"in/x": x, "in/mask": mask}, **r, **extra)

    torch.manual_seed(seed + 1)
    m2 = rswin.WindowAttention(False, False, 64, 2, (7, 7), qkv_bias=True).eval()
    mask2 = rswin.compute_mask([14, 14], (7, 7), (3, 3), "cpu")  # nW = 4
    x2 = torch.randn(8, 49, 64)
    r2 = fwd_bwd(m2, x2, grads=("relative_position_bias_table",), mask=mask2)
    dump("window_attn_2d", m2, **{"in/x": x2, "in/mask": mask2}, **r2)


def swin_layer(seed):
    torch.manual_seed(seed)
    layer = rswin.BasicLayer(False, False, dim=64, depth=2, num_heads=2, window_size=(7, 7, 7),
                             drop_path=[0.0, 0.0], qkv_bias=True,
                             downsample=rswin.PatchMergingV2).eval()
    x = torch.randn(1, 64, 10, 10, 10)
    r = fwd_bwd(layer, x, grads=("blocks.1.attn.relative_position_bias_table",))
    dump("swin_basic_layer", layer, **{"in/x": x}, **r)


# Swin-tiny with Hyena / Mamba inside the windows: what every reference project script trains
# (projects/run_*.sh: --Swin.size tiny, patch 2, window 4 or 8, use_hyena xor use_mamba; shift forced to 0 at
# backbone_swin.py:674). Stage-1 shapes: dim 96, 3 heads (Hyena head_dim 32), Mamba d_inner 96 -> Dx 48.
SWIN_ALT = [
    # name, use_hyena, use_mamba, batch, grid, window
    ("swin_hyena_w7", True, False, 1, (10, 10, 10), (7, 7, 7)),     # pad 10 -> 14, N = 343 (configs[2] window)
    ("swin_mamba_w7", False, True, 1, (10, 10, 10), (7, 7, 7)),
    ("swin_hyena_w4", True, False, 2, (8, 6, 10), (4, 4, 4)),       # run_cmr/abct-style window 4, ragged pad
    ("swin_mamba_w4", False, True, 2, (8, 6, 10), (4, 4, 4)),
    ("swin_hyena_w8", True, False, 1, (8, 9, 12), (8, 8, 8)),       # window 8, N = 512, pad 9 -> 16, 12 -> 16
    ("swin_mamba_w8", False, True, 1, (8, 9, 12), (8, 8, 8)),
    ("swin_mamba_w4_2d", False, True, 2, (18, 14), (4, 4)),         # run_micro: 2-D, window 4, N = 16
    ("swin_hyena_w8_2d", True, False, 2, (12, 20), (8, 8)),         # run_vessel/ptx-style 2-D window 8
]


def swin_alt_layer(name, use_hyena, use_mamba, B, grid, ws, seed):
    """BasicLayer(use_hyena | use_mamba, dim 96, depth 2, 3 heads) + PatchMergingV2, fp32 CPU fwd/bwd."""
    torch.manual_seed(seed)
    down = rswin.PatchMergingV2 if name.endswith("_w7") else None   # merging pinned once per mixer (size)
    layer = rswin.BasicLayer(use_hyena, use_mamba, dim=96, depth=2, num_heads=3, window_size=ws,
                             drop_path=[0.0, 0.0], qkv_bias=True, downsample=down).eval()
    x = torch.randn(B, 96, *grid)
    if use_hyena:
        gn = ("blocks.0.attn.hyena.in_proj.weight", "blocks.1.attn.hyena.short_filter.weight",
              "blocks.0.attn.hyena.filter_fn.bias", "blocks.1.attn.hyena.filter_fn.implicit_filter.0.weight",
              "blocks.1.attn.hyena.out_proj.weight", "blocks.0.norm1.weight")
    else:
        gn = ("blocks.0.attn.mamba.in_proj.weight", "blocks.1.attn.mamba.A_log", "blocks.1.attn.mamba.D",
              "blocks.0.attn.mamba.dt_proj.bias", "blocks.1.attn.mamba.x_proj.weight",
              "blocks.0.attn.mamba.conv1d_z.weight", "blocks.1.attn.mamba.out_proj.weight", "blocks.0.norm1.weight")
    if down is not None:
        gn = gn + ("downsample.reduction.weight",)
    r = fwd_bwd(layer, x, grads=gn)
    dump(name, layer, **{"in/x": x, "cfg/window": np.array(ws), "cfg/hyena": int(use_hyena),
                         "cfg/downsample": int(down is not None)}, **r)


class _Ns:
    """The config fields custom_ViT / ViTLinear read (backbone_vit.py:45-116, class_heads.py:13-49)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class _EncDec(torch.nn.Module):
    """EncoderDecoderModel's structure (model_base.py:23-83: encoder built first, then decoder; same keys)."""

    def __init__(self, enc, dec):
        super().__init__()
        self.encoder, self.decoder = enc, dec

    def forward(self, x):
        return self.decoder(self.encoder(x))


def _vit_cls_model(size, img, patch, n_cls, **vit):
    cfg = _Ns(ViT=_Ns(size=size, patch_size=list(patch), use_hyena=False, use_mamba=False, **vit),
              time=1, height=img[0], width=img[1], task_type="class", encoder_name="ViT")
    enc, ch = rvit.custom_ViT(cfg, 1)
    dec = rcls.ViTLinear(cfg, ch, n_cls)
    return _EncDec(enc, dec)


def vit_cls_c1(seed):
    """BASELINE configs[0]: ViT-small + ViTLinear classification, 64x64 2-D, patch 16 (L = 16 + cls token).
    ViT-small's 21.7M weights are not stored: the state_dict is pinned by per-tensor checksums (this package's
    modules reproduce the seeded init bit-for-bit; tests/test_modules_cpu.py), outputs and selected gradients."""
    torch.manual_seed(seed)
    m = _vit_cls_model("small", (64, 64), (16, 16, 16), 4).eval()
    x = torch.rand(2, 1, 1, 64, 64)
    gn = ("decoder.classification_head.0.weight", "decoder.classification_head.0.bias", "encoder.cls_token",
          "encoder.patch_embedding.patch_embeddings.weight", "encoder.patch_embedding.position_embeddings",
          "encoder.norm.weight", "encoder.blocks.11.mlp.linear2.bias", "encoder.blocks.0.attn.out_proj.weight")
    r = fwd_bwd(m, x, grads=gn)
    r = {k: v for k, v in r.items() if not k.startswith("grad/in")}
    arr = {"in/x": x}
    for k, v in m.state_dict().items():
        arr[f"chk/{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item(), float(v.numel())])
    for k, v in m.named_parameters():
        arr[f"gsum/{k}"] = np.array([v.grad.double().sum().item(), v.grad.double().abs().sum().item()])
    dump("vit_cls_c1", None, **arr, **r)


def train_step_product(seed):
    """Two steps of the reference's training loop (trainer_base.py:166-182, use_amp off, iters_to_accumulate 1, no
    clipping) with its SGD (optim_base.py:90-91: momentum 0.9, lr 0.1) and CrossEntropy loss on a small ViT +
    ViTLinear (cls token) classifier, fp32 on CPU. Every weight is stored before and after, element by element."""
    torch.manual_seed(seed)
    m = _vit_cls_model("custom", (16, 16), (2, 2, 2), 3, hidden_size=128, mlp_dim=256, num_layers=2, num_heads=2)
    m.train()
    g = torch.Generator().manual_seed(seed + 1)
    xs = [torch.rand(2, 1, 1, 16, 16, generator=g) for _ in range(2)]
    ys = [torch.randint(0, 3, (2,), generator=g) for _ in range(2)]
    arr = {f"sd/{k}": v.clone() for k, v in m.state_dict().items()}
    opt = torch.optim.SGD([{"params": list(m.parameters()), "lr": 0.1, "weight_decay": 0.0}], lr=0.1, momentum=0.9,
                          weight_decay=0.0)
    loss_f = torch.nn.CrossEntropyLoss()
    for i, (x, y) in enumerate(zip(xs, ys)):
        loss = loss_f(m(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        arr[f"in/x{i}"], arr[f"in/y{i}"], arr[f"out/loss{i}"] = x, y, loss.detach()
    for k, v in m.state_dict().items():
        arr[f"post/{k}"] = v
    dump("train_step_product", None, **arr)


def train_step_adam(seed):
    """Two steps of the reference's loop (trainer_base.py:166-182) with the recipes' optimizer: Adam
    (optim_base.py:86-87, betas (beta1, beta2) = (0.9, 0.95) config defaults, lr 1e-4 as projects/run_abct.sh:36-37,
    weight decay 0), CrossEntropy, same small ViT + ViTLinear as train_step_product. Run on CPU, where the
    reference's torch.autocast(device_type='cuda') is inactive and GradScaler(enabled=True) disables itself (no CUDA):
    the fp32 step. Each step's gradients are stored too (the test weighs Adam's sign-like first updates by them)."""
    torch.manual_seed(seed)
    m = _vit_cls_model("custom", (16, 16), (2, 2, 2), 3, hidden_size=128, mlp_dim=256, num_layers=2, num_heads=2)
    m.train()
    g = torch.Generator().manual_seed(seed + 1)
    xs = [torch.rand(2, 1, 1, 16, 16, generator=g) for _ in range(2)]
    ys = [torch.randint(0, 3, (2,), generator=g) for _ in range(2)]
    arr = {f"sd/{k}": v.clone() for k, v in m.state_dict().items()}
    opt = torch.optim.Adam([{"params": list(m.parameters()), "lr": 1e-4, "weight_decay": 0.0}], lr=1e-4,
                           betas=(0.9, 0.95), weight_decay=0.0)
    loss_f = torch.nn.CrossEntropyLoss()
    for i, (x, y) in enumerate(zip(xs, ys)):
        loss = loss_f(m(x), y)
        loss.backward()
        for k, v in m.named_parameters():
            arr[f"grad{i}/{k}"] = v.grad.clone()
        opt.step()
        opt.zero_grad(set_to_none=True)
        arr[f"in/x{i}"], arr[f"in/y{i}"], arr[f"out/loss{i}"] = x, y, loss.detach()
    for k, v in m.state_dict().items():
        arr[f"post/{k}"] = v
    dump("train_step_adam", None, **arr)


def _sub(t, n=8192):
    """A deterministic strided subsample of t (at most ~n elements) and its stride: the fixture keeps big
    activations and gradients as samples (tests/test_unetr.py compares the same positions)."""
    flat = t.detach().reshape(-1)
    step = max(1, flat.numel() // n)
    return flat[::step].clone(), np.array(step)


def _unetr_run(m, ins, grad_idx, seed, small_params):
    """Forward on the input list, backward of sum(out * seeded cotangent); -> dict of outputs / gradients."""
    ins = [x.clone().requires_grad_(i in grad_idx) for i, x in enumerate(ins)]
    out = m(list(ins))
    cot = torch.randn(out.shape, generator=torch.Generator().manual_seed(123))
    m.zero_grad(set_to_none=True)
    (out * cot).sum().backward()
    arr = {}
    arr["out/0"], arr["stride/out"] = _sub(out)
    for i in grad_idx:
        arr[f"grad/in{i}"], arr[f"stride/in{i}"] = _sub(ins[i].grad)
    params = dict(m.named_parameters())
    for k, v in m.state_dict().items():
        arr[f"chk/{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item(), float(v.numel())])
    for k, v in params.items():
        arr[f"gsum/{k}"] = np.array([v.grad.double().sum().item(), v.grad.double().abs().sum().item()])
    for k in small_params:
        arr[f"grad/{k}"] = params[k].grad
    for i, x in enumerate(ins):
        arr[f"inchk/{i}"] = np.array([x.double().sum().item(), x.double().abs().sum().item()])
    return arr


def unetr_vit(name, nd, patch, S, hidden, seed):
    """The reference ViTUNETR (enhance_heads.py:187-356) on the restated MONAI-1.3 blocks, fp32 CPU, fed the input
    image, 12 hidden-state taps (3, 6, 9 read, enhance_heads.py:338-345; the others zero) and the last tokens.
    Weights come from torch.manual_seed(seed) (stored as checksums: the product module is seed-identical); inputs
    from torch.Generator().manual_seed(seed + 1), in list order (stored as checksums); out and input gradients as
    strided samples, a few small weight gradients whole, every weight gradient's sum and L1 mass."""
    torch.manual_seed(seed)
    ns = types.SimpleNamespace
    cfg = ns(no_in_channel=1, encoder_name="ViT", time=S[0], height=S[1], width=S[2],
             ViT=ns(hidden_size=hidden, patch_size=tuple(patch)))
    m = renh.ViTUNETR(cfg, None, 2).train()
    g = torch.Generator().manual_seed(seed + 1)
    L = 1
    for a, b in zip(S, patch):
        L *= a // b
    B = 2
    ins = [torch.randn(B, 1, *S, generator=g)]
    ins += [torch.randn(B, L, hidden, generator=g) if i in (3, 6, 9) else torch.zeros(B, L, hidden) for i in range(12)]
    ins.append(torch.randn(B, L, hidden, generator=g))
    arr = _unetr_run(m, ins, (0, 4, 7, 10, 13), 123,
                     ("encoder1.layer.conv1.conv.weight", "out.conv.conv.weight", "out.conv.conv.bias",
                      "encoder2.transp_conv_init.conv.weight", "decoder2.transp_conv.conv.weight"))
    arr["cfg/shape"] = np.array([nd, *patch, *S, hidden, seed])
    dump(name, None, **arr)


def unetr_swin(name, S, f0, seed):
    """The reference SwinUNETR (enhance_heads.py:30-184), 3-D, patch 2, Swin-tiny channels [f0 .. 16 f0], fed the
    input image and the five stage taps (S/2 .. S/32), fp32 CPU; stored as unetr_vit."""
    torch.manual_seed(seed)
    ns = types.SimpleNamespace
    cfg = ns(no_in_channel=1, encoder_name="Swin", time=S[0], height=S[1], width=S[2], Swin=ns(patch_size=(2, 2, 2)))
    chans = [f0 * 2 ** i for i in range(5)]
    m = renh.SwinUNETR(cfg, chans, 2).train()
    g = torch.Generator().manual_seed(seed + 1)
    B = 1
    ins = [torch.randn(B, 1, *S, generator=g)]
    ins += [torch.randn(B, c, *(s // 2 ** (i + 1) for s in S), generator=g) for i, c in enumerate(chans)]
    arr = _unetr_run(m, ins, (0, 1, 4, 5), 123,
                     ("encoder1.layer.conv1.conv.weight", "out.conv.conv.weight", "out.conv.conv.bias",
                      "decoder1.transp_conv.conv.weight"))
    arr["cfg/shape"] = np.array([3, *S, f0, seed])
    dump(name, None, **arr)


UNETR = [("unetr_vit2d_p2", 2, (1, 2, 2), (1, 32, 32), 96, 40), ("unetr_vit2d_p4", 2, (1, 4, 4), (1, 32, 32), 96, 41),
         ("unetr_vit3d_p2", 3, (2, 2, 2), (8, 16, 16), 96, 42)]


def swin_index():
    arr = {}
    ws, ss = (7, 7, 7), (3, 3, 3)
    arr["out/rp_index_3d"] = rswin.WindowAttention(False, False, 96, 3, ws).relative_position_index.numpy()
    arr["out/rp_index_2d"] = rswin.WindowAttention(False, False, 96, 3, (7, 7)).relative_position_index.numpy()
    for d in (14, 21, 35, 70):
        dims = [d, d, d]
        mask = rswin.compute_mask(dims, ws, ss, "cpu").numpy()
        nz = (mask != 0)
        assert set(np.unique(mask).tolist()) <= {0.0, -100.0}
        arr[f"out/mask_sha256_{d}"] = np.array(hashlib.sha256(np.packbits(nz).tobytes()).hexdigest())
        arr[f"out/mask_shape_{d}"] = np.array(mask.shape)
        arr[f"out/mask_nnz_{d}"] = np.array(int(nz.sum()))
        if d <= 21:
            arr[f"out/mask_bits_{d}"] = np.packbits(nz)
        # shifted partition as a permutation of voxel ids
        idx = torch.arange(d * d * d, dtype=torch.float64).reshape(1, d, d, d, 1)
        sh = torch.roll(idx, shifts=(-3, -3, -3), dims=(1, 2, 3))
        perm = rswin.window_partition(sh, ws).reshape(-1).long().numpy().astype(np.int32)
        if d <= 21:
            arr[f"out/partition_perm_{d}"] = perm
        arr[f"out/partition_sha256_{d}"] = np.array(hashlib.sha256(perm.tobytes()).hexdigest())
    for x_size in ((64, 64, 64), (5, 9, 40), (4, 4, 4)):
        w, s = rswin.get_window_size(x_size, ws, ss)
        arr[f"out/gws_{'x'.join(map(str, x_size))}"] = np.array(list(w) + list(s))
    dump("swin_index", None, **arr)


def train_step(seed):
    """One SGD step of a small ViT encoder + mean-pool linear head, MSE loss (CPU, fp32)."""
    torch.manual_seed(seed)
    enc = rvit.ViT_with_alt_ops(False, False, in_channels=1, img_size=(16, 16), patch_size=(2, 2),
                                hidden_size=128, mlp_dim=256, num_layers=2, num_heads=2, dropout_rate=0.0,
                                spatial_dims=2).eval()
    head = torch.nn.Linear(128, 3)
    x = torch.rand(2, 1, 1, 16, 16)
    y = torch.randn(2, 3)
    sd0 = {**{f"enc.{k}": v.clone() for k, v in enc.state_dict().items()},
           **{f"head.{k}": v.clone() for k, v in head.state_dict().items()}}
    params = list(enc.parameters()) + list(head.parameters())
    opt = torch.optim.SGD(params, lr=0.1)
    loss = torch.nn.functional.mse_loss(head(enc(x)[-1].mean(1)), y)
    loss.backward()
    opt.step()
    arr = {"in/x": x, "in/y": y, "out/loss": loss.detach()}
    for k, v in sd0.items():
        arr[f"sd/{k}"] = v
    post = {**{f"enc.{k}": v for k, v in enc.state_dict().items()},
            **{f"head.{k}": v for k, v in head.state_dict().items()}}
    for k, v in post.items():
        arr[f"post_sum/{k}"] = np.array([v.double().sum().item(), v.double().abs().sum().item()])
    dump("train_step", None, **arr)


class _Cfg:
    """The config fields UperNet2D/3D read (seg_heads.py:96-117, 248-269)."""

    def __init__(self, encoder_name, time, height, width, patch):
        self.encoder_name, self.time, self.height, self.width = encoder_name, time, height, width
        self.ViT = type("V", (), {"patch_size": patch})()


def upernet(name, nd, encoder, seed):
    """UperNet2D/3D (seg_heads.py:79-277) in training mode (BatchNorm batch statistics) with the PSP dropout set
    to p = 0, fed a Swin-like (5 stage taps + image) or ViT-like (13 token taps + image) feature list."""
    torch.manual_seed(seed)
    if encoder == "Swin":
        chans = [1, 8, 16, 32, 64, 128]
        S = (8, 16, 16) if nd == 3 else (1, 32, 32)
        shapes = [(2, 1) + S] + [(2, c) + tuple(max(1, s // 2 ** (i + 1)) if (nd == 3 or k > 0) else 1
                                            for k, s in enumerate(S)) for i, c in enumerate(chans[1:])]
        cfg = _Cfg("Swin", S[0], S[1], S[2], None)
    else:
        chans = [1] + [32] * 13
        S = (8, 16, 16) if nd == 3 else (1, 32, 32)
        patch = (2, 4, 4) if nd == 3 else (1, 4, 4)
        L = 1
        for s, p in zip(S, patch):
            L *= s // p
        shapes = [(2, 1) + S] + [(2, L, 32)] * 13
        cfg = _Cfg("ViT", S[0], S[1], S[2], patch)
    cls = rseg.UperNet3D if nd == 3 else rseg.UperNet2D
    m = cls(cfg, chans, 3).train()
    m.PPN.bottleneck[3].p = 0.0
    feats = [torch.randn(s) for s in shapes]
    idx = [c % len(feats) for c in m.upernet_feature_channels]
    ins = [f.clone().requires_grad_(True) if i in idx else f for i, f in enumerate(feats)]
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    out = m(list(ins))
    cot = torch.randn(out.shape, generator=torch.Generator().manual_seed(123))
    m.zero_grad(set_to_none=True)
    (out * cot).sum().backward()
    arr = {f"in/f{i}": f for i, f in enumerate(feats)}
    arr["out/0"] = out
    for i in idx:
        arr[f"grad/f{i}"] = ins[i].grad
    params = dict(m.named_parameters())
    for p in ("head.weight", "FPN.conv_fusion.0.weight", "FPN.smooth_conv.0.weight", "PPN.bottleneck.0.weight",
              "PPN.stages.0.1.weight"):
        arr[f"grad/{p}"] = params[p].grad
    for k, v in sd0.items():
        arr[f"sd/{k}"] = v
    dump(name, None, **arr)


def main(only=None):
    os.makedirs(OUT, exist_ok=True)
    if only:                       # python tools/gen_golden.py swin_alt vit_cls_c1 train_step_product
        torch.set_num_threads(min(8, os.cpu_count() or 1))
        for name in only:
            if name == "swin_alt":
                for i, cfg in enumerate(SWIN_ALT):
                    swin_alt_layer(*cfg, seed=20 + i)
            elif name == "vit_cls_c1":
                vit_cls_c1(15)
            elif name == "train_step_product":
                train_step_product(16)
            elif name == "train_step_adam":
                train_step_adam(16)
            elif name == "unetr":
                for cfg in UNETR:
                    unetr_vit(*cfg)
                unetr_swin("unetr_swin3d_p2", (64, 64, 64), 96, 43)
            else:
                raise SystemExit(f"unknown fixture group {name}")
        return
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    sablock("sablock_attn_h128", 128, 2, 2, 256, 0)
    sablock("sablock_attn_h192_l77", 192, 3, 1, 77, 1)
    vit_encoder("vit_enc_attn", 128, 2, 256, 2, (16, 16), (2, 2), 2, 2)
    vit_encoder("vit_enc_cls", 128, 2, 256, 1, (8, 8), (2, 2), 2, 3, classification=True)
    vit_encoder("vit_enc_hyena", 128, 2, 256, 1, (16, 16), (2, 2), 1, 4, use_hyena=True)
    vit_encoder("vit_enc_mamba", 128, 2, 256, 1, (16, 16), (2, 2), 1, 5, use_mamba=True)
    hyena_op(6)
    mamba_mixer(7)
    window_attention(8)
    swin_layer(9)
    swin_index()
    train_step(10)
    train_step_product(16)
    train_step_adam(16)
    vit_cls_c1(15)
    for cfg in UNETR:
        unetr_vit(*cfg)
    unetr_swin("unetr_swin3d_p2", (64, 64, 64), 96, 43)
    for i, cfg in enumerate(SWIN_ALT):
        swin_alt_layer(*cfg, seed=20 + i)
    upernet("upernet2d_swin", 2, "Swin", 11)
    upernet("upernet2d_vit", 2, "ViT", 12)
    upernet("upernet3d_swin", 3, "Swin", 13)
    upernet("upernet3d_vit", 3, "ViT", 14)


if __name__ == "__main__":
    main(sys.argv[1:])
