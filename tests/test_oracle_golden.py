"""Pin the CPU oracle (oracle/) against golden vectors produced by the reference (tools/gen_golden.py)."""
import hashlib

import numpy as np
import pytest
import torch

from golden_util import Golden, assert_close, cotangents
from oracle import attention, hyena, patch_embed, selective_scan, vit, window

torch.set_num_threads(4)


def _grad(fn, inputs):
    ins = [x.clone().double().requires_grad_(True) for x in inputs]
    out = fn(*ins)
    return out, ins


@pytest.mark.parametrize("name", ["sablock_attn_h128", "sablock_attn_h192_l77"])
def test_sablock_attention(name):
    g = Golden(name)
    sd = {k: v.double() for k, v in g.sd().items()}
    heads = int(g.scalar("cfg/heads"))
    x = g.t("in/x").double().requires_grad_(True)
    out = attention.sablock_attention(x, sd["qkv.weight"], sd.get("qkv.bias"), sd["out_proj.weight"],
                                      sd["out_proj.bias"], heads)
    assert_close(out, g.t("out/0"), 1e-5, 1e-5, "sablock out")
    (out * cotangents([out])[0].double()).sum().backward()
    assert_close(x.grad, g.t("grad/in0"), 1e-4, 1e-5, "sablock dx")


def test_attention_core_chunked_equals_full():
    torch.manual_seed(0)
    q, k, v = (torch.randn(1, 2, 300, 64, dtype=torch.float64) for _ in range(3))
    o1, l1 = attention.attention_core(q, k, v, 0.125)
    o2, l2 = attention.attention_core(q, k, v, 0.125, q_chunk=64)
    assert torch.allclose(o1, o2) and torch.allclose(l1, l2)


@pytest.mark.parametrize("name,mode", [("vit_enc_attn", "attention"), ("vit_enc_cls", "attention"),
                                       ("vit_enc_hyena", "hyena"), ("vit_enc_mamba", "mamba")])
def test_vit_encoder(name, mode):
    g = Golden(name)
    sd = g.sd()
    if mode == "hyena":
        for i in range(int(g.scalar("cfg/layers"))):
            z, t = hyena.pos_emb(66000)
            pre = f"blocks.{i}.attn.hyena.filter_fn.pos_emb."
            chk = g.t(f"chk/{pre}z", torch.float64)
            assert abs(z.double().sum().item() - chk[0].item()) < 1e-6 * max(1, abs(chk[0].item()))
            assert abs(z.double().abs().sum().item() - chk[1].item()) < 1e-6 * chk[1].item()
            sd[pre + "z"], sd[pre + "t"] = z, t
    outs = vit.vit_forward(g.t("in/x"), sd, int(g.scalar("cfg/layers")), int(g.scalar("cfg/heads")), 2, mode)
    ref = g.outs()
    assert len(outs) == len(ref)
    for i, (a, b) in enumerate(zip(outs, ref)):
        assert_close(a, b, 2e-4, 2e-4, f"{name} out {i}")


def test_hyena_operator_and_filter():
    g = Golden("hyena_op")
    sd = g.sd()
    z, t = hyena.pos_emb(66000)
    sd["filter_fn.pos_emb.z"], sd["filter_fn.pos_emb.t"] = z, t
    x = g.t("in/x")
    L = x.shape[1]
    ws = [sd[f"filter_fn.implicit_filter.{i}.weight"] for i in (0, 2, 4, 6)]
    bs = [sd.get(f"filter_fn.implicit_filter.{i}.bias") for i in (0, 2, 4, 6)]
    k = hyena.implicit_filter(L, z, t, ws, bs, sd["filter_fn.implicit_filter.1.freq"],
                              sd["filter_fn.modulation.deltas"])[0].transpose(0, 1)
    assert_close(k, g.t("out/k"), 1e-5, 1e-6, "hyena filter k")
    y = hyena.hyena_forward(x, sd, num_heads=2)
    assert_close(y, g.t("out/0"), 1e-4, 1e-5, "hyena out")


@pytest.mark.parametrize("L", [1000, 2048])
def test_fftconv_matches_reference_and_direct(L):
    g = Golden(f"fftconv_L{L}")
    u, k, D = g.t("in/u"), g.t("in/k"), g.t("in/D")
    y = hyena.fftconv(u, k, D)
    assert_close(y, g.t("out/y"), 1e-5, 1e-5, "fftconv vs reference")
    if L == 1000:
        yd = hyena.causal_conv_direct(u[:, :1, :8], k[:8], D[:8])
        assert_close(yd, g.t("out/y")[:, :1, :8], 1e-4, 1e-4, "direct causal conv vs reference")


def test_hyena_lmax_behaviour():
    g = Golden("hyena_lmax")
    err = str(g.z["out/err"])
    assert err.startswith("AttributeError") and "max_l" in err


def test_selective_scan_and_grads():
    g = Golden("selective_scan")
    names = ["u", "delta", "A", "B", "C", "D", "delta_bias"]
    ins = [g.t(f"in/{n}").double().requires_grad_(True) for n in names]
    y = selective_scan.selective_scan(*ins[:6], delta_bias=ins[6], delta_softplus=True)
    assert_close(y, g.t("out/y"), 1e-5, 1e-5, "scan y")
    (y * g.t("cot/y").double()).sum().backward()
    for n, x in zip(names, ins):
        assert_close(x.grad, g.t(f"grad/{n}"), 1e-4, 1e-4, f"scan grad {n}")


def test_selective_scan_naive_loop_fp64():
    """Independent check of the scan restatement: a plain per-element fp64 loop."""
    torch.manual_seed(1)
    b, d, n, L = 1, 3, 4, 40
    u, dl = torch.randn(b, d, L, dtype=torch.float64), torch.randn(b, d, L, dtype=torch.float64)
    A = -torch.rand(d, n, dtype=torch.float64)
    B, C = torch.randn(b, n, L, dtype=torch.float64), torch.randn(b, n, L, dtype=torch.float64)
    Dv, db = torch.randn(d, dtype=torch.float64), torch.randn(d, dtype=torch.float64)
    y = selective_scan.selective_scan(u, dl, A, B, C, Dv, db, True).double()
    ref = torch.zeros_like(u)
    import math
    for bi in range(b):
        for di in range(d):
            x = [0.0] * n
            for t in range(L):
                v = dl[bi, di, t].item() + db[di].item()
                dt = v if v > 20 else math.log1p(math.exp(v))
                acc = 0.0
                for ni in range(n):
                    x[ni] = math.exp(dt * A[di, ni].item()) * x[ni] + dt * B[bi, ni, t].item() * u[bi, di, t].item()
                    acc += C[bi, ni, t].item() * x[ni]
                ref[bi, di, t] = acc + Dv[di].item() * u[bi, di, t].item()
    assert_close(y, ref, 1e-5, 1e-6, "scan vs naive loop")


def test_mamba_mixer():
    g = Golden("mamba_mixer")
    sd = g.sd()
    x = g.t("in/x")
    y = selective_scan.mamba_mixer(x, sd)
    assert_close(y, g.t("out/0"), 1e-4, 1e-5, "mamba mixer out")


@pytest.mark.parametrize("name,ws", [("window_attn_3d", (7, 7, 7)), ("window_attn_2d", (7, 7))])
def test_window_attention(name, ws):
    g = Golden(name)
    sd = g.sd()
    x = g.t("in/x").double().requires_grad_(True)
    rpb = sd["relative_position_bias_table"].double().requires_grad_(True)
    assert np.array_equal(sd["relative_position_index"].numpy(), window.relative_position_index(ws))
    mask = g.t("in/mask")
    assert torch.equal(mask, window.compute_mask(
        [7, 7, 14] if len(ws) == 3 else [14, 14], ws, (3,) * len(ws)))
    out = window.window_attention(x, mask.double(), sd["qkv.weight"].double(), sd["qkv.bias"].double(),
                                  sd["proj.weight"].double(), sd["proj.bias"].double(), rpb,
                                  sd["relative_position_index"], 2)
    assert_close(out, g.t("out/0"), 1e-5, 1e-5, "window attn out")
    (out * cotangents([out])[0].double()).sum().backward()
    assert_close(x.grad, g.t("grad/in0"), 1e-4, 1e-5, "window attn dx")
    assert_close(rpb.grad, g.t("grad/relative_position_bias_table"), 1e-4, 1e-5, "window attn drpb")


def test_swin_index_ops_bit_exact():
    g = Golden("swin_index")
    assert np.array_equal(g.z["out/rp_index_3d"], window.relative_position_index((7, 7, 7)))
    assert np.array_equal(g.z["out/rp_index_2d"], window.relative_position_index((7, 7)))
    for d in (14, 21, 35, 70):
        m = window.compute_mask([d] * 3, (7, 7, 7), (3, 3, 3)).numpy()
        nz = m != 0
        assert list(m.shape) == list(g.z[f"out/mask_shape_{d}"])
        assert int(nz.sum()) == int(g.z[f"out/mask_nnz_{d}"])
        assert hashlib.sha256(np.packbits(nz).tobytes()).hexdigest() == str(g.z[f"out/mask_sha256_{d}"])
        idx = torch.arange(d ** 3, dtype=torch.float64).reshape(1, d, d, d, 1)
        perm = window.window_partition(torch.roll(idx, (-3, -3, -3), (1, 2, 3)), (7, 7, 7)).reshape(-1)
        perm = perm.long().numpy().astype(np.int32)
        assert hashlib.sha256(perm.tobytes()).hexdigest() == str(g.z[f"out/partition_sha256_{d}"])
    for key in [k for k in g.z.files if k.startswith("out/gws_")]:
        size = tuple(int(s) for s in key[8:].split("x"))
        w, s = window.get_window_size(size, (7, 7, 7), (3, 3, 3))
        assert list(w) + list(s) == list(g.z[key])


def test_partition_reverse_roundtrip():
    x = torch.randn(2, 14, 21, 7, 5)
    assert torch.equal(window.window_reverse(window.window_partition(x, (7, 7, 7)), (7, 7, 7), [2, 14, 21, 7]), x)


def test_patch_embed_vit_block():
    g = Golden("vit_enc_attn")
    sd = g.sd()
    x = g.t("in/x").squeeze(2)
    y = patch_embed.vit_patch_embed(x, sd["patch_embedding.patch_embeddings.weight"],
                                    sd["patch_embedding.patch_embeddings.bias"],
                                    sd["patch_embedding.position_embeddings"])
    assert y.shape == (2, 64, 128)


def test_oracle_gradients_fp64_gradcheck():
    """the CPU restatements' autograd gradients (which the GPU backward kernels are checked
    against) are verified by finite differences in fp64."""
    from torch.autograd import gradcheck
    from oracle import attention as oatt
    from oracle import hyena as ohy
    from oracle import selective_scan as oss
    from oracle import window as owin
    g = torch.Generator().manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g, dtype=torch.float64).requires_grad_(True)   # noqa: E731
    q, k, v = r(1, 2, 5, 4), r(1, 2, 5, 4), r(1, 2, 5, 4)
    assert gradcheck(lambda a, b, c: oatt.attention_core(a, b, c, 0.5), (q, k, v))
    rpb, mask = r(2, 5, 5), torch.zeros(1, 5, 5, dtype=torch.float64)
    mask[0, 0, 3:] = -100.0
    assert gradcheck(lambda a, b, c, p: owin.window_attention_core(a, b, c, p, mask, 0.5), (q, k, v, rpb))
    u, dt, A = r(1, 3, 6), r(1, 3, 6), (-torch.rand(3, 2, generator=g, dtype=torch.float64)).requires_grad_(True)
    B, C, D, db = r(1, 2, 6), r(1, 2, 6), r(3), r(3)
    assert gradcheck(lambda *a: oss.selective_scan(*a, delta_softplus=True), (u, dt, A, B, C, D, db))
    uu, kk, dd = r(2, 3, 8), r(3, 8), r(3)
    assert gradcheck(ohy.fftconv, (uu, kk, dd))


def test_scan_c_oracle_matches_python_restatement():
    """oracle/scan_ref.c (fp64 per-step loop, used for the L = 2^21 GPU check) == oracle/selective_scan.py
    (pinned by the reference fixture) on the same inputs: output and all seven gradients, fp64."""
    from oracle import scan_c
    from oracle import selective_scan as oss
    torch.manual_seed(11)
    L, d, n = 777, 16, 8
    u = torch.randn(1, d, L)
    delta = torch.randn(1, d, L) * 0.5 - 1.0
    delta[0, 3, 100] = 25.0   # softplus threshold branch
    A = -torch.exp(torch.randn(d, n) * 0.3)
    Bm, Cm = torch.randn(1, n, L), torch.randn(1, n, L)
    D, db = torch.randn(d), torch.randn(d) * 0.1
    dy = torch.randn(1, d, L)
    ins = [t.double().requires_grad_(True) for t in (u, delta, A, Bm, Cm, D, db)]
    yr = oss.selective_scan(*ins[:6], delta_bias=ins[6], delta_softplus=True)
    (yr * dy.double()).sum().backward()
    cl = lambda t: t[0].T.numpy()  # noqa: E731  (1, c, L) -> (L, c)
    y = scan_c.scan_fwd(cl(u), cl(delta), A.numpy(), cl(Bm), cl(Cm), D.numpy(), db.numpy())
    assert np.abs(y - cl(yr.detach())).max() < 1e-10 * max(1.0, np.abs(y).max())
    du, dd, dA, dD, ddb, dB, dC = scan_c.scan_bwd(cl(u), cl(delta), A.numpy(), cl(Bm), cl(Cm), D.numpy(),
                                                   db.numpy(), cl(dy))
    for mine, ref in ((du, cl(ins[0].grad)), (dd, cl(ins[1].grad)), (dA, ins[2].grad.numpy()), (dB, cl(ins[3].grad)),
                      (dC, cl(ins[4].grad)), (dD, ins[5].grad.numpy()), (ddb, ins[6].grad.numpy())):
        assert np.abs(mine - ref).max() < 1e-9 * max(1.0, np.abs(ref).max())
