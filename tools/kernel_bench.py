#!/usr/bin/env python3
"""Per-kernel benchmark of every liblci hot-path kernel at its BASELINE config size (HIP events, random data).

Prints one JSON line per kernel with the algorithmic work per launch and the roofline fraction:
  attention   C2/metric: B=2, H=6, L=65536, d=64            FLOPs fwd 4BHL^2d, bwd 8BHL^2d (MFMA bf16)
  window      C3 stage 1: 128^3 p2 -> 64^3 grid, C=96, H=3, w=7, shift 3   FLOPs 4*Bw*H*N^2*32 (N=343)
  scan        ViT-mamba 512^2 p2 (L=65536) and C5 256^3 p2 (L=2^21), Dx=192, N=8, bf16
              bytes/token fwd 2*(3*192+16)=1184, bwd 1984
  fftconv     ViT-hyena 512^2 p2: rows B*D = 768, L = 65536, f32 in/out: bytes/row-elem 8 fwd, 16 bwd
  patch embed ViT p2 512^2: image 4 B/px + tokens B*L*384*4 B
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from long_context_biomedical_imaging_amd import kernels  # noqa: E402

MFMA = 2500.0
HBM = 8000.0


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def emit(name, ms, work, unit, cfg):
    if unit == "TFLOP/s":
        ach = work / (ms * 1e-3) / 1e12
        peak = MFMA
    else:
        ach = work / (ms * 1e-3) / 1e9
        peak = HBM
    print(json.dumps({"kernel": name, "ms": round(ms, 3), "achieved": round(ach, 1), "unit": unit,
                      "peak": peak, "frac": round(ach / peak, 4), "work_per_launch": work, "config": cfg}),
          flush=True)


def bench_attention():
    B, H, L = 2, 6, 65536
    qkv = torch.randn(B, L, 3 * H * 64, device="cuda").to(torch.bfloat16)
    dout = torch.randn(B, L, H * 64, device="cuda").to(torch.bfloat16)
    out, lse = kernels.attn_fwd(qkv, H, 0.125)
    f = 4.0 * B * H * L * L * 64
    emit("attn_fwd", timeit(lambda: kernels.attn_fwd(qkv, H, 0.125)), f, "TFLOP/s", f"B{B} H{H} L{L} d64")
    emit("attn_bwd(3 launches)", timeit(lambda: kernels.attn_bwd(qkv, out, dout, lse, H, 0.125)), 2 * f, "TFLOP/s",
         f"B{B} H{H} L{L} d64")
    kernels.KernelTimer.reset()
    kernels.KernelTimer.enabled = True
    for _ in range(3):
        kernels.attn_bwd(qkv, out, dout, lse, H, 0.125)
    kernels.KernelTimer.enabled = False
    for name, d in kernels.KernelTimer.summary().items():
        if d["work_per_call"]:
            emit(name, d["avg_ms"], d["work_per_call"], "TFLOP/s", f"B{B} H{H} L{L} d64 (MFMA FLOPs of this stage)")
        else:
            print(json.dumps({"kernel": name, "ms": round(d["avg_ms"], 3)}), flush=True)


def bench_window():
    B, S, C, H, w, sh = 2, 64, 96, 3, 7, 3
    qkv = torch.randn(B, S, S, S, 3 * C, device="cuda").to(torch.bfloat16).requires_grad_(True)
    bias = torch.randn(3 * C, device="cuda") * 0.1
    rpb = torch.randn(H, w ** 3, w ** 3, device="cuda") * 0.1
    N = w ** 3
    Bw = B * (-(-S // w)) ** 3
    f = 4.0 * Bw * H * N * N * 32
    run = lambda: kernels.window_attention_grid(qkv, bias, rpb, H, 32 ** -0.5, (w, w, w), (sh, sh, sh))  # noqa
    emit("window_attn_fwd", timeit(lambda: run()), f, "TFLOP/s", f"Swin-tiny stage1 128^3 p2: B{B} 64^3 C{C} H{H} w7 s3")
    o = run()
    g = torch.randn_like(o)
    emit("window_attn_fwd+bwd", timeit(lambda: torch.autograd.grad(run(), qkv, g)), 3 * f, "TFLOP/s",
         "same, fwd+bwd (rpb grad off)")
    rpb.requires_grad_(True)
    emit("window_attn_fwd+bwd+drpb", timeit(lambda: torch.autograd.grad(run(), [qkv, rpb], g)), 3 * f, "TFLOP/s",
         "same, fwd+bwd with the rpb gradient (dS tiles + window reduction)")


def bench_window_stages():
    """Window attention at every Swin-tiny stage of C3 (128^3 p2, B = 1, window 7): fwd, bwd without / with the
    rpb gradient, per stage and shift (the block pairs run shift 0 then 3)."""
    for S, C, H in ((64, 96, 3), (32, 192, 6), (16, 384, 12), (8, 768, 24)):
        w, B = 7, 1
        N = w ** 3
        Bw = B * (-(-S // w)) ** 3
        f = 4.0 * Bw * H * N * N * 32
        for sh in (0, 3):
            qkv = torch.randn(B, S, S, S, 3 * C, device="cuda").to(torch.bfloat16).requires_grad_(True)
            bias = torch.randn(3 * C, device="cuda") * 0.1
            rpb = torch.randn(H, N, N, device="cuda") * 0.1
            run = lambda: kernels.window_attention_grid(qkv, bias, rpb, H, 32 ** -0.5, (w, w, w), (sh, sh, sh))  # noqa
            cfg = f"S{S} C{C} H{H} Bw{Bw} w7 s{sh}"
            tf = timeit(lambda: run(), iters=10)
            emit("window_attn_fwd", tf, f, "TFLOP/s", cfg)
            o = run()
            g = torch.randn_like(o)
            tb = timeit(lambda: torch.autograd.grad(run(), qkv, g), iters=10) - tf
            emit("window_attn_bwd", tb, 2 * f, "TFLOP/s", cfg + " (bwd = fwd+bwd - fwd, rpb grad off)")
            rpb.requires_grad_(True)
            tr = timeit(lambda: torch.autograd.grad(run(), [qkv, rpb], g), iters=10) - tf
            emit("window_attn_bwd+drpb", tr, 2 * f, "TFLOP/s", cfg + " (with the rpb gradient)")


def bench_scan(L, B=2, Dx=192):
    u = torch.randn(B, L, Dx, device="cuda").to(torch.bfloat16).requires_grad_(True)
    dl = (torch.randn(B, L, Dx, device="cuda") * 0.5 - 3).to(torch.bfloat16).requires_grad_(True)
    A = -torch.rand(Dx, 8, device="cuda") - 0.5
    xdbl = torch.randn(B, L, 40, device="cuda").to(torch.bfloat16).requires_grad_(True)
    D = torch.randn(Dx, device="cuda")
    db = torch.randn(Dx, device="cuda") * 0.1

    def fwd(grad=False):
        yz = torch.empty(B, L, 2 * Dx, device="cuda", dtype=torch.bfloat16)
        with torch.set_grad_enabled(grad):
            return kernels.selective_scan_cl(u, dl, A, xdbl[..., 24:32], xdbl[..., 32:], D, db, yz)

    emit("selective_scan_fwd", timeit(lambda: fwd(False)), 1184.0 * B * L, "GB/s", f"B{B} L{L} Dx{Dx} N8 bf16")
    y = fwd(True)
    gy = torch.randn_like(y)
    # LCI_NO_KTIMER=1 (rocprofv3 --pmc passes): no per-launch HIP events (the counters then come from the profiler)
    timed = not os.environ.get("LCI_NO_KTIMER")
    kernels.KernelTimer.reset()
    kernels.KernelTimer.enabled = timed
    for _ in range(3):
        y = fwd(True)
        torch.autograd.grad(y, [u, dl, xdbl], gy)
    kernels.KernelTimer.enabled = False
    if timed:
        s = kernels.KernelTimer.summary()
        if "selective_scan_fwd" in s:
            emit("selective_scan_fwd(+ckpt)", s["selective_scan_fwd"]["avg_ms"], 1184.0 * B * L, "GB/s",
                 f"B{B} L{L} Dx{Dx} N8 bf16, training forward (writes the backward's state checkpoints)")
        emit("selective_scan_bwd", s["selective_scan_bwd"]["avg_ms"], 1984.0 * B * L, "GB/s",
             f"B{B} L{L} Dx{Dx} N8 bf16")


def bench_scan_windows():
    """The Swin-Mamba recipe's scans (projects/run_abct.sh: Swin-tiny p2, 4^3 windows, 128^3 volume, B = 2): every
    window is an L = 64 sequence; stages 1-4 give (B nW, Dx) = (8192, 48), (1024, 96), (128, 192), (16, 384).
    Algorithmic bytes per token: fwd 2 (3 Dx + 2 N), bwd 2 (5 Dx + 4 N) (bf16 I/O)."""
    for B, Dx in ((8192, 48), (1024, 96), (128, 192), (16, 384)):
        L, N = 64, 8
        u = torch.randn(B, L, Dx, device="cuda").to(torch.bfloat16).requires_grad_(True)
        dl = (torch.randn(B, L, Dx, device="cuda") * 0.5 - 3).to(torch.bfloat16).requires_grad_(True)
        A = -torch.rand(Dx, N, device="cuda") - 0.5
        bc = torch.randn(B, L, 2 * N, device="cuda").to(torch.bfloat16).requires_grad_(True)
        D = torch.randn(Dx, device="cuda")
        db = torch.randn(Dx, device="cuda") * 0.1

        def fwd(grad=False):
            yz = torch.empty(B, L, 2 * Dx, device="cuda", dtype=torch.bfloat16)
            with torch.set_grad_enabled(grad):
                return kernels.selective_scan_cl(u, dl, A, bc[..., :N], bc[..., N:], D, db, yz)

        fb, bb = 2.0 * (3 * Dx + 2 * N) * B * L, 2.0 * (5 * Dx + 4 * N) * B * L
        cfg = f"B{B} L{L} Dx{Dx} N8 bf16 (window scan)"
        emit("selective_scan_fwd_win", timeit(lambda: fwd(False), iters=20), fb, "GB/s", cfg)
        y = fwd(True)
        gy = torch.randn_like(y)
        tb = timeit(lambda: torch.autograd.grad(fwd(True), [u, dl, bc], gy), iters=20)
        tf = timeit(lambda: fwd(True), iters=20)
        emit("selective_scan_bwd_win", tb - tf, bb, "GB/s", cfg + " (fwd+bwd minus the training fwd)")


def bench_dwconv(L=1 << 21, B=1, C=192):
    """Mamba depthwise conv + SiLU pair (mamba.py:118-119) at the C5 shape: in (B, L, 2C) bf16; fwd reads 2C and
    writes 2C values per token (4 B each way per channel at bf16), bwd reads in + dout and writes din."""
    xz = torch.randn(B, L, 2 * C, device="cuda").to(torch.bfloat16).requires_grad_(True)
    wx, wz = torch.randn(C, 1, 3, device="cuda"), torch.randn(C, 1, 3, device="cuda")
    bx, bz = torch.randn(C, device="cuda"), torch.randn(C, device="cuda")
    for t in (wx, wz, bx, bz):
        t.requires_grad_(True)
    fb = 2.0 * 2 * C * B * L * 2
    emit("dwconv_silu_fwd", timeit(lambda: kernels.dwconv_silu_pair(xz, wx, bx, wz, bz)), fb, "GB/s",
         f"B{B} L{L} 2C{2 * C} bf16")
    xs, yz = kernels.dwconv_silu_pair(xz, wx, bx, wz, bz)
    gx, gz = torch.randn_like(xs), torch.randn_like(yz)
    emit("dwconv_silu_fwd+bwd", timeit(lambda: torch.autograd.grad(kernels.dwconv_silu_pair(xz, wx, bx, wz, bz),
                                                                     [xz, wx, wz], [gx, gz])),
         fb + 3.0 * 2 * C * B * L * 2, "GB/s", f"B{B} L{L} 2C{2 * C} bf16 (bwd: in + dout read, din written)")


def bench_fftconv():
    for L, tag in ((65536, "ViT-hyena 512^2 p2"), (262144, "C4: ViT-hyena 1024^2 p2, n = 2^19")):
        B, H, hd = 2, 6, 64
        u = torch.randn(B * H, hd, L, device="cuda").requires_grad_(True)
        k = (torch.randn(hd, L, device="cuda") * torch.exp(-torch.linspace(0, 8, L, device="cuda"))).requires_grad_(True)
        D = torch.randn(hd, device="cuda").requires_grad_(True)
        rows = B * H * hd
        emit("fftconv_fwd", timeit(lambda: kernels.fftconv(u, k, D)), 8.0 * rows * L, "GB/s", f"rows {rows} L{L} f32 ({tag})")
        y = kernels.fftconv(u, k, D)
        g = torch.randn_like(y)
        emit("fftconv_fwd+bwd", timeit(lambda: torch.autograd.grad(kernels.fftconv(u, k, D), [u, k, D], g)),
             24.0 * rows * L, "GB/s", f"L{L}, fwd+bwd (u, k, D grads)")
        del u, k, D, y, g
        torch.cuda.empty_cache()


def bench_direct_conv():
    """Direct (Toeplitz, f32 MFMA) long conv at the Swin-Hyena window shapes (128^3 p2, B=2: stage 1-4 at window 8,
    window 7 and window 4 stage 1). FLOPs = R C L (L + 1) per launch (fwd, adjoint and filter gradient alike)."""
    for R, C, L, tag in ((3072, 32, 512, "w8 stage1"), (768, 32, 512, "w8 stage2"), (192, 32, 512, "w8 stage3"),
                         (48, 32, 512, "w8 stage4"), (6000, 32, 343, "w7 stage1"), (24576, 32, 64, "w4 stage1")):
        u = torch.randn(R, C, L, device="cuda").requires_grad_(True)
        k = (torch.randn(C, L, device="cuda") * 0.1).requires_grad_(True)
        D = torch.randn(C, device="cuda").requires_grad_(True)
        fl = float(R * C) * L * (L + 1)
        y = kernels._DirectConv.apply(u, k, D)
        g = torch.randn_like(y)
        t_f = timeit(lambda: kernels._DirectConv.apply(u, k, D))
        t_fb = timeit(lambda: torch.autograd.grad(kernels._DirectConv.apply(u, k, D), [u, k, D], g))
        for name, ms, w in (("direct_conv_fwd", t_f, fl), ("direct_conv_fwd+bwd", t_fb, 3 * fl)):
            print(json.dumps({"kernel": name, "ms": round(ms, 4), "achieved": round(w / (ms * 1e-3) / 1e12, 1),
                              "unit": "TFLOP/s", "peak": 157.3, "frac": round(w / (ms * 1e-3) / 1e12 / 157.3, 3),
                              "config": f"R{R} C{C} L{L} ({tag})"}), flush=True)


def bench_patch_embed():
    B, S, D = 2, 512, 384
    x = torch.rand(B, 1, S, S, device="cuda")
    w = (torch.randn(D, 1, 2, 2, device="cuda") * 0.1).requires_grad_(True)
    b = torch.zeros(D, device="cuda").requires_grad_(True)
    pos = torch.zeros(1, (S // 2) ** 2, D, device="cuda").requires_grad_(True)
    byt = 4.0 * B * S * S + 4.0 * B * (S // 2) ** 2 * D + 4.0 * (S // 2) ** 2 * D
    emit("patch_embed_fwd", timeit(lambda: kernels.patch_embed(x, w, b, pos, True)), byt, "GB/s",
         "ViT p2 512^2 -> (2, 65536, 384) f32 + pos")


def bench_linear():
    """Linear weight gradient dW = dY^T X (+ db) at the ViT (M = 131072) and C5 (M = 2^21) token counts: the HIP
    split-token kernel vs torch's hipBLASLt GEMM of the same bf16 operands."""
    from long_context_biomedical_imaging_amd.trainer import use_tuned_gemms
    print(json.dumps({"tuned_gemm_table": use_tuned_gemms()}), flush=True)   # torch's side as the product runs it
    shapes = {"qkv": (1152, 384), "proj": (384, 384), "fc1": (1536, 384), "fc2": (384, 1536),
              "m_x": (40, 192), "m_dt": (192, 24), "swin_qkv96": (288, 96), "swin_fc2_96": (96, 384)}
    for M in (131072, 1 << 21):
        for name, (N, K) in shapes.items():
            dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            f = 2.0 * M * N * K
            if kernels.linear_wgrad_supported(dy, x):
                emit(f"linear_wgrad {name}", timeit(lambda: kernels.linear_wgrad(dy, x, True)), f, "TFLOP/s",
                     f"M{M} N{N} K{K} (+db, split partials summed)")
            emit(f"torch dy^T x {name}", timeit(lambda: dy.t() @ x), f, "TFLOP/s", f"M{M} N{N} K{K}")
            del dy, x
            torch.cuda.empty_cache()


def bench_lw_split():
    """lci_linear_wgrad + the caller's partial sums (the product path) at the metric / C4 / C5 token counts; run under
    different LCI_LW_WGS / LCI_LW_MINROWS to price the split count."""
    shapes = {"qkv": (1152, 384), "proj": (384, 384), "fc1": (1536, 384), "fc2": (384, 1536), "m_in": (768, 384),
              "m_x": (40, 192), "m_dt": (192, 24)}
    for M in (131072, 524288, 1 << 21):
        for name, (N, K) in shapes.items():
            dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            ns = kernels._lib.load().lci_linear_wgrad_splits(M, N, K)
            emit(f"linear_wgrad {name}", timeit(lambda: kernels.linear_wgrad(dy, x, True), iters=10), 2.0 * M * N * K,
                 "TFLOP/s", f"M{M} N{N} K{K} ns{ns}")
            del dy, x
        torch.cuda.empty_cache()


def bench_mlp():
    """The MLPBlock (linear1 -> GELU -> linear2, backbone_vit.py:249) forward + backward under bf16 autocast at the
    ViT (M = 131072) and C5 (M = 2^21) token counts: forward / data-gradient GEMMs on lci_gemm_bt (the default) vs
    hipBLASLt (LCI_HIP_GEMM=0), the GELU and weight gradients on the HIP kernels either way."""
    from long_context_biomedical_imaging_amd import blocks, trainer
    trainer.use_tuned_gemms()
    D, H = 384, 1536
    for M in (131072, 1 << 21):
        f = 2.0 * M * D * H
        mb = blocks.MLPBlock(D, H).cuda()
        xm = torch.randn(M, D, device="cuda", requires_grad=True)
        gy = torch.randn(M, D, device="cuda").to(torch.bfloat16)

        def step():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = mb(xm)
            y.backward(gy)
        for hip in (True, False, True, False):
            kernels.HIP_GEMM = hip
            emit(f"MLPBlock fwd+bwd {'gemm_bt' if hip else 'hipBLASLt'}", timeit(step, 10), 6 * f, "TFLOP/s",
                 f"M{M} D{D} H{H}")
        kernels.HIP_GEMM = True
        del xm, gy, mb
        torch.cuda.empty_cache()


def bench_gemm():
    """Projection GEMMs y = x w^T (+ b), bf16: lci_gemm_bt vs torch's (hipBLASLt, TunableOp table if present) at the
    ViT-small shapes (qkv 384->1152, out_proj 384->384, fc1 384->1536, fc2 1536->384 and its data gradient) for the
    metric's M = 131072 tokens and C5's 2^21."""
    from long_context_biomedical_imaging_amd import trainer
    trainer.use_tuned_gemms()
    for M in (131072, 1 << 21):
        for K, N, nm in ((384, 1152, "qkv"), (384, 384, "out_proj"), (384, 1536, "fc1"), (1536, 384, "fc2"),
                         (384, 2048, "convup 384->8x256"), (256, 1024, "convup 256->8x128"), (512, 2048, "convup K512")):
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
            b = torch.randn(N, device="cuda").to(torch.bfloat16)
            f = 2.0 * M * N * K
            emit(f"gemm_bt {nm}", timeit(lambda: kernels.gemm_bt(x, w, b), iters=10), f, "TFLOP/s", f"M{M} K{K} N{N} bf16")
            emit(f"torch linear {nm}", timeit(lambda: torch.nn.functional.linear(x, w, b), iters=10), f, "TFLOP/s",
                 f"M{M} K{K} N{N} bf16 (hipBLASLt)")
            del x, w, b
            torch.cuda.empty_cache()


def bench_gemm_swin():
    """lci_gemm_bt vs torch at the Swin-tiny projection shapes of C3 (128^3 p2, B = 1: 64^3 / 32^3 / 16^3 / 8^3 tokens;
    widths 96 / 192 / 384 / 768) that the HIP GEMM takes (N % 384 == 0), forward and data gradient."""
    from long_context_biomedical_imaging_amd import trainer
    trainer.use_tuned_gemms()
    for M, K, N, nm in ((262144, 96, 384, "s1 fc1"), (262144, 96, 384, "s1 fc2 dX"), (32768, 192, 768, "s2 fc1"),
                        (32768, 192, 384, "s2 qkv dX? (192->576 no) fc2 dX"), (4096, 384, 1152, "s3 qkv"),
                        (4096, 384, 1536, "s3 fc1"), (4096, 1536, 384, "s3 fc2"), (512, 768, 3072 - 3072 % 384, "s4 fc1"),
                        (131072, 96, 384, "K96 M131072"), (131072, 192, 384, "K192"), (131072, 288, 384, "K288")):
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda").to(torch.bfloat16)
        f = 2.0 * M * N * K
        emit(f"gemm_bt {nm}", timeit(lambda: kernels.gemm_bt(x, w, b), iters=20), f, "TFLOP/s", f"M{M} K{K} N{N} bf16")
        emit(f"torch linear {nm}", timeit(lambda: torch.nn.functional.linear(x, w, b), iters=20), f, "TFLOP/s",
             f"M{M} K{K} N{N} bf16 (hipBLASLt)")


def main():
    which = sys.argv[1:] or ["attention", "window", "scan", "fftconv", "patch", "linear", "mlp"]
    if "attention" in which:
        bench_attention()
    if "window" in which:
        bench_window()
    if "wstages" in which:
        bench_window_stages()
    if "scan" in which:
        bench_scan(65536)
        bench_scan(1 << 21)
    if "scanwin" in which:
        bench_scan_windows()
    if "dwconv" in which:
        bench_dwconv()
    if "fftconv" in which:
        bench_fftconv()
    if "dconv" in which:
        bench_direct_conv()
    if "patch" in which:
        bench_patch_embed()
    if "linear" in which:
        bench_linear()
    if "mlp" in which:
        bench_mlp()
    if "lwsplit" in which:
        bench_lw_split()
    if "gemm" in which:
        bench_gemm()
    if "gemm_swin" in which:
        bench_gemm_swin()


if __name__ == "__main__":
    main()
