"""torch.autograd wrappers over the liblci C-ABI. Each op runs the HIP kernels; none has a CPU path."""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib


class KernelTimer:
    """Optional HIP-event timing of individual liblci launches, recorded on the launch stream.

    bench.py enables it for the timed region; each entry is (name, start_event, end_event, algorithmic work).
    """
    enabled = False
    only = None          # a set of names: time only those launches (None: every launch)
    records: list = []

    @classmethod
    def run(cls, name, work, t, fn):
        if not cls.enabled or (cls.only is not None and name not in cls.only):
            fn()
            return
        st = torch.cuda.current_stream(t.device)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        cls.records.append((name, e0, e1, work))

    @classmethod
    def summary(cls):
        """name -> {calls, avg_ms, total_ms, work_per_call} (synchronizes)."""
        torch.cuda.synchronize()
        out = {}
        for name, e0, e1, work in cls.records:
            d = out.setdefault(name, {"calls": 0, "total_ms": 0.0, "total_work": 0.0})
            d["calls"] += 1
            d["total_ms"] += e0.elapsed_time(e1)
            d["total_work"] += work
        for d in out.values():
            d["avg_ms"] = d["total_ms"] / d["calls"]
            # mean work per launch: with avg_ms, gives the time-weighted rate total_work / total_ms even when
            # one name covers launches of different shapes (window attention per stage, decoder convs)
            d["work_per_call"] = d["total_work"] / d["calls"]
        return out

    @classmethod
    def reset(cls):
        cls.records = []


# ------------------------------------------------------------------------------------- attention
def attn_fwd(qkv: torch.Tensor, num_heads: int, scale: float):
    """qkv (B, L, 3*H*64) bf16 -> out (B, L, H*64) bf16, lse2 (B, H, L) f32."""
    _lib.require_gpu(qkv)
    B, L, C = qkv.shape
    dh = C // (3 * num_heads)
    if qkv.dtype != torch.bfloat16:
        raise _lib.LciError("attn_fwd expects bf16 qkv")
    out = torch.empty(B, L, num_heads * dh, device=qkv.device, dtype=torch.bfloat16)
    lse2 = torch.empty(B, num_heads, L, device=qkv.device, dtype=torch.float32)
    ws = torch.empty(_lib.load().lci_attn_fwd_ws_bytes(B, L, num_heads) // 4, device=qkv.device,
                     dtype=torch.float32)
    KernelTimer.run("attn_fwd", 4.0 * B * num_heads * L * L * dh, qkv, lambda: _lib.call(
        "lci_attn_fwd", qkv.data_ptr(), out.data_ptr(), lse2.data_ptr(), ws.data_ptr(), B, L, num_heads, dh,
        float(scale), _lib.stream_of(qkv)))
    return out, lse2


def attn_bwd(qkv, out, dout, lse2, num_heads: int, scale: float):
    _lib.require_gpu(qkv, out, dout, lse2)
    B, L, C = qkv.shape
    dh = C // (3 * num_heads)
    dqkv = torch.empty_like(qkv)
    # -lse2 | -delta rows (include/lci.h lci_attn_bwd_ws_bytes)
    delta = torch.empty(int(_lib.load().lci_attn_bwd_ws_bytes(B, num_heads, L)), device=qkv.device, dtype=torch.uint8)
    args = (qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse2.data_ptr(), dqkv.data_ptr(), delta.data_ptr(),
            B, L, num_heads, dh, float(scale), _lib.stream_of(qkv))
    if not KernelTimer.enabled:
        _lib.call("lci_attn_bwd", *args)
        return dqkv
    f = float(B) * num_heads * L * L * dh
    # same three launches as lci_attn_bwd, timed one by one (algorithmic FLOPs: dP, dV, dK | dQ)
    KernelTimer.run("attn_bwd_delta", 0.0, qkv, lambda: _lib.call("lci_attn_bwd_stage", 0, *args))
    KernelTimer.run("attn_bwd_dkdv", 6.0 * f, qkv, lambda: _lib.call("lci_attn_bwd_stage", 1, *args))
    KernelTimer.run("attn_bwd_dq", 2.0 * f, qkv, lambda: _lib.call("lci_attn_bwd_stage", 2, *args))
    return dqkv


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, num_heads, scale):
        out, lse2 = attn_fwd(qkv, num_heads, scale)
        ctx.save_for_backward(qkv, out, lse2)
        ctx.num_heads, ctx.scale = num_heads, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse2 = ctx.saved_tensors
        dout = dout.to(torch.bfloat16).contiguous()
        return attn_bwd(qkv, out, dout, lse2, ctx.num_heads, ctx.scale), None, None


ATTN_HEAD_DIM = 64        # csrc/attention.hip DH (the placed bf16 kernels)
ATTN_GEN_MAX_HEAD_DIM = 256   # csrc/attention_gen.hip (f32 products: fp32 mode, and head dims above 64)
WIN_HEAD_DIM = 32    # csrc/window.hip WHD


def attn_gen_fwd(qkv: torch.Tensor, num_heads: int, scale: float):
    """qkv (B, L, 3*H*D) f32 or bf16, any D <= 256 -> out (B, L, H*D) same dtype, lse (B, H, L) f32 (natural log).

    csrc/attention_gen.hip: every product on the f32-input MFMA (exact f32), f32 softmax."""
    _lib.require_gpu(qkv)
    B, L, C = qkv.shape
    dh = C // (3 * num_heads)
    out = torch.empty(B, L, num_heads * dh, device=qkv.device, dtype=qkv.dtype)
    lse = torch.empty(B, num_heads, L, device=qkv.device, dtype=torch.float32)
    KernelTimer.run("attn_gen_fwd", 4.0 * B * num_heads * L * L * dh, qkv, lambda: _lib.call(
        "lci_attn_gen_fwd", _DT[qkv.dtype], qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), B, L, num_heads, dh,
        float(scale), _lib.stream_of(qkv)))
    return out, lse


def attn_gen_bwd(qkv, out, dout, lse, num_heads: int, scale: float):
    _lib.require_gpu(qkv, out, dout, lse)
    B, L, C = qkv.shape
    dh = C // (3 * num_heads)
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, num_heads, L, device=qkv.device, dtype=torch.float32)
    KernelTimer.run("attn_gen_bwd", 8.0 * B * num_heads * L * L * dh, qkv, lambda: _lib.call(
        "lci_attn_gen_bwd", _DT[qkv.dtype], qkv.data_ptr(), out.data_ptr(), dout.data_ptr(), lse.data_ptr(),
        dqkv.data_ptr(), delta.data_ptr(), B, L, num_heads, dh, float(scale), _lib.stream_of(qkv)))
    return dqkv


class _GenAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, num_heads, scale):
        out, lse = attn_gen_fwd(qkv, num_heads, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.num_heads, ctx.scale = num_heads, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        dout = dout.to(qkv.dtype).contiguous()
        return attn_gen_bwd(qkv, out, dout, lse, ctx.num_heads, ctx.scale), None, None


def pad_heads(x: torch.Tensor, parts: int, num_heads: int, to: int) -> torch.Tensor:
    """(..., parts*H*hd) -> (..., parts*H*to): every head's channels zero-padded from hd to `to` (hd <= to).

    Lets the fixed-head-dim kernels run the reference's `custom` splits with a smaller head dim exactly: zero
    q / k channels add nothing to q.k, zero v channels give zero output channels (sliced off by unpad_heads), and
    F.pad's adjoint drops the padded channels' gradients. The softmax scale stays the caller's hd ** -0.5.
    """
    lead = x.shape[:-1]
    hd = x.shape[-1] // (parts * num_heads)
    return torch.nn.functional.pad(x.reshape(*lead, parts, num_heads, hd), (0, to - hd)).reshape(
        *lead, parts * num_heads * to)


def unpad_heads(o: torch.Tensor, num_heads: int, hd: int) -> torch.Tensor:
    """(..., H*to) -> (..., H*hd): the first hd channels of every head."""
    lead = o.shape[:-1]
    return o.reshape(*lead, num_heads, o.shape[-1] // num_heads)[..., :hd].reshape(*lead, num_heads * hd)


def _check_head_dim(hd: int, limit: int, what: str) -> None:
    if hd > limit:
        raise ValueError(f"{what} head_dim {hd} is not supported: the HIP kernels take head_dim <= {limit} "
                         f"(smaller splits run zero-padded to {limit}; DESIGN.md §7)")


def flash_attention(qkv: torch.Tensor, num_heads: int, scale: float) -> torch.Tensor:
    """softmax(q k^T * scale) v for the packed qkv projection (B, L, 3*H*dh) -> (B, L, H*dh).

    bf16 qkv (the trainer's autocast) with dh <= 64: the placed bf16-MFMA kernels (csrc/attention.hip), f32
    accumulation and softmax; dh < 64 runs zero-padded to 64 (pad_heads). f32 qkv (a model run without autocast,
    whose reference einsums run in fp32, backbone_vit.py:193,200) and head dims 65..256 (the `custom` splits):
    csrc/attention_gen.hip, every product in exact f32 (bf16 I/O rounded once on the way out).
    """
    hd = qkv.shape[-1] // (3 * num_heads)
    _check_head_dim(hd, ATTN_GEN_MAX_HEAD_DIM, "attention")
    dt = qkv.dtype
    if dt != torch.bfloat16 or hd > ATTN_HEAD_DIM:
        q = qkv if dt in (torch.float32, torch.bfloat16) else qkv.float()
        o = _GenAttention.apply(q.contiguous(), num_heads, scale)
        return o if o.dtype == dt else o.to(dt)
    q = qkv
    if hd < ATTN_HEAD_DIM:
        q = pad_heads(q, 3, num_heads, ATTN_HEAD_DIM)
    o = _FlashAttention.apply(q.contiguous(), num_heads, scale)
    if hd < ATTN_HEAD_DIM:
        o = unpad_heads(o, num_heads, hd)
    return o


# ------------------------------------------------------------------------------------- patch embed
_DT = {torch.float32: 0, torch.bfloat16: 1}


def _i32arr(vals):
    import ctypes
    return (ctypes.c_int * 3)(*(list(vals) + [1] * (3 - len(vals))))


class _PatchEmbed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, pos, channels_last, out_dtype):
        B, C = x.shape[:2]
        S = list(x.shape[2:])
        D = w.shape[0]
        P = list(w.shape[2:])
        G = [-(-s // p) for s, p in zip(S, P)]
        L = 1
        for g in G:
            L *= g
        y = torch.empty((B, L, D) if channels_last else (B, D, *G), device=x.device, dtype=out_dtype)
        wf = w.float().contiguous()
        bf = bias.float().contiguous() if bias is not None else None
        pf = pos.float().reshape(L, D).contiguous() if pos is not None else None
        _lib.call("lci_patch_embed_fwd", x.data_ptr(), _DT[x.dtype], wf.data_ptr(), _lib.ptr(bf), _lib.ptr(pf),
                  y.data_ptr(), _DT[out_dtype], B, C, D, len(S), _i32arr(S), _i32arr(P), int(channels_last),
                  _lib.stream_of(x))
        ctx.save_for_backward(x)
        ctx.meta = (B, C, D, S, P, L, channels_last, w.shape, w.dtype, bias is not None, pos is not None,
                    pos.shape if pos is not None else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        B, C, D, S, P, L, cl, wshape, wdtype, has_b, has_p, pshape = ctx.meta
        dy = dy.contiguous()
        if dy.dtype not in _DT:
            dy = dy.float()
        dw = torch.zeros(wshape, device=x.device, dtype=torch.float32)
        db = torch.zeros(D, device=x.device, dtype=torch.float32) if has_b else None
        dpos = torch.empty(pshape, device=x.device, dtype=torch.float32) if has_p else None
        _lib.call("lci_patch_embed_bwd", x.data_ptr(), _DT[x.dtype], dy.data_ptr(), _DT[dy.dtype], dw.data_ptr(),
                  _lib.ptr(db), _lib.ptr(dpos), B, C, D, len(S), _i32arr(S), _i32arr(P), int(cl),
                  _lib.stream_of(x))
        if ctx.needs_input_grad[0]:
            raise NotImplementedError("patch_embed: gradient w.r.t. the input image is not provided")
        return None, dw.to(wdtype), (db if has_b else None), dpos, None, None


def patch_embed(x, weight, bias, pos, channels_last_tokens: bool):
    """Conv(k = s = patch) + bias (+ pos) via the HIP kernel.

    channels_last_tokens=True (ViT PatchEmbeddingBlock): (B, C, *S) -> (B, L, D) in f32 (the reference's
    bf16-conv + f32 pos-embed add promotes to f32). False (Swin PatchEmbed): (B, C, *S) -> (B, D, *ceil(S/p))
    in the autocast dtype when autocast is on (the reference's conv output dtype), else f32.
    """
    _lib.require_gpu(x.contiguous())
    x = x.contiguous()
    if x.dtype not in _DT:
        x = x.float()
    if channels_last_tokens:
        out_dtype = torch.float32
    else:
        out_dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else torch.float32
        if out_dtype not in _DT:
            out_dtype = torch.float32
    return _PatchEmbed.apply(x, weight, bias, pos, channels_last_tokens, out_dtype)


# ----------------------------------------------------------------------------------------- mamba
SCAN_N = 8
CKPT = 8          # = csrc/mamba.hip CKPT (backward checkpoint spacing)


def _ll_array(vals):
    import ctypes
    return (ctypes.c_longlong * len(vals))(*vals)


def _scan_chunk(L, B=1, Dx=64):
    """Chunk length (multiple of CKPT): enough chunks for ~8K waves in flight (B * ceil(Dx/64) waves per chunk),
    at least 64 steps per chunk and at most 4096 chunks (the carry passes walk the chunks sequentially)."""
    waves_per_chunk = B * (-(-Dx // 64))
    target = max(1, int(os.environ.get("LCI_SCAN_WAVES", 8192)) // waves_per_chunk)
    tc = max(64, -(-L // target), -(-L // 4096))
    return -(-tc // CKPT) * CKPT


def _bt(t):
    """(batch stride, token stride) in elements of a (B, L, C)-shaped view with unit channel stride."""
    assert t.stride(-1) == 1, "channel dimension must be contiguous"
    return t.stride(0), t.stride(1)


class _DWConvSiLUPair(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xz, wx, bx, wz, bz):
        B, L, C2 = xz.shape
        C = C2 // 2
        xs = torch.empty(B, L, C, device=xz.device, dtype=xz.dtype)
        yz = torch.empty(B, L, C2, device=xz.device, dtype=xz.dtype)
        w = [t.float().reshape(C, -1).contiguous() if t is not None else None for t in (wx, bx, wz, bz)]
        K = w[0].shape[1]
        KernelTimer.run("dwconv_silu_fwd", 0.0, xz, lambda: _lib.call(
            "lci_dwconv_silu_fwd", _DT[xz.dtype], xz.data_ptr(), w[0].data_ptr(), _lib.ptr(w[1]), w[2].data_ptr(),
            _lib.ptr(w[3]), xs.data_ptr(), yz.data_ptr(), B, L, C, K, C2, C, C2, C, _lib.stream_of(xz)))
        ctx.save_for_backward(xz, *[t for t in w if t is not None])
        ctx.meta = (bx is not None, bz is not None, wx.shape, wz.shape)
        return xs, yz

    @staticmethod
    def backward(ctx, gxs, gyz):
        xz, *ws = ctx.saved_tensors
        has_bx, has_bz, wxs, wzs = ctx.meta
        wx = ws.pop(0)
        bx = ws.pop(0) if has_bx else None
        wz = ws.pop(0)
        bz = ws.pop(0) if has_bz else None
        B, L, C2 = xz.shape
        C = C2 // 2
        K = wx.shape[1]
        gxs = torch.zeros(B, L, C, device=xz.device, dtype=xz.dtype) if gxs is None else gxs.to(xz.dtype).contiguous()
        gyz = torch.zeros(B, L, C2, device=xz.device, dtype=xz.dtype) if gyz is None else gyz.to(xz.dtype).contiguous()
        din = torch.empty_like(xz)
        rows = int(_lib.load().lci_dwconv_silu_bwd_part_rows(B, L))
        part = torch.empty(rows, 2 * C, 4, device=xz.device, dtype=torch.float32)
        KernelTimer.run("dwconv_silu_bwd", 0.0, xz, lambda: _lib.call(
            "lci_dwconv_silu_bwd", _DT[xz.dtype], xz.data_ptr(), wx.data_ptr(), _lib.ptr(bx), wz.data_ptr(),
            _lib.ptr(bz), gxs.data_ptr(), gyz.data_ptr(), din.data_ptr(), part.data_ptr(), B, L, C, K, C2, C, C2, C,
            _lib.stream_of(xz)))
        g = part.sum(0)                      # (2C, 4): dw0, dw1, dw2, db per channel (deterministic order)
        dwx, dwz = g[:C, :K].contiguous(), g[C:, :K].contiguous()
        dbx = g[:C, 3].contiguous() if has_bx else None
        dbz = g[C:, 3].contiguous() if has_bz else None
        return din, dwx.reshape(wxs), dbx, dwz.reshape(wzs), dbz


def dwconv_silu_pair(xz, wx, bx, wz, bz):
    """SiLU(depthwise conv1d(k, 'same')) of both channel halves of the channels-last in_proj output.

    xz (B, L, 2C) -> xs (B, L, C), yz (B, L, 2C) whose second half holds SiLU(conv z) (mamba.py:118-119);
    the first half of yz is left for the selective scan to fill (the reference's cat([y, z]), :136).
    """
    _lib.require_gpu(xz)
    if xz.dtype not in _DT:
        xz = xz.float()
    xs, yz = _DWConvSiLUPair.apply(xz, wx, bx, wz, bz)
    yz._lci_z_half_only = True   # its backward reads only the z half of yz's gradient (see selective_scan_cl)
    return xs, yz


class _SelectiveScanCL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, delta, A, Bm, Cm, D, delta_bias, yz, softplus=True, want_last=False):
        B, L, Dx = u.shape
        N = A.shape[1]
        ctx.bc_joint = Cm is None            # Bm = [B | C] in one (B, L, 2N) tensor: one gradient for both
        if ctx.bc_joint:
            Bm, Cm = Bm[..., :N], Bm[..., N:]
        dt = u.dtype
        tc = _scan_chunk(L, B, Dx)
        nch = -(-L // tc)
        nck = -(-L // CKPT)
        f32 = dict(device=u.device, dtype=torch.float32)
        # one chunk (the Swin recipes' window sequences, L <= 512): nothing is carried into it, so without a
        # requested final state the end-state pass and the carry are skipped (lci.h ABI 32)
        one = nch == 1 and not want_last and os.environ.get("LCI_SCAN_ONE", "1") != "0"   # (=0: A/B hook)
        xend = None if one else torch.empty(B, nch, Dx, N, **f32)
        xinit = None if one else torch.empty(B, nch, Dx, N, **f32)
        sdt = None if one else torch.empty(B, nch, Dx, **f32)
        need_grad = any(ctx.needs_input_grad)
        # states every CKPT steps for the backward's recompute, in the I/O dtype (bf16 I/O: bf16 states, half the bytes)
        ckpt = torch.empty(B, nck, Dx, N, device=u.device, dtype=dt) if need_grad else None
        Af = A.float().contiguous()
        Dv = D.float().contiguous() if D is not None else torch.zeros(Dx, **f32)
        bv = delta_bias.float().contiguous() if delta_bias is not None else torch.zeros(Dx, **f32)
        y = yz[..., :Dx]
        strides = _ll_array([*_bt(u), *_bt(delta), *_bt(Bm), *_bt(Cm), *_bt(y), 0, 0, 0, 0, 0, 0])
        es = u.element_size()   # algorithmic bytes: read u, delta, B, C; write y
        KernelTimer.run("selective_scan_fwd", float(B * L * (3 * Dx + 2 * N) * es), u, lambda: _lib.call(
            "lci_selective_scan_fwd", _DT[dt], u.data_ptr(), delta.data_ptr(), Af.data_ptr(), Bm.data_ptr(),
            Cm.data_ptr(), Dv.data_ptr(), bv.data_ptr(), y.data_ptr(), strides, B, L, Dx, N, tc, int(softplus),
            _lib.ptr(xend), _lib.ptr(xinit), _lib.ptr(sdt), _lib.ptr(ckpt), _lib.stream_of(u)))
        ctx.mark_dirty(yz)
        if need_grad:
            ctx.save_for_backward(u, delta, Af, Bm, Cm, Dv, bv, sdt, ckpt)
        ctx.tc, ctx.softplus = tc, softplus
        ctx.z_half_only = getattr(yz, "_lci_z_half_only", False)
        ctx.has_D, ctx.has_b = D is not None, delta_bias is not None
        if one:   # no final state requested (an empty placeholder output)
            last = torch.empty(0, **f32)
        else:     # final state x_L = exp(A sum(dt) over the last chunk) xinit_last + xend_last (return_last_state)
            last = torch.exp(Af[None] * sdt[:, -1, :, None]) * xinit[:, -1] + xend[:, -1]
        ctx.mark_non_differentiable(last)
        return yz, last

    @staticmethod
    def backward(ctx, gyz, _glast=None):
        u, delta, Af, Bm, Cm, Dv, bv, sdt, ckpt = ctx.saved_tensors
        B, L, Dx = u.shape
        N = Af.shape[1]
        tc = ctx.tc
        nch = -(-L // tc)
        gyz = gyz.to(u.dtype)
        if gyz.stride(-1) != 1:
            gyz = gyz.contiguous()
        dy = gyz[..., :Dx]
        f32 = dict(device=u.device, dtype=torch.float32)
        du = torch.empty_like(u)
        dd = torch.empty(B, L, Dx, device=u.device, dtype=u.dtype)
        plain = _lib.load().lci_selective_scan_bwd_plain_dbc(L, Dx, tc)   # every entry stored once: no zero fill
        dBC = (torch.empty if plain else torch.zeros)(B, L, 2 * N, **f32)
        dA = torch.zeros(Dx, N, **f32)
        dD = torch.zeros(Dx, **f32)
        db = torch.zeros(Dx, **f32)
        gl = torch.empty(B, nch, Dx, N, **f32)
        gin = torch.empty(B, nch, Dx, N, **f32)
        strides = _ll_array([*_bt(u), *_bt(delta), *_bt(Bm), *_bt(Cm), 0, 0, *_bt(dy), *_bt(du), *_bt(dd)])
        es = u.element_size()   # read u, delta, dy, B, C; write du, ddelta, dB, dC
        KernelTimer.run("selective_scan_bwd", float(B * L * (5 * Dx + 4 * N) * es), u, lambda: _lib.call(
            "lci_selective_scan_bwd", _DT[u.dtype], u.data_ptr(), delta.data_ptr(), Af.data_ptr(), Bm.data_ptr(),
            Cm.data_ptr(), Dv.data_ptr(), bv.data_ptr(), dy.data_ptr(), du.data_ptr(), dd.data_ptr(),
            dBC.data_ptr(), dA.data_ptr(), dD.data_ptr(), db.data_ptr(), strides, B, L, Dx, N, tc,
            int(ctx.softplus), _lib.ptr(sdt), ckpt.data_ptr(), gl.data_ptr(), gin.data_ptr(), _lib.stream_of(u)))
        # grad of yz: its first half was overwritten by y (zero gradient there), its second half is the SiLU(conv z)
        # operand of the out_proj input. When yz came from dwconv_silu_pair (tagged there), whose backward reads
        # only the z half (column offset C), gyz passes through as is instead of a clone + zero of the x half (a
        # full (B, L, 2 Dx) copy, 0.6 ms per C5 layer); any other producer gets the exact gradient.
        if not ctx.z_half_only:
            gyz = gyz.clone()
            gyz[..., :Dx] = 0
        if ctx.bc_joint:   # autograd casts the f32 sums to the input's bf16 (what .to(Bm.dtype) did)
            return du, dd, dA, dBC, None, dD if ctx.has_D else None, db if ctx.has_b else None, gyz, None, None
        return (du, dd, dA, dBC[..., :N].to(Bm.dtype), dBC[..., N:].to(Cm.dtype), dD if ctx.has_D else None,
                db if ctx.has_b else None, gyz, None, None)


def selective_scan_cl(u, delta, A, Bm, Cm, D, delta_bias, yz, delta_softplus=True, return_last_state=False):
    """Channels-last selective scan (mamba-ssm selective_scan_fn semantics with delta_softplus=True).

    u, delta (B, L, Dx); Bm, Cm (B, L, N) views with unit channel stride (e.g. column slices of x_proj's
    output); A (Dx, N) f32; D, delta_bias (Dx) f32; yz (B, L, 2*Dx): y is written into yz[..., :Dx] in place
    and yz is returned (the reference's cat([y, z]) target). y dtype = u dtype.
    """
    _lib.require_gpu(u, delta, yz)
    dt = u.dtype
    if dt not in _DT:
        raise _lib.LciError("selective_scan: u must be bf16 or f32")
    u = u.contiguous()
    delta = delta.to(dt)
    Bm = Bm.to(dt)
    if Bm.stride(-1) != 1:
        Bm = Bm.contiguous()
    if Cm is not None:       # Cm None: Bm is the joint (B, L, 2N) [B | C] tensor
        Cm = Cm.to(dt)
        if Cm.stride(-1) != 1:
            Cm = Cm.contiguous()
    if delta.stride(-1) != 1:
        delta = delta.contiguous()
    if yz.dtype != dt:
        raise _lib.LciError("selective_scan: yz dtype must match u")
    out, last = _SelectiveScanCL.apply(u, delta, A, Bm, Cm, D, delta_bias, yz, bool(delta_softplus),
                                       bool(return_last_state))
    return (out, last) if return_last_state else out


# --------------------------------------------------------------------- Mamba x_proj -> split -> dt_proj
_MP_IDX = {}


def _mp_dims(Dx, R, N2):
    import ctypes
    d = (ctypes.c_int * 5)()
    _lib.call("lci_mamba_proj_dims", Dx, R, N2, d)
    return tuple(int(v) for v in d)


def _mp_slot_rows(ks2, device):
    """x_dbl row feeding k-slot 16 s + 8 h + j of dt_proj's MFMA (the accumulator-pack order; include/lci.h)."""
    key = (ks2, str(device))
    t = _MP_IDX.get(key)
    if t is None:
        rows = []
        for sl in range(16 * ks2):
            st, k = sl // 16, sl % 16
            h, j = k >> 3, k & 7
            rows.append(32 * (st >> 1) + 16 * (st & 1) + (j & 3) + 8 * (j >> 2) + 4 * h)
        t = torch.tensor(rows, device=device)
        _MP_IDX[key] = t
    return t


def _mp_images(Wx, Wdt, R, N2):
    """bf16 weight images of lci_mamba_proj_fwd / _bwd from the f32 parameters (include/lci.h)."""
    RN, Dx = Wx.shape
    Dxp, nb1, ks2, nb3, ks4 = _mp_dims(Dx, R, N2)
    dev = Wx.device
    wx = Wx.detach().to(torch.bfloat16)
    wd = Wdt.detach().to(torch.bfloat16)
    w1 = torch.zeros(nb1 * 32, Dx, device=dev, dtype=torch.bfloat16)
    w1[:RN] = wx
    rows = _mp_slot_rows(ks2, dev)
    wdp = torch.zeros(Dxp, 32 * max(nb1, 2), device=dev, dtype=torch.bfloat16)
    wdp[:Dx, :R] = wd
    w2p = wdp[:, rows].contiguous()
    w2t = torch.zeros(nb3 * 32, Dx, device=dev, dtype=torch.bfloat16)
    w2t[:R] = wd.t()
    w1t = torch.zeros(Dxp, ks4 * 16, device=dev, dtype=torch.bfloat16)
    w1t[:Dx, :RN] = wx.t()
    return w1, w2p, w2t, w1t


class _MambaProj(torch.autograd.Function):
    """x_dbl = x_proj(xs); dt_low, B|C = split; dt = dt_proj(dt_low) (mamba.py:120-124) under bf16 autocast, in one
    HIP pass per direction (lci_mamba_proj_fwd / _bwd); weight gradients on lci_linear_wgrad."""

    @staticmethod
    def forward(ctx, xs, Wx, Wdt, bias, R, N2):
        Bb, L, Dx = xs.shape
        M = Bb * L
        w1, w2p, w2t, w1t = _mp_images(Wx, Wdt, R, N2)
        bf = bias.detach().to(torch.bfloat16).float().contiguous()
        b16 = dict(device=xs.device, dtype=torch.bfloat16)
        dt = torch.empty(Bb, L, Dx, **b16)
        bc = torch.empty(Bb, L, N2, **b16)
        ldl = -(-R // 8) * 8
        dtl = torch.empty(Bb, L, ldl, **b16)
        KernelTimer.run("mamba_proj_fwd", 0.0, xs, lambda: _lib.call(
            "lci_mamba_proj_fwd", xs.data_ptr(), Dx, w1.data_ptr(), w2p.data_ptr(), bf.data_ptr(), dt.data_ptr(), Dx,
            bc.data_ptr(), dtl.data_ptr(), ldl, M, Dx, R, N2, _lib.stream_of(xs)))
        ctx.save_for_backward(xs, dtl, w2t, w1t)
        ctx.meta = (R, N2, Wx.shape, Wdt.shape)
        # xs again as an output: the scan reads this alias, so its input gradient du arrives here and is added to
        # dxs inside lci_mamba_proj_bwd instead of by an autograd add of two (B, L, Dx) gradients
        return dt, bc, xs.view_as(xs)

    @staticmethod
    def backward(ctx, gdt, gbc, gu):
        xs, dtl, w2t, w1t = ctx.saved_tensors
        R, N2, wxs, wds = ctx.meta
        Bb, L, Dx = xs.shape
        M = Bb * L
        b16 = dict(device=xs.device, dtype=torch.bfloat16)
        gdt = torch.zeros(Bb, L, Dx, **b16) if gdt is None else gdt.to(torch.bfloat16).contiguous()
        gbc = torch.zeros(Bb, L, N2, **b16) if gbc is None else gbc.to(torch.bfloat16).contiguous()
        ldx = -(-(R + N2) // 8) * 8
        dxs = torch.empty(Bb, L, Dx, **b16)
        dxdbl = torch.empty(Bb, L, ldx, **b16)
        if gu is not None:
            gu = gu.to(torch.bfloat16).contiguous()
            if gu.data_ptr() % 16:
                gu = gu.clone()
        KernelTimer.run("mamba_proj_bwd", 0.0, xs, lambda: _lib.call(
            "lci_mamba_proj_bwd", gdt.data_ptr(), Dx, gbc.data_ptr(), w2t.data_ptr(), w1t.data_ptr(), _lib.ptr(gu),
            Dx if gu is not None else 0, dxs.data_ptr(), Dx, dxdbl.data_ptr(), ldx, M, Dx, R, N2,
            _lib.stream_of(xs)))
        dW, _ = _wgrad_any(dxdbl.view(M, ldx), xs.reshape(M, Dx), False)
        dWd, db = _wgrad_any(gdt.view(M, Dx), dtl.view(M, -1), True)
        return dxs, dW[:R + N2].reshape(wxs), dWd[:, :R].reshape(wds), db, None, None


def _wgrad_any(dy2, x2, bias):
    """dW = dy2^T x2 (f32) and db: the HIP split-token kernel where its tiles fit, else the GEMM (narrow shapes)."""
    if linear_wgrad_supported(dy2, x2):
        return linear_wgrad(dy2, x2, bias)
    return (dy2.t() @ x2).float(), (dy2.float().sum(0) if bias else None)


def mamba_proj_supported(xs: torch.Tensor, Dx: int, R: int, N2: int) -> bool:
    """The fused projection runs under bf16 autocast on contiguous bf16 rows of the shapes it tiles."""
    if os.environ.get("LCI_MAMBA_PROJ", "1") == "0" or not xs.is_cuda:
        return False
    if not (torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16):
        return False
    if xs.dtype != torch.bfloat16 or not xs.is_contiguous() or xs.data_ptr() % 16:
        return False
    return not (Dx % 16 or N2 % 8 or R + N2 > 64 or Dx > 1024)


def mamba_proj(xs, Wx, Wdt, bias, R, N2, with_u=False):
    """(dt (B, L, Dx) bf16, bc (B, L, 2N) bf16 = [B | C]) of MambaVisionMixer's x_proj / dt_proj (mamba.py:120-124);
    with_u: also xs itself for the scan to read, whose gradient is then summed inside the projection's backward."""
    dt, bc, u = _MambaProj.apply(xs, Wx, Wdt, bias, R, N2)
    return (dt, bc, u) if with_u else (dt, bc)


# ------------------------------------------------------------------------------------ window attention
def _i32(vals):
    import ctypes
    return (ctypes.c_int * len(vals))(*[int(v) for v in vals])


def _window_bias(rpb, mask, geo, transposed=False, plain=True):
    """(T, H, Npad, Npad) log2-domain logit term and / or its transpose: rpb + region/explicit mask, padding."""
    g = _i32(geo)
    n = int(_lib.load().lci_window_bias_elems(g, int(mask is not None)))
    if n <= 0:
        raise _lib.LciError(_lib.load().lci_last_error().decode())
    b16 = dict(device=rpb.device, dtype=torch.bfloat16)
    bias = torch.empty(n, **b16) if plain else None
    bt = torch.empty(n, **b16) if transposed else None
    _lib.call("lci_window_bias", rpb.data_ptr(), _lib.ptr(mask), _lib.ptr(bias), _lib.ptr(bt), g,
              _lib.stream_of(rpb))
    return bias, bt


class _WindowAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, bias, rpb, mask, geo, scale):
        C = qkv.shape[-1] // 3
        out = torch.empty(*qkv.shape[:-1], C, device=qkv.device, dtype=torch.bfloat16)
        g = _i32(geo)
        N, H = geo[13], geo[15]
        Bw = geo[11] * (geo[12] if geo[0] == 1 else 1)
        lse2 = torch.empty(Bw, H, N, device=qkv.device, dtype=torch.float32)
        bf = bias.float().contiguous() if bias is not None else None
        mk = mask.float().contiguous() if mask is not None else None
        rp = rpb.float().contiguous()
        _, tabT = _window_bias(rp, mk, geo, transposed=True, plain=False)   # the key-major table only
        KernelTimer.run("window_attn_fwd", 4.0 * Bw * H * N * N * 32, qkv, lambda: _lib.call(
            "lci_window_attn_fwd", qkv.data_ptr(), _lib.ptr(bf), tabT.data_ptr(), int(mk is not None), out.data_ptr(),
            lse2.data_ptr(), g, float(scale), _lib.stream_of(qkv)))
        ctx.save_for_backward(qkv, bf, rp, mk, out, lse2, tabT)   # the backward reuses the table
        ctx.geo, ctx.scale, ctx.has_bias = geo, scale, bias is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, bf, rp, mk, out, lse2, tabT = ctx.saved_tensors
        geo, scale = ctx.geo, ctx.scale
        g = _i32(geo)
        N, C, H = geo[13], geo[14], geo[15]
        Bw = lse2.shape[0]
        dout = dout.to(torch.bfloat16).contiguous()
        dqkv = torch.empty_like(qkv)
        f32 = dict(device=qkv.device, dtype=torch.float32)
        dbias = torch.zeros(3 * C, **f32) if (ctx.has_bias and ctx.needs_input_grad[1]) else None
        pad_ws = torch.empty(int(_lib.load().lci_window_pad_ws_elems(g)), **f32) if dbias is not None else None
        want_rpb = ctx.needs_input_grad[2]
        dS = drpb = None
        if want_rpb:
            n_el = _lib.load().lci_window_dS_elems(g)
            dS = torch.empty(int(n_el), device=qkv.device, dtype=torch.bfloat16)
            drpb = torch.empty(H, N, N, **f32)
        # the plain (query-major) table only for the two-phase kernel (the library says which kernel runs)
        tab = None
        if _lib.load().lci_window_bwd_needs_plain(g):
            tab, _ = _window_bias(rp, mk, geo)
        KernelTimer.run("window_attn_bwd", 8.0 * Bw * H * N * N * 32, qkv, lambda: _lib.call(
            "lci_window_attn_bwd", qkv.data_ptr(), _lib.ptr(bf), _lib.ptr(tab), tabT.data_ptr(), int(mk is not None),
            out.data_ptr(), dout.data_ptr(), lse2.data_ptr(), dqkv.data_ptr(), _lib.ptr(dbias), _lib.ptr(pad_ws),
            _lib.ptr(dS),
            _lib.ptr(drpb), g, float(scale), _lib.stream_of(qkv)))
        return dqkv, dbias, drpb, None, None, None


def _win_prep(qkv):
    dt = qkv.dtype
    q = qkv if dt == torch.bfloat16 else qkv.to(torch.bfloat16)
    return q.contiguous(), dt


def grid_geo(B, S, window_size, shift_size, C, num_heads):
    """geo[16] of the grid mode (include/lci.h) for a (B, *S, .) channels-last grid."""
    S = list(S)
    nd = len(S)
    N = 1
    for w in window_size:
        N *= w
    nW = 1
    for s, w in zip(S, window_size):
        nW *= -(-s // w)
    return (1, nd, *(S + [1] * (3 - nd)), *(list(window_size) + [1] * (3 - nd)),
            *(list(shift_size) + [0] * (3 - nd)), B, nW, N, C, num_heads)


def window_index_map(B, S, window_size, shift_size, device="cuda"):
    """The grid mode's index maps as the kernels compute them (lci_window_index_map): int32 src_row, region, rid
    (B*nW, N) and wtype (B*nW,) on `device`. See include/lci.h."""
    geo = grid_geo(B, S, window_size, shift_size, 32, 1)
    Bw, N = geo[11] * geo[12], geo[13]
    i32 = dict(device=device, dtype=torch.int32)
    src, reg, rid = (torch.empty(Bw, N, **i32) for _ in range(3))
    wt = torch.empty(Bw, **i32)
    _lib.call("lci_window_index_map", _i32(geo), src.data_ptr(), reg.data_ptr(), rid.data_ptr(), wt.data_ptr(),
              torch.cuda.current_stream(torch.device(device)).cuda_stream)
    return src, reg, rid, wt


def window_bias_table(rpb, B, S, window_size, shift_size, num_heads):
    """The (T, H, Npad, Npad) bf16 logit table lci_window_bias builds for the grid mode from rpb (H, N, N)."""
    geo = grid_geo(B, S, window_size, shift_size, 32 * num_heads, num_heads)
    tab, _ = _window_bias(rpb.float().contiguous(), None, geo)
    npad = -(-geo[13] // 32) * 32
    return tab.view(-1, num_heads, npad, npad)


def window_attention_grid(qkv, bias, rpb, num_heads, scale, window_size, shift_size):
    """Fused pad + roll(-shift) + window_partition + window attention + window_reverse + roll(+shift) + crop.

    qkv: (B, S0, S1[, S2], 3C) = qkv Linear of the LN1 output on the un-padded channels-last grid;
    bias: the qkv Linear bias (the q/k/v of padded voxels) or None; rpb: (H, N, N) = table[index].
    Returns (B, S0, S1[, S2], C) — the reference's forward_part1 output before proj (backbone_swin.py:435-487).
    """
    _lib.require_gpu(qkv.contiguous())
    q, dt = _win_prep(qkv)
    hd = q.shape[-1] // (3 * num_heads)
    _check_head_dim(hd, WIN_HEAD_DIM, "window attention")
    if hd < WIN_HEAD_DIM:   # custom Swin splits: zero-padded heads (pad_heads), the padded voxels' bias likewise
        q = pad_heads(q, 3, num_heads, WIN_HEAD_DIM).contiguous()
        bias = None if bias is None else pad_heads(bias, 3, num_heads, WIN_HEAD_DIM)
    geo = grid_geo(q.shape[0], q.shape[1:-1], window_size, shift_size, q.shape[-1] // 3, num_heads)
    o = _WindowAttention.apply(q, bias, rpb.float(), None, geo, scale)
    if hd < WIN_HEAD_DIM:
        o = unpad_heads(o, num_heads, hd)
    return o if dt == torch.bfloat16 else o.to(dt)


def _win_move(src, dst, geo, scatter):
    _lib.call("lci_window_gather", src.data_ptr(), dst.data_ptr(), src.element_size(), _i32(geo), int(scatter),
              _lib.stream_of(src))


class _WindowGather(torch.autograd.Function):
    """grid (B, *S, C) -> windows (B*nW, N, C): F.pad + roll(-shift) + window_partition; adjoint = the scatter."""

    @staticmethod
    def forward(ctx, x, geo):
        B, C = x.shape[0], x.shape[-1]
        x = x.contiguous()
        win = torch.empty(B * geo[12], geo[13], C, device=x.device, dtype=x.dtype)
        KernelTimer.run("window_gather", 0.0, x, lambda: _win_move(x, win, geo, False))
        ctx.geo, ctx.shape = geo, x.shape
        return win

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dx = torch.empty(ctx.shape, device=g.device, dtype=g.dtype)
        KernelTimer.run("window_scatter", 0.0, g, lambda: _win_move(g, dx, ctx.geo, True))
        return dx, None


class _WindowScatter(torch.autograd.Function):
    """windows (B*nW, N, C) -> grid (B, *S, C): window_reverse + roll(+shift) + crop; adjoint = the gather."""

    @staticmethod
    def forward(ctx, win, geo, shape):
        win = win.contiguous()
        out = torch.empty(shape, device=win.device, dtype=win.dtype)
        KernelTimer.run("window_scatter", 0.0, win, lambda: _win_move(win, out, geo, True))
        ctx.geo, ctx.wshape = geo, win.shape
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dw = torch.empty(ctx.wshape, device=g.device, dtype=g.dtype)
        KernelTimer.run("window_gather", 0.0, g, lambda: _win_move(g, dw, ctx.geo, False))
        return dw, None, None


def window_gather_supported(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and (x.shape[-1] * x.element_size()) % 16 == 0


def window_partition_grid(x, window_size, shift_size):
    """x (B, S0, S1[, S2], C) channels-last -> (B * nW, N, C) windows, zero rows for the padding (the reference's
    F.pad of the LayerNorm output, roll(-shift) and window_partition, backbone_swin.py:445-465)."""
    geo = grid_geo(x.shape[0], x.shape[1:-1], window_size, shift_size, x.shape[-1], 1)
    return _WindowGather.apply(x, geo)


def window_reverse_grid(win, grid_shape, window_size, shift_size):
    """(B * nW, N, C) windows -> (B, S0, S1[, S2], C): window_reverse, roll(+shift) and the crop (:469-487)."""
    geo = grid_geo(grid_shape[0], grid_shape[1:-1], window_size, shift_size, grid_shape[-1], 1)
    return _WindowScatter.apply(win, geo, tuple(grid_shape))


def window_attention(qkv, rpb, mask, num_heads, scale):
    """Pre-partitioned windows (WindowAttention.forward signature): qkv (Bw, N, 3C), mask (nW, N, N) or None."""
    _lib.require_gpu(qkv.contiguous())
    q, dt = _win_prep(qkv)
    hd = q.shape[-1] // (3 * num_heads)
    _check_head_dim(hd, WIN_HEAD_DIM, "window attention")
    if hd < WIN_HEAD_DIM:
        q = pad_heads(q, 3, num_heads, WIN_HEAD_DIM).contiguous()
    Bw, N, C3 = q.shape
    nW = mask.shape[0] if mask is not None else 1
    geo = (0, 0, 1, 1, 1, 1, 1, 1, 0, 0, 0, Bw, nW, N, C3 // 3, num_heads)
    o = _WindowAttention.apply(q, None, rpb.float(), mask, geo, scale)
    if hd < WIN_HEAD_DIM:
        o = unpad_heads(o, num_heads, hd)
    return o if dt == torch.bfloat16 else o.to(dt)


# ----------------------------------------------------------------------------------------- hyena
_TW = {}


def _twiddles(n, device):
    key = (n, str(device))
    t = _TW.get(key)
    if t is None:
        t = torch.empty(n, 2, device=device, dtype=torch.float32)
        _lib.call("lci_fft_twiddles", t.data_ptr(), n, _lib.stream_of(t))
        _TW[key] = t
    return t


def _fft_n(L):
    return int(_lib.load().lci_fft_size(int(L)))


def _spectrum(k, Dv=None):
    """Filter spectra K = FFT_n(k) / n (+ D / n: the + D u term of fftconv_ref folded into the convolution)."""
    C, L = k.shape
    n = _fft_n(L)
    tw = _twiddles(n, k.device)
    K = torch.empty(C, n, 2, device=k.device, dtype=torch.float32)
    SK = torch.empty(C, n, 2, device=k.device, dtype=torch.float32)
    KernelTimer.run("fftconv_spectrum", 0.0, k, lambda: _lib.call(
        "lci_fftconv_spectrum", k.data_ptr(), _lib.ptr(Dv), K.data_ptr(), SK.data_ptr(), tw.data_ptr(), C, L,
        _lib.stream_of(k)))
    return K


_KEEP_U_SPECTRUM = os.environ.get("LCI_FFT_KEEP_SPECTRUM", "1") != "0"


class _FFTConv(torch.autograd.Function):
    """y = causal_conv(u, k) + D u along L for rows (R, C, L) f32; filter = channel index. D rides in the filter
    spectra (K + D / n), so neither pass reads u / dy again for the D term, and dD is the lag-0 entry of dk."""

    @staticmethod
    def forward(ctx, u, k, D):
        R, C, L = u.shape
        kf = k.float().contiguous()
        Dv = D.float().contiguous()
        K = _spectrum(kf, Dv)
        n = K.shape[1]
        tw = _twiddles(n, u.device)
        y = torch.empty_like(u)
        S = torch.empty(C * ((R + 1) // 2), n, 2, device=u.device, dtype=torch.float32)
        # column spectra of u kept for the filter gradient (one column pass fewer in the backward), when k needs one
        Su = torch.empty_like(S) if (ctx.needs_input_grad[1] and _KEEP_U_SPECTRUM) else None
        KernelTimer.run("fftconv_fwd", float(R * C * L), u, lambda: _lib.call(
            "lci_fftconv_fwd", u.data_ptr(), K.data_ptr(), None, y.data_ptr(), S.data_ptr(), _lib.ptr(Su),
            tw.data_ptr(), R, C, L, _lib.stream_of(u)))
        del S
        ctx.save_for_backward(u, K, Su)
        ctx.kdtype = k.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        u, K, Su = ctx.saved_tensors
        R, C, L = u.shape
        n = K.shape[1]
        tw = _twiddles(n, u.device)
        dy = dy.float().contiguous()
        du = torch.empty_like(u)
        want_k = ctx.needs_input_grad[1]
        want_d = ctx.needs_input_grad[2]
        dk = torch.empty(C, L, device=u.device, dtype=torch.float32) if want_k else None
        dD = torch.zeros(C, device=u.device, dtype=torch.float32) if want_d else None
        P = (R + 1) // 2
        S = torch.empty(C * P, n, 2, device=u.device, dtype=torch.float32)
        S2 = torch.empty(C * P, n, 2, device=u.device, dtype=torch.float32) if (want_k and Su is None) else None
        SK = torch.empty(C, n, 2, device=u.device, dtype=torch.float32) if want_k else None
        KernelTimer.run("fftconv_bwd", float(R * C * L), u, lambda: _lib.call(
            "lci_fftconv_bwd", dy.data_ptr(), u.data_ptr(), K.data_ptr(), None, du.data_ptr(),
            _lib.ptr(dk), _lib.ptr(dD), S.data_ptr(), _lib.ptr(S2), _lib.ptr(Su if want_k else None), _lib.ptr(SK),
            tw.data_ptr(), R, C, L, _lib.stream_of(u)))
        return du, (dk.to(ctx.kdtype) if dk is not None else None), dD


_DIRECT_MAX = None


def direct_conv_max_len() -> int:
    """Longest row on the direct (Toeplitz, f32 MFMA) long-conv path; LCI_DIRECT_CONV=0 forces the FFT path."""
    global _DIRECT_MAX
    if _DIRECT_MAX is None:
        _DIRECT_MAX = int(_lib.load().lci_direct_conv_max_len()) if os.environ.get("LCI_DIRECT_CONV", "1") != "0" else 0
    return _DIRECT_MAX


class _DirectConv(torch.autograd.Function):
    """y = causal_conv(u, k) + D u for short rows (R, C, L) f32 (Swin windows): lci_direct_conv_fwd / _dk."""

    @staticmethod
    def forward(ctx, u, k, D):
        R, C, L = u.shape
        kf = k.float().contiguous()
        Dv = D.float().contiguous()
        y = torch.empty_like(u)
        fl = float(R * C) * L * (L + 1)     # algorithmic FLOPs: 2 per multiply-add of the causal (triangular) sum
        KernelTimer.run("direct_conv_fwd", fl, u, lambda: _lib.call(
            "lci_direct_conv_fwd", u.data_ptr(), kf.data_ptr(), Dv.data_ptr(), y.data_ptr(), R, C, L, 0,
            _lib.stream_of(u)))
        ctx.save_for_backward(u, kf, Dv)
        ctx.kdtype = k.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        u, kf, Dv = ctx.saved_tensors
        R, C, L = u.shape
        dy = dy.float().contiguous()
        du = torch.empty_like(u)
        fl = float(R * C) * L * (L + 1)
        KernelTimer.run("direct_conv_bwd", fl, u, lambda: _lib.call(
            "lci_direct_conv_fwd", dy.data_ptr(), kf.data_ptr(), Dv.data_ptr(), du.data_ptr(), R, C, L, 1,
            _lib.stream_of(u)))
        dk = dD = None
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            ns = int(_lib.load().lci_direct_conv_dk_splits(R, C, L))
            nt = -(-L // 32)
            part = torch.empty(ns, C, nt, 64, device=u.device, dtype=torch.float32)
            KernelTimer.run("direct_conv_dk", fl, u, lambda: _lib.call(
                "lci_direct_conv_dk", dy.data_ptr(), u.data_ptr(), part.data_ptr(), R, C, L, _lib.stream_of(u)))
            band = part.sum(0)                                     # (C, nt, 64): diagonal sums per band
            g = band[:, :, 31:63].clone()                          # lag 32 d + e from band d
            g[:, :-1, 1:] += band[:, 1:, 0:31]                     # ... and from band d + 1 (slot e - 1)
            g = g.reshape(C, nt * 32)[:, :L]
            dk = g.to(ctx.kdtype) if ctx.needs_input_grad[1] else None
            dD = g[:, 0].clone() if ctx.needs_input_grad[2] else None
        return du, dk, dD


def _long_conv(rows, k, D):
    """The long-conv autograd op for channel-major f32 rows (R, C, L): direct for short rows, FFT otherwise."""
    if rows.shape[-1] <= direct_conv_max_len():
        return _DirectConv.apply(rows, k, D)
    return _FFTConv.apply(rows, k, D)


def fftconv(u, k, D):
    """fftconv_ref (hyena.py:32-51, gelu=False): u (..., C, L), k (C, L), D (C) -> causal conv + D u, in u.dtype.

    Computed in f32 (the reference casts u to k's f32 dtype for the FFT) with the HIP four-step FFT.
    """
    _lib.require_gpu(u.contiguous(), k.contiguous())
    shp = u.shape
    C, L = shp[-2], shp[-1]
    rows = u.float().reshape(-1, C, L).contiguous()
    y = _long_conv(rows, k, D)
    return y.reshape(shp).to(u.dtype)


class _HyenaPre(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, w, b, num_heads):
        BB, L, C3 = z.shape
        D = C3 // 3
        hd = D // num_heads
        K = w.shape[-1]
        wf = w.float().reshape(C3, K).contiguous()
        bf = b.float().contiguous() if b is not None else None
        vg = torch.empty(BB, D, L, device=z.device, dtype=torch.float32)
        x2 = torch.empty(BB, L, D, device=z.device, dtype=z.dtype)
        KernelTimer.run("hyena_pre_fwd", 0.0, z, lambda: _lib.call(
            "lci_hyena_pre_fwd", _DT[z.dtype], z.data_ptr(), wf.data_ptr(), _lib.ptr(bf), vg.data_ptr(),
            x2.data_ptr(), BB, L, num_heads, hd, K, _lib.stream_of(z)))
        ctx.save_for_backward(z, wf, bf)
        ctx.meta = (num_heads, w.shape, b is not None)
        return vg, x2

    @staticmethod
    def backward(ctx, dvg, dx2):
        z, wf, bf = ctx.saved_tensors
        num_heads, wshape, has_b = ctx.meta
        BB, L, C3 = z.shape
        D = C3 // 3
        hd = D // num_heads
        K = wf.shape[1]
        f32 = dict(device=z.device, dtype=torch.float32)
        dvg = torch.zeros(BB, D, L, **f32) if dvg is None else dvg.float().contiguous()
        # dx2 in z's dtype (lci_hyena_post_bwd writes it in x2's = z's dtype: no cast either side, ABI 26)
        dx2 = (torch.zeros(BB, L, D, device=z.device, dtype=z.dtype) if dx2 is None
               else dx2.to(z.dtype).contiguous())
        dz = torch.empty_like(z)
        dw = torch.zeros(C3, K, **f32)
        db = torch.zeros(C3, **f32) if has_b else None
        KernelTimer.run("hyena_pre_bwd", 0.0, z, lambda: _lib.call(
            "lci_hyena_pre_bwd", _DT[z.dtype], z.data_ptr(), wf.data_ptr(), _lib.ptr(bf), dvg.data_ptr(),
            dx2.data_ptr(), dz.data_ptr(), dw.data_ptr(), _lib.ptr(db), BB, L, num_heads, hd, K, _lib.stream_of(z)))
        return dz, dw.reshape(wshape), db, None


class _HyenaPost(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, x2):
        BB, D, L = y.shape
        out = torch.empty(BB, L, D, device=y.device, dtype=x2.dtype)
        KernelTimer.run("hyena_post_fwd", 0.0, y, lambda: _lib.call(
            "lci_hyena_post_fwd", _DT[x2.dtype], y.data_ptr(), x2.data_ptr(), out.data_ptr(), BB, L, D,
            _lib.stream_of(y)))
        ctx.save_for_backward(y, x2)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, x2 = ctx.saved_tensors
        BB, D, L = y.shape
        dout = dout.to(x2.dtype).contiguous()
        dy = torch.empty(BB, D, L, device=y.device, dtype=torch.float32)
        dx2 = torch.empty(BB, L, D, device=y.device, dtype=x2.dtype)   # x2's dtype: the engine casts nothing
        KernelTimer.run("hyena_post_bwd", 0.0, y, lambda: _lib.call(
            "lci_hyena_post_bwd", _DT[x2.dtype], y.data_ptr(), x2.data_ptr(), dout.data_ptr(), dy.data_ptr(),
            dx2.data_ptr(), BB, L, D, _lib.stream_of(y)))
        return dy, dx2


def hyena_pre(z, weight, bias, num_heads):
    """Causal depthwise short conv of the channels-last in_proj output z (B, L, 3D) + pre-gate (hyena.py:321-333).

    Returns vg = v * x1 as channel-major f32 rows (B, D, L) for the long conv, and x2 channels-last (B, L, D).
    """
    _lib.require_gpu(z.contiguous())
    z = z.contiguous()
    if z.dtype not in _DT:
        z = z.float()
    return _HyenaPre.apply(z, weight, bias, num_heads)


def hyena_fftconv_gate(vg, k, bias, x2):
    """(causal_conv(vg, k) + bias * vg) * x2, returned channels-last (B, L, D) in x2's dtype (hyena.py:343-355)."""
    BB, D, L = vg.shape
    hd = k.shape[0]
    y = _long_conv(vg.reshape(BB * (D // hd), hd, L), k, bias).reshape(BB, D, L)
    return _HyenaPost.apply(y, x2)


def _hf_feature_of_column():
    """Feature index of each permuted column of the filter backward's (L, 64) tensors (include/lci.h)."""
    c = torch.arange(64)
    t, h, j = c >> 4, (c >> 3) & 1, c & 7
    return 32 * (t >> 1) + 16 * (t & 1) + 8 * (j >> 2) + 4 * h + (j & 3)


_HF_INV = {}


def _hf_inv(device):
    """inv[f] = permuted column holding feature f."""
    inv = _HF_INV.get(str(device))
    if inv is None:
        inv = torch.argsort(_hf_feature_of_column()).to(device)
        _HF_INV[str(device)] = inv
    return inv


class _HyenaFilter(torch.autograd.Function):
    """k (64, L) f32 = Filter.filter(L)[0].T under bf16 autocast (hyena.py:54-117,190-199), fused on the GPU.

    Forward and the data-gradient chain are one HIP kernel each (lci_hyena_filter_fwd / _bwd: MFMA layers, sin,
    modulation, dz, dfreq, db1, dW1); the three 64x64 weight gradients run on lci_linear_wgrad over the bf16
    activations / gradients the backward kernel writes. Weight and bias gradients are returned in f32 without
    autocast's bf16 rounding of the GEMM output (as kernels._Linear does); data gradients keep it.
    """

    @staticmethod
    def forward(ctx, z, W1, b1, freq, W2, b2, W3, b3, W4, t, deltas, shift, L):
        E = z.shape[-1]
        dev = z.device
        lib = _lib.load()
        img = torch.empty(int(lib.lci_hyena_filter_img_elems()), device=dev, dtype=torch.bfloat16)
        vec = torch.empty(5 * 64, device=dev, dtype=torch.float32)
        ps = [p.detach().float().contiguous() for p in (W1, b1, freq, W2, b2, W3, b3, W4, deltas)]
        st = _lib.stream_of(z)
        _lib.call("lci_hyena_filter_prep", *[p.data_ptr() for p in ps], E, img.data_ptr(), vec.data_ptr(), st)
        k = torch.empty(64, L, device=dev, dtype=torch.float32)
        KernelTimer.run("hyena_filter_fwd", 0.0, z, lambda: _lib.call(
            "lci_hyena_filter_fwd", z.data_ptr(), t.data_ptr(), img.data_ptr(), vec.data_ptr(), E, L, float(shift),
            k.data_ptr(), st))
        ctx.save_for_backward(z, t, img, vec)
        ctx.meta = (float(shift), L)
        return k

    @staticmethod
    def backward(ctx, dk):
        z, t, img, vec = ctx.saved_tensors
        shift, L = ctx.meta
        E = z.shape[-1]
        dev = z.device
        lib = _lib.load()
        dk = dk.float().contiguous()
        bufs = torch.empty(6, L, 64, device=dev, dtype=torch.bfloat16)
        dh, s3, da3, s2, da2, s1 = bufs.unbind(0)
        dz = torch.zeros_like(z)
        part = torch.empty(int(lib.lci_hyena_filter_partials(L, E)), device=dev, dtype=torch.float32)
        KernelTimer.run("hyena_filter_bwd", 0.0, z, lambda: _lib.call(
            "lci_hyena_filter_bwd", z.data_ptr(), t.data_ptr(), img.data_ptr(), vec.data_ptr(), E, L, shift,
            dk.data_ptr(), dh.data_ptr(), s3.data_ptr(), da3.data_ptr(), s2.data_ptr(), da2.data_ptr(),
            s1.data_ptr(), dz.data_ptr(), part.data_ptr(), _lib.stream_of(z)))
        sums = part.view(-1, 2 + E, 64).sum(0)
        inv = _hf_inv(dev)
        dW4, _ = linear_wgrad(dh, s3, False)
        dW3, db3 = linear_wgrad(da3, s2, True)
        dW2, db2 = linear_wgrad(da2, s1, True)
        unp = lambda w: w[inv][:, inv]   # noqa: E731
        return (dz, sums[2:].t().contiguous(), sums[0], sums[1].view(1, 64), unp(dW2), db2[inv], unp(dW3),
                db3[inv], unp(dW4), None, None, None, None)


def hyena_filter(z, W1, b1, freq, W2, b2, W3, b3, W4, t, deltas, shift, L):
    """Modulated implicit filter k (64, L) f32 (Filter.filter(L)[0].transpose(0, 1), hyena.py:190-199) for the
    default MLP (emb_dim E <= 8, order = d_model = 64, one shared Sin): z (1, >=L, E) f32 parameter rows, t (1, >=L, 1)
    positions, deltas (1, 1, 64) buffer. bf16-autocast numerics (see _HyenaFilter)."""
    _lib.require_gpu(z, t)
    return _HyenaFilter.apply(z, W1, b1, freq, W2, b2, W3, b3, W4, t, deltas, shift, int(L))


class _GELU(torch.autograd.Function):
    """nn.GELU() (erf) on a contiguous bf16 tensor: lci_gelu_fwd / _bwd, torch's arithmetic, bf16 results."""

    @staticmethod
    def forward(ctx, x):
        y = torch.empty_like(x)
        KernelTimer.run("gelu_fwd", 2.0 * x.element_size() * x.numel(), x, lambda: _lib.call(
            "lci_gelu_fwd", x.data_ptr(), y.data_ptr(), x.numel(), _lib.stream_of(x)))
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous()
        if dy.data_ptr() % 16:          # a contiguous view at a storage offset: the kernel needs 16-byte vectors
            dy = dy.clone()
        dx = torch.empty_like(x)
        KernelTimer.run("gelu_bwd", 3.0 * x.element_size() * x.numel(), x, lambda: _lib.call(
            "lci_gelu_bwd", x.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), _lib.stream_of(x)))
        return dx


def gelu_supported(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0 and x.numel() > 0
            and x.data_ptr() % 16 == 0)


def gelu(x: torch.Tensor) -> torch.Tensor:
    """F.gelu(x) (approximate='none') for contiguous bf16 CUDA tensors on the HIP kernels."""
    return _GELU.apply(x)


class _Upsample2x(torch.autograd.Function):
    """F.interpolate(x, size=2x, mode="bilinear") (align_corners=False) returned as the bf16 channels-last operand of
    the next conv (what that conv's autocast cast produces), adjoint by gather (lci_upsample2x_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, x):
        B, C, H, W = x.shape
        nhwc = x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)
        y = torch.empty(B, 2 * H, 2 * W, C, device=x.device, dtype=torch.bfloat16)
        if nhwc:   # channels-last input map: read it in place
            xf = x.float().permute(0, 2, 3, 1).contiguous()
            KernelTimer.run("upsample2x_fwd", 0.0, x, lambda: _lib.call(
                "lci_upsample2x_nhwc_fwd", xf.data_ptr(), y.data_ptr(), B, C, H, W, _lib.stream_of(x)))
        else:
            xf = x.float().contiguous()
            KernelTimer.run("upsample2x_fwd", 0.0, x, lambda: _lib.call(
                "lci_upsample2x_fwd", xf.data_ptr(), y.data_ptr(), B, C, H, W, _lib.stream_of(x)))
        ctx.shape = (B, C, H, W)
        ctx.xdtype = x.dtype
        ctx.nhwc = nhwc
        return y.permute(0, 3, 1, 2)                      # (B, C, 2H, 2W), channels-last strides

    @staticmethod
    def backward(ctx, dy):
        B, C, H, W = ctx.shape
        g = dy.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()
        if ctx.nhwc:
            dx = torch.empty(B, H, W, C, device=dy.device, dtype=torch.float32)
            KernelTimer.run("upsample2x_bwd", 0.0, dy, lambda: _lib.call(
                "lci_upsample2x_nhwc_bwd", g.data_ptr(), dx.data_ptr(), B, C, H, W, _lib.stream_of(dy)))
            return dx.permute(0, 3, 1, 2).to(ctx.xdtype)
        dx = torch.empty(B, C, H, W, device=dy.device, dtype=torch.float32)
        KernelTimer.run("upsample2x_bwd", 0.0, dy, lambda: _lib.call(
            "lci_upsample2x_bwd", g.data_ptr(), dx.data_ptr(), B, C, H, W, _lib.stream_of(dy)))
        return dx.to(ctx.xdtype)


def upsample2x_supported(x: torch.Tensor, size) -> bool:
    return (x.is_cuda and x.dim() == 4 and tuple(size) == (2 * x.shape[2], 2 * x.shape[3]) and x.shape[1] % 8 == 0
            and x.dtype in (torch.float32, torch.bfloat16))


def upsample2x_bilinear_cl(x: torch.Tensor) -> torch.Tensor:
    """Bilinear 2x up-sampling, align_corners=False (seg_heads.py:138), as bf16 with channels-last strides."""
    if not x.is_cuda:
        raise _lib.LciError("upsample2x runs on the GPU only; there is no CPU path")
    return _Upsample2x.apply(x)


class _Upsample3d(torch.autograd.Function):
    """F.interpolate(x, size, mode="trilinear") (align_corners=False) returned as the bf16 channels-last operand of the
    next conv (lci_upsample3d_cl_fwd); the adjoint one axis at a time (lci_resample1d_adj, deterministic gathers)
    instead of torch's atomic scatter (upsample_trilinear3d_backward: 136 ms per Swin-UperNet3D step at 128^3)."""

    @staticmethod
    def forward(ctx, x, size):
        B, C, D, H, W = x.shape
        OD, OH, OW = size
        xf = x.float().permute(0, 2, 3, 4, 1).contiguous()
        y = torch.empty(B, OD, OH, OW, C, device=x.device, dtype=torch.bfloat16)
        KernelTimer.run("upsample3d_fwd", 0.0, x, lambda: _lib.call(
            "lci_upsample3d_cl_fwd", xf.data_ptr(), y.data_ptr(), B, C, D, H, W, OD, OH, OW, _lib.stream_of(x)))
        ctx.shape, ctx.xdtype = (B, C, D, H, W, OD, OH, OW), x.dtype
        return y.permute(0, 4, 1, 2, 3)                   # (B, C, OD, OH, OW), channels-last strides

    @staticmethod
    def backward(ctx, dy):
        B, C, D, H, W, OD, OH, OW = ctx.shape
        g = dy.permute(0, 2, 3, 4, 1)
        if g.dtype not in (torch.bfloat16, torch.float32):
            g = g.float()
        g = g.contiguous()
        f32 = dict(device=dy.device, dtype=torch.float32)
        st = _lib.stream_of(dy)

        def adj(src, outer, n_out, n_in, inner):
            out = torch.empty(outer * n_in * inner, **f32)
            KernelTimer.run("upsample3d_bwd", 0.0, dy, lambda: _lib.call(
                "lci_resample1d_adj", src.data_ptr(), int(src.dtype == torch.bfloat16), out.data_ptr(), outer, n_out,
                n_in, inner, st))
            return out

        t = adj(g, B, OD, D, OH * OW * C)                       # (B, D, OH, OW, C)
        t = adj(t, B * D, OH, H, OW * C)                        # (B, D, H, OW, C)
        t = adj(t, B * D * H, OW, W, C)                         # (B, D, H, W, C)
        return t.view(B, D, H, W, C).permute(0, 4, 1, 2, 3).to(ctx.xdtype), None


class _ResampleCL(torch.autograd.Function):
    """F.interpolate(x, size, mode=(bi|tri)linear, align_corners=ac) [+ add] in f32 (what autocast's fp32 interpolate
    returns) with channels-last strides: lci_resample_cl_fwd, one pass, the addend summed in it; the adjoint one axis
    at a time (lci_resample1d_adj_ac, deterministic gathers) instead of torch's atomic upsample backward
    (upsample_bilinear2d_backward at C4's FPN, 514^2 -> 512^2 x 384 channels: 3.2 ms per call)."""

    @staticmethod
    def forward(ctx, x, add, size, ac):
        nd = x.dim() - 2
        B, C = x.shape[:2]
        S, OS = tuple(x.shape[2:]), tuple(int(s) for s in size)
        xl = x.movedim(1, -1)
        if xl.dtype not in (torch.bfloat16, torch.float32):
            xl = xl.float()
        xl = xl.contiguous()
        al = None
        if add is not None:
            al = add.movedim(1, -1)
            if al.dtype not in (torch.bfloat16, torch.float32):
                al = al.float()
            al = al.contiguous()
        D, H, W = (1,) + S if nd == 2 else S
        OD, OH, OW = (1,) + OS if nd == 2 else OS
        y = torch.empty(B, *OS, C, device=x.device, dtype=torch.float32)
        KernelTimer.run("resample_fwd", 0.0, x, lambda: _lib.call(
            "lci_resample_cl_fwd", xl.data_ptr(), int(xl.dtype == torch.bfloat16), _lib.ptr(al),
            int(al is not None and al.dtype == torch.bfloat16), y.data_ptr(), B, C, D, H, W, OD, OH, OW, int(ac),
            _lib.stream_of(x)))
        ctx.meta = (nd, B, C, S, OS, int(ac), x.dtype, add.dtype if add is not None else None)
        return y.movedim(-1, 1)

    @staticmethod
    def backward(ctx, dy):
        nd, B, C, S, OS, ac, xdtype, adtype = ctx.meta
        g = dy.movedim(1, -1)
        if g.dtype not in (torch.bfloat16, torch.float32):
            g = g.float()
        g = g.contiguous()
        st = _lib.stream_of(dy)
        dx = None
        if ctx.needs_input_grad[0]:
            # axis k of the (B, *spatial, C) map: outer = B * (axes before, already at input size), inner = (axes
            # after, still at output size) * C; an axis whose size does not change is the identity (skipped)
            t = g
            cur = list(OS)
            for k in range(nd):
                if S[k] == OS[k]:
                    continue
                outer = B
                for j in range(k):
                    outer *= S[j]
                inner = C
                for j in range(k + 1, nd):
                    inner *= cur[j]
                out = torch.empty(outer * S[k] * inner, device=dy.device, dtype=torch.float32)
                src = t
                KernelTimer.run("resample_bwd", 0.0, dy, lambda: _lib.call(
                    "lci_resample1d_adj_ac", src.data_ptr(), int(src.dtype == torch.bfloat16), out.data_ptr(), outer,
                    OS[k], S[k], inner, ac, st))
                t = out
                cur[k] = S[k]
            dx = t.view(B, *S, C).movedim(-1, 1)
            dx = dx.to(xdtype) if dx.dtype != xdtype else dx
        da = None
        if adtype is not None and ctx.needs_input_grad[1]:
            da = dy if dy.dtype == adtype else dy.to(adtype)
        return dx, da, None, None


def resample_cl_supported(x: torch.Tensor, size, add: torch.Tensor | None = None) -> bool:
    """lci_resample_cl_fwd takes 4-D / 5-D GPU maps with C % 8 == 0 (any strides: made channels-last contiguous)."""
    if not (x.is_cuda and x.dim() in (4, 5) and len(size) == x.dim() - 2 and x.shape[1] % 8 == 0):
        return False
    if (x.shape[0] * (int(size[0]) if x.dim() == 5 else 1) > 65535) or int(size[-2]) > 65535:   # grid y / z
        return False
    return add is None or (add.is_cuda and tuple(add.shape) == tuple(x.shape[:2]) + tuple(int(s) for s in size))


def resample_cl(x: torch.Tensor, size, align_corners: bool, add: torch.Tensor | None = None) -> torch.Tensor:
    """F.interpolate(x, size, mode='bilinear' (4-D) / 'trilinear' (5-D), align_corners) [+ add], f32 with
    channels-last strides (csrc/resample.hip)."""
    if not x.is_cuda:
        raise _lib.LciError("resample runs on the GPU only; there is no CPU path")
    return _ResampleCL.apply(x, add, tuple(int(s) for s in size), bool(align_corners))


def upsample3d_supported(x: torch.Tensor, size) -> bool:
    return (x.is_cuda and x.dim() == 5 and len(size) == 3 and x.shape[1] % 8 == 0
            and x.dtype in (torch.float32, torch.bfloat16))


def upsample3d_trilinear_cl(x: torch.Tensor, size) -> torch.Tensor:
    """Trilinear up-sampling to `size`, align_corners=False (seg_heads.py:273), as bf16 with channels-last strides."""
    if not x.is_cuda:
        raise _lib.LciError("upsample3d runs on the GPU only; there is no CPU path")
    return _Upsample3d.apply(x, tuple(int(s) for s in size))


# ------------------------------------------------------- transposed-conv (kernel == stride) output interleave
class _ConvUpInterleave(torch.autograd.Function):
    """Y (V, taps*C) bf16 -> channels-last (B, D*kd, H*kh, W*kw, C) [cat with `skip` (B, .., Cs) along channels];
    adjoint: the same rows gathered back (lci_convup_interleave)."""

    @staticmethod
    def forward(ctx, y2, skip, geo):
        B, D, H, W, kd, kh, kw, C = geo
        Cs = skip.shape[-1] if skip is not None else 0
        out = torch.empty(B, D * kd, H * kh, W * kw, C + Cs, device=y2.device, dtype=torch.bfloat16)
        KernelTimer.run("convup_interleave", 0.0, y2, lambda: _lib.call(
            "lci_convup_interleave", y2.data_ptr(), out.data_ptr(), B, D, H, W, kd, kh, kw, C, C + Cs, 0,
            _lib.stream_of(y2)))
        if skip is not None:
            out[..., C:].copy_(skip)
        ctx.geo, ctx.Cs = geo, Cs
        return out

    @staticmethod
    def backward(ctx, g):
        B, D, H, W, kd, kh, kw, C = ctx.geo
        g = g.to(torch.bfloat16).contiguous()
        dy = torch.empty(B * D * H * W, kd * kh * kw * C, device=g.device, dtype=torch.bfloat16)
        KernelTimer.run("convup_interleave", 0.0, g, lambda: _lib.call(
            "lci_convup_interleave", g.data_ptr(), dy.data_ptr(), B, D, H, W, kd, kh, kw, C, C + ctx.Cs, 1,
            _lib.stream_of(g)))
        return dy, (g[..., C:] if ctx.Cs else None), None


def convup_interleave_supported(y2: torch.Tensor, C: int, skip: torch.Tensor | None = None) -> bool:
    ok = (y2.is_cuda and y2.dtype == torch.bfloat16 and y2.is_contiguous() and y2.data_ptr() % 16 == 0
          and C % 8 == 0)
    if skip is not None:
        ok = ok and skip.dtype == torch.bfloat16 and skip.shape[-1] % 8 == 0
    return ok


def convup_interleave(y2: torch.Tensor, B: int, S, k, C: int, skip: torch.Tensor | None = None) -> torch.Tensor:
    """The up-sampling GEMM output y2 (B*prod(S), prod(k)*C) as the channels-last grid (B, *(S*k), C [+ Cs]); with
    skip (B, *(S*k), Cs) channels-last, torch.cat((up, skip), channels) in the same pass (UnetrUpBlock)."""
    S3 = list(S) + [1] * (3 - len(S))
    k3 = list(k) + [1] * (3 - len(k))
    if len(S) == 2:   # 2-D: (H, W) -> D = 1 (the skip too, as a view, so its gradient keeps its 4-D shape)
        S3, k3 = [1] + list(S), [1] + list(k)
        if skip is not None:
            skip = skip.unsqueeze(1)
    geo = (B, *S3, *k3, C)
    out = _ConvUpInterleave.apply(y2, skip, geo)
    return out.view(B, *(s * kk for s, kk in zip(S, k)), -1)


# ------------------------------------------------------------------- decoder-head 3x3(x3) convolution
def conv3_cl(x_cl: torch.Tensor, w_packed: torch.Tensor, kd: int) -> torch.Tensor:
    """x_cl (B, D, H, W, Cin) bf16 channels-last, w_packed (Cout, kd*9, Cin) bf16 -> (B, D, H, W, Cout) bf16."""
    _lib.require_gpu(x_cl, w_packed)
    B, D, H, W, Cin = x_cl.shape
    Cout = w_packed.shape[0]
    y = torch.empty(B, D, H, W, Cout, device=x_cl.device, dtype=torch.bfloat16)
    V = B * D * H * W
    ns = int(_lib.load().lci_conv3_fwd_splits(V, Cin, Cout, kd))
    if ns > 1:   # small volume: split-K with f32 partials (lci_conv3_fwd_split)
        part = torch.empty(ns, V, Cout, device=x_cl.device, dtype=torch.float32)
        KernelTimer.run("conv3", 2.0 * V * Cout * Cin * kd * 9, x_cl, lambda: _lib.call(
            "lci_conv3_fwd_split", x_cl.data_ptr(), w_packed.data_ptr(), y.data_ptr(), part.data_ptr(), ns, B, D, H,
            W, Cin, Cout, kd, _lib.stream_of(x_cl)))
        return y
    KernelTimer.run("conv3", 2.0 * V * Cout * Cin * kd * 9, x_cl, lambda: _lib.call(
        "lci_conv3_fwd", x_cl.data_ptr(), w_packed.data_ptr(), y.data_ptr(), B, D, H, W, Cin, Cout, kd,
        _lib.stream_of(x_cl)))
    return y


def _to_cl(x: torch.Tensor, nd: int) -> torch.Tensor:
    """(B, C, [D,] H, W) any layout/dtype -> (B, D, H, W, C) bf16 contiguous (D = 1 for 2-D): one copy at most."""
    if nd == 2:
        x = x.unsqueeze(2)
    return x.permute(0, 2, 3, 4, 1).to(torch.bfloat16).contiguous()


def _from_cl(y: torch.Tensor, nd: int) -> torch.Tensor:
    """(B, D, H, W, C) -> (B, C, [D,] H, W) view (channels-last strides)."""
    y = y.permute(0, 4, 1, 2, 3)
    return y.squeeze(2) if nd == 2 else y


def _conv3_wgrad(x_cl: torch.Tensor, dy_cl: torch.Tensor, kd: int) -> torch.Tensor:
    """dW (Cout, Cin, [3,] 3, 3) f32 = sum_p x[p + off(tap)] (x) dy[p], as kd*9 GEMMs over flat-shifted rows.

    Both volumes are zero-padded by one voxel per convolved axis and flattened to rows; for tap offset o the
    rows p in [s, Np - s) of dy_pad pair with rows p + o of x_pad (border rows of dy_pad are zero, so rows whose
    neighbour wraps into another line / sample contribute nothing). Each tap is one (Cin x n) . (n x Cout)
    GEMM with f32 output (hipBLASLt, bf16 inputs, f32 accumulation).
    """
    B, D, H, W, Cin = x_cl.shape
    Cout = dy_cl.shape[-1]
    pz = 1 if kd == 3 else 0
    xp = torch.nn.functional.pad(x_cl, (0, 0, 1, 1, 1, 1, pz, pz))
    dp = torch.nn.functional.pad(dy_cl, (0, 0, 1, 1, 1, 1, pz, pz))
    Pd, Ph, Pw = D + 2 * pz, H + 2, W + 2
    X = xp.view(-1, Cin)
    Y = dp.view(-1, Cout)
    s = pz * Ph * Pw + Pw + 1
    n = X.shape[0] - 2 * s
    G = torch.empty(kd * 9, Cin, Cout, device=x_cl.device, dtype=torch.float32)
    Ys = Y[s:s + n]
    t = 0
    for a in range(kd):
        for b in range(3):
            for c in range(3):
                o = ((a - 1) if kd == 3 else 0) * Ph * Pw + (b - 1) * Pw + (c - 1)
                if X.is_cuda:
                    G[t] = torch.mm(X[s + o:s + o + n].t(), Ys, out_dtype=torch.float32)
                else:   # host check of the row-shift algebra (tests); the HIP conv itself has no CPU path
                    G[t] = X[s + o:s + o + n].t().float() @ Ys.float()
                t += 1
    dw = G.permute(2, 1, 0)                                       # (Cout, Cin, taps)
    return dw.reshape(Cout, Cin, *((3, 3, 3) if kd == 3 else (3, 3)))


def conv3_wgrad_cl(x_cl: torch.Tensor, dy_cl: torch.Tensor, kd: int) -> torch.Tensor:
    """dW (Cout, Cin, [3,] 3, 3) f32 by the HIP split-voxel kernel (per-split partials summed here).
    Cin is zero-padded to a multiple of 32 (the 1-channel image of encoder1) and sliced off again."""
    _lib.require_gpu(x_cl, dy_cl)
    B, D, H, W, Cin = x_cl.shape
    Cout = dy_cl.shape[-1]
    if Cin <= 2:
        # the image into encoder1 (Cin = 1): padding Cin to 32 left 31/32 of the kernel's MFMAs on zeros (0.77 ms at
        # 128^3); as a GEMM over the (V, taps*Cin) im2col rows it is the token-wise weight gradient instead
        T = kd * 9
        pz = 1 if kd == 3 else 0
        xp = torch.nn.functional.pad(x_cl, (0, 0, 1, 1, 1, 1, pz, pz))
        cols = [xp[:, a:a + D, b:b + H, c:c + W, :] for a in range(kd) for b in range(3) for c in range(3)]
        K = -(-(T * Cin) // 32) * 32
        im = torch.zeros(B * D * H * W, K, device=x_cl.device, dtype=torch.bfloat16)
        im[:, :T * Cin].view(B, D, H, W, Cin, T).copy_(torch.stack(cols, -1))   # column c * T + tap
        dw, _ = _wgrad_any(dy_cl.reshape(-1, Cout), im, False)                  # (Cout, K) f32
        return dw[:, :T * Cin].reshape(Cout, Cin, *((3, 3, 3) if kd == 3 else (3, 3)))
    cp = -(-Cin // 32) * 32
    xp = x_cl if cp == Cin else torch.nn.functional.pad(x_cl, (0, cp - Cin))
    lib = _lib.load()
    ns = lib.lci_conv3_wgrad_splits(B * D * H * W, cp, Cout, kd)
    part = torch.empty(ns, kd * 9, Cout, cp, device=x_cl.device, dtype=torch.float32)
    KernelTimer.run("conv3_wgrad", 2.0 * B * D * H * W * Cout * Cin * kd * 9, x_cl, lambda: _lib.call(
        "lci_conv3_wgrad", xp.data_ptr(), dy_cl.data_ptr(), part.data_ptr(), B, D, H, W, cp, Cout, kd,
        _lib.stream_of(x_cl)))
    g = (part[0] if ns == 1 else part.sum(0))[..., :Cin]         # (taps, Cout, Cin)
    return g.permute(1, 2, 0).reshape(Cout, Cin, *((3, 3, 3) if kd == 3 else (3, 3)))


def _conv3_pack(weight: torch.Tensor, kd: int, mode: int, cin_pad: int) -> torch.Tensor:
    """bf16 kernel operand of a Conv{2,3}d weight (Cout, Cin, [3,] 3, 3): mode 0 (Cout, T, Cin) for the forward,
    mode 1 (cin_pad, T, Cout) flipped + transposed for the data gradient (lci_conv3_pack_weight on f32 weights)."""
    Cout, Cin = weight.shape[:2]
    T = kd * 9
    if weight.dtype == torch.float32 and weight.is_cuda:
        w = weight.detach().contiguous()
        out = torch.empty((Cout, T, Cin) if mode == 0 else (cin_pad, T, Cout), device=w.device, dtype=torch.bfloat16)
        _lib.call("lci_conv3_pack_weight", w.data_ptr(), out.data_ptr(), Cout, Cin, kd, mode, cin_pad,
                  _lib.stream_of(w))
        return out
    nd = weight.dim() - 2
    sp = tuple(range(2, 2 + nd))
    if mode == 0:
        return weight.to(torch.bfloat16).permute(0, *sp, 1).reshape(Cout, T, Cin).contiguous()
    wd = weight.to(torch.bfloat16).flip(sp).permute(1, *sp, 0).reshape(Cin, T, Cout)
    if cin_pad != Cin:
        wd = torch.cat([wd, wd.new_zeros(cin_pad - Cin, T, Cout)])
    return wd.contiguous()


class _Conv3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, nd):
        kd = 3 if nd == 3 else 1
        Cout, Cin = weight.shape[:2]
        x_cl = _to_cl(x, nd)
        wp = _conv3_pack(weight, kd, 0, Cin)
        y = conv3_cl(x_cl, wp, kd)
        ctx.save_for_backward(x_cl, weight)
        ctx.nd = nd
        return _from_cl(y, nd)

    @staticmethod
    def backward(ctx, dy):
        x_cl, weight = ctx.saved_tensors
        nd = ctx.nd
        kd = 3 if nd == 3 else 1
        Cout, Cin = weight.shape[:2]
        dy_cl = _to_cl(dy, nd)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            cp = -(-Cin // 32) * 32                      # the kernel's Cout multiple: zero rows, sliced off
            wd = _conv3_pack(weight, kd, 1, cp)
            dx = conv3_cl(dy_cl, wd, kd)
            dx = _from_cl(dx if cp == Cin else dx[..., :Cin], nd)
        if ctx.needs_input_grad[1]:
            dw = conv3_wgrad_cl(x_cl, dy_cl, kd).to(weight.dtype)
        return dx, dw, None


def conv3(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """Conv{2,3}d(kernel 3, stride 1, padding 1) in bf16 MFMA with f32 accumulation (the dtype autocast gives
    the reference's conv). x (B, Cin, [D,] H, W) -> (B, Cout, [D,] H, W) bf16, channels-last strides.
    Cout not a multiple of 32 (a head's class count) runs on zero-padded weight rows and is sliced back."""
    _lib.require_gpu(weight)
    if not x.is_cuda:
        raise _lib.LciError("conv3 runs on the GPU only; there is no CPU path")
    cout = weight.shape[0]
    cp = -(-cout // 32) * 32
    w = weight if cp == cout else torch.cat([weight, weight.new_zeros(cp - cout, *weight.shape[1:])])
    y = _Conv3.apply(x, w, weight.dim() - 2)
    if cp != cout:
        y = y[:, :cout]
    if bias is not None:
        y = y + bias.to(y.dtype).view(1, -1, *([1] * (y.dim() - 2)))
    return y


class _ResConvs(torch.autograd.Function):
    """UnetResBlock's conv1 (3x3[x3], stride 1, no bias) and conv3 (1x1 residual projection, no bias) of the same
    input (MONAI-1.3 UnetResBlock via enhance_heads.py:30-356) as one node: the forward is conv3_cl and the 1x1 GEMM
    as before; the backward computes conv1's data gradient and adds conv3's (dr . W3) into it with the GEMM itself
    (addmm_, beta = 1) instead of autograd summing two full-resolution gradients (C5's 512-channel 256^3 input: 8.6 GB
    per pass). That sum is rounded once (the unfused path rounds dr . W3 to bf16 first: <= 1 bf16 ulp apart)."""

    @staticmethod
    def forward(ctx, x, w1, w3, nd):
        kd = 3 if nd == 3 else 1
        Cin = w1.shape[1]
        x_cl = _to_cl(x, nd)
        c1 = conv3_cl(x_cl, _conv3_pack(w1, kd, 0, Cin), kd)
        x2 = x_cl.view(-1, Cin)
        w3b = w3.reshape(w3.shape[0], Cin).to(torch.bfloat16)
        N3 = w3b.shape[0]
        if HIP_GEMM and gemm_bt_preferred(x2.shape[0], N3) and gemm_bt_supported(x2, N3, Cin):
            r2 = gemm_bt(x2, w3b)
        elif SMALL_GEMM and gemm_small_supported(x2, N3, Cin):
            r2 = gemm_small(x2, w3b)
        else:
            with torch.autocast("cuda", enabled=False):
                r2 = torch.nn.functional.linear(x2, w3b)
        ctx.save_for_backward(x_cl, w1, w3b)
        ctx.nd, ctx.w3shape, ctx.w3dtype = nd, w3.shape, w3.dtype
        return _from_cl(c1, nd), _from_cl(r2.view(*x_cl.shape[:-1], N3), nd)

    @staticmethod
    def backward(ctx, dc1, dr):
        x_cl, w1, w3b = ctx.saved_tensors
        nd = ctx.nd
        kd = 3 if nd == 3 else 1
        Cin = w1.shape[1]
        N3 = w3b.shape[0]
        dy_cl = _to_cl(dc1, nd) if dc1 is not None else None
        dr2 = _to_cl(dr, nd).view(-1, N3) if dr is not None else None
        dx = dw1 = dw3 = None
        if ctx.needs_input_grad[0] and (dy_cl is not None or dr2 is not None):
            if dy_cl is not None:
                dx = conv3_cl(dy_cl, _conv3_pack(w1, kd, 1, Cin), kd)      # (B, D, H, W, Cin) bf16
                if dr2 is not None:
                    dx2 = dx.view(-1, Cin)
                    if HIP_GEMM and gemm_bt_preferred(dr2.shape[0], Cin) and gemm_bt_supported(dr2, Cin, N3):
                        # += bf16(dr . W3) in lci_gemm_bt's epilogue: the autograd sum's own roundings
                        w3t = w3b.t().contiguous()
                        KernelTimer.run("gemm_bt", 2.0 * dr2.shape[0] * Cin * N3, dr2, lambda: _lib.call(
                            "lci_gemm_bt_acc", dr2.data_ptr(), dr2.stride(0), w3t.data_ptr(), dx2.data_ptr(), Cin,
                            dr2.shape[0], Cin, N3, _lib.stream_of(dr2)))
                    elif SMALL_GEMM and gemm_small_supported(dr2, Cin, N3):
                        gemm_small(dr2, w3b.t(), out=dx2)                  # += bf16(dr . W3), as lci_gemm_bt_acc
                    else:
                        dx2.addmm_(dr2, w3b)                                 # += dr . W3 in the GEMM (beta = 1)
            elif SMALL_GEMM and gemm_small_supported(dr2, Cin, N3):
                dx = gemm_small(dr2, w3b.t()).view(*x_cl.shape)
            else:
                dx = (dr2 @ w3b).view(*x_cl.shape)
            dx = _from_cl(dx, nd)
        if ctx.needs_input_grad[1] and dy_cl is not None:
            dw1 = conv3_wgrad_cl(x_cl, dy_cl, kd).to(w1.dtype)
        if ctx.needs_input_grad[2] and dr2 is not None:
            x2 = x_cl.view(-1, Cin)
            if linear_wgrad_supported(dr2, x2):
                dw3, _ = linear_wgrad(dr2, x2, False)
            else:
                dw3 = (dr2.t() @ x2).float()
            dw3 = dw3.reshape(ctx.w3shape).to(ctx.w3dtype)
        return dx, dw1, dw3, None


def res_convs_supported(x: torch.Tensor, w1: torch.Tensor, w3: torch.Tensor) -> bool:
    """_ResConvs takes GPU maps whose conv channel counts are multiples of 32 (the UNETR decoder blocks)."""
    return (x.is_cuda and w1.shape[0] % 32 == 0 and w1.shape[1] % 32 == 0 and w3.shape[0] == w1.shape[0]
            and w3.shape[1] == w1.shape[1] and all(k == 1 for k in w3.shape[2:]) and x.shape[1] == w1.shape[1])


def res_convs(x: torch.Tensor, w1: torch.Tensor, w3: torch.Tensor):
    """(conv3x3(x, w1), conv1x1(x, w3)) in bf16, channels-last strides; one backward node (see _ResConvs)."""
    return _ResConvs.apply(x, w1, w3, w1.dim() - 2)


# ------------------------------------------------------- decoder-head instance norm (+ LeakyReLU), channels-last
INORM_EPS = 1e-5
LRELU_SLOPE = 0.01


def _inorm_sums(x_cl, dz_cl, stats, act, mode):
    """(B, 2, C) f32 from the voxel sums (lci_inorm_reduce partials, combined in f64 by lci_inorm_finalize):
    mode 0 the stats (mean, rstd) of x; mode 1 the voxel means of (dn, dn * n) for the backward."""
    B, V, C = x_cl.shape
    lib = _lib.load()
    nch = lib.lci_inorm_chunks(V, B)
    part = torch.empty(B, 2, C, nch, device=x_cl.device, dtype=torch.float32)
    out = torch.empty(B, 2, C, device=x_cl.device, dtype=torch.float32)
    st = _lib.stream_of(x_cl)
    _lib.call("lci_inorm_reduce", x_cl.data_ptr(), _lib.ptr(dz_cl), _lib.ptr(stats), part.data_ptr(), V, B, C,
              int(act), LRELU_SLOPE, st)
    _lib.call("lci_inorm_finalize", part.data_ptr(), out.data_ptr(), V, B, C, mode, INORM_EPS, st)
    return out


class _BatchNormReLU(torch.autograd.Function):
    """relu(batch_norm(x)) in training mode over x_cl (V, C) bf16 = every voxel of the batch, f32 out (autocast's
    fp32 batch_norm): statistics by the instance-norm reduction with the batch as one sample, the affine map + ReLU
    and the backward by lci_bn_relu_*. Returns (y, stats) -- stats (1, 2, C) = (mean, rstd) for the running-stat
    update."""

    @staticmethod
    def forward(ctx, x_cl, w, b):
        V, C = x_cl.shape
        stats = _inorm_stats(x_cl.view(1, V, C), False)
        y = torch.empty(V, C, device=x_cl.device, dtype=torch.float32)
        KernelTimer.run("bn_relu_fwd", 0.0, x_cl, lambda: _lib.call(
            "lci_bn_relu_fwd", x_cl.data_ptr(), stats.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), V, C,
            _lib.stream_of(x_cl)))
        ctx.save_for_backward(x_cl, stats, w, b)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x_cl, stats, w, b = ctx.saved_tensors
        V, C = x_cl.shape
        g = dy if dy.dtype in (torch.float32, torch.bfloat16) else dy.float()
        g = g.contiguous()
        if g.data_ptr() % 16:
            g = g.clone()
        f32 = int(g.dtype == torch.float32)
        lib = _lib.load()
        st = _lib.stream_of(x_cl)
        part = torch.empty(2, C, lib.lci_inorm_chunks(V, 1), device=x_cl.device, dtype=torch.float32)
        coef = torch.empty(1, 2, C, device=x_cl.device, dtype=torch.float32)
        dx = torch.empty_like(x_cl)
        KernelTimer.run("bn_relu_bwd", 0.0, x_cl, lambda: (
            _lib.call("lci_bn_relu_bwd_reduce", x_cl.data_ptr(), g.data_ptr(), f32, stats.data_ptr(), w.data_ptr(),
                      b.data_ptr(), part.data_ptr(), V, C, st),
            _lib.call("lci_inorm_finalize", part.data_ptr(), coef.data_ptr(), V, 1, C, 1, INORM_EPS, st),
            _lib.call("lci_bn_relu_bwd_apply", x_cl.data_ptr(), g.data_ptr(), f32, stats.data_ptr(), coef.data_ptr(),
                      w.data_ptr(), b.data_ptr(), dx.data_ptr(), V, C, st)))
        dw = coef[0, 1] * V if ctx.needs_input_grad[1] else None
        db = coef[0, 0] * V if ctx.needs_input_grad[2] else None
        return dx, dw, db


def batch_norm_relu_supported(x: torch.Tensor, bn) -> bool:
    """The fused training BatchNorm + ReLU takes a bf16 map with dense channels-last strides, 8 | C <= 2048, an
    affine BN with eps 1e-5 and a momentum, in training mode."""
    C = x.shape[1]
    if not (x.is_cuda and x.dtype == torch.bfloat16 and bn.training and bn.affine and bn.track_running_stats
            and bn.momentum is not None and bn.eps == INORM_EPS and C % 8 == 0 and C <= 2048):
        return False
    x_cl = x.movedim(1, -1)
    return x_cl.is_contiguous() and x_cl.data_ptr() % 16 == 0 and x.numel() // C > 1


def batch_norm_relu(x: torch.Tensor, bn) -> torch.Tensor:
    """relu(bn(x)) for a training-mode nn.BatchNorm{2,3}d `bn` (running statistics updated as torch does: momentum,
    unbiased variance), x (B, C, *S) bf16 channels-last -> f32 with channels-last strides."""
    B, C = x.shape[:2]
    x_cl = x.movedim(1, -1).reshape(-1, C)
    V = x_cl.shape[0]
    y, stats = _BatchNormReLU.apply(x_cl, bn.weight, bn.bias)
    with torch.no_grad():
        m = bn.momentum
        mean = stats[0, 0]
        var = (1.0 / stats[0, 1].double() ** 2 - bn.eps).clamp_min(0.0) * (V / max(V - 1, 1))
        bn.running_mean.mul_(1.0 - m).add_(mean, alpha=m)
        bn.running_var.mul_(1.0 - m).add_(var.float(), alpha=m)
        bn.num_batches_tracked.add_(1)
    return y.view(B, *x.shape[2:], C).movedim(-1, 1)


def _inorm_stats(x_cl, act):
    """(B, 2, C) f32 mean, rstd of a (B, V, C) bf16 tensor over its voxels."""
    return _inorm_sums(x_cl, None, None, act, 0)


def _inorm_bwd(x_cl, stats, dz, act):
    """dx of z = [lrelu](norm(x)) for the upstream gradient dz (B, V, C)."""
    B, V, C = x_cl.shape
    dz = dz.to(torch.bfloat16).contiguous()
    coef = _inorm_sums(x_cl, dz, stats, act, 1)
    dx = torch.empty_like(x_cl)
    KernelTimer.run("inorm_bwd", 0.0, x_cl, lambda: _lib.call(
        "lci_inorm_apply", x_cl.data_ptr(), dz.data_ptr(), stats.data_ptr(), coef.data_ptr(), dx.data_ptr(),
        V, B, C, int(act), LRELU_SLOPE, _lib.stream_of(x_cl)))
    return dx


class _InstanceNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_cl, act):
        B, V, C = x_cl.shape
        stats = _inorm_stats(x_cl, act)
        z = torch.empty_like(x_cl)
        KernelTimer.run("inorm_fwd", 0.0, x_cl, lambda: _lib.call(
            "lci_inorm_apply", x_cl.data_ptr(), None, stats.data_ptr(), None, z.data_ptr(), V, B, C, int(act),
            LRELU_SLOPE, _lib.stream_of(x_cl)))
        ctx.save_for_backward(x_cl, stats)
        ctx.act = act
        return z

    @staticmethod
    def backward(ctx, dz):
        x_cl, stats = ctx.saved_tensors
        return _inorm_bwd(x_cl, stats, dz, ctx.act), None


class _InormAddLrelu(torch.autograd.Function):
    """lrelu(norm(x) + r) with r = norm(y) (pre_norm) or y, one pass forward (lci_inorm_apply_res); backward: the
    LeakyReLU mask from the saved output, then the instance-norm backward of each normalised input."""

    @staticmethod
    def forward(ctx, x_cl, y_cl, pre_norm):
        B, V, C = x_cl.shape
        sx = _inorm_stats(x_cl, False)
        sy = _inorm_stats(y_cl, False) if pre_norm else None
        out = torch.empty_like(x_cl)
        KernelTimer.run("inorm_fwd", 0.0, x_cl, lambda: _lib.call(
            "lci_inorm_apply_res", x_cl.data_ptr(), sx.data_ptr(), y_cl.data_ptr(), _lib.ptr(sy), out.data_ptr(),
            V, B, C, LRELU_SLOPE, _lib.stream_of(x_cl)))
        ctx.save_for_backward(x_cl, sx, y_cl if pre_norm else None, sy, out)
        ctx.pre_norm = pre_norm
        return out

    @staticmethod
    def backward(ctx, g):
        x_cl, sx, y_cl, sy, out = ctx.saved_tensors
        gs = torch.ops.aten.leaky_relu_backward(g.to(torch.bfloat16), out, LRELU_SLOPE, True)
        dx = _inorm_bwd(x_cl, sx, gs, False)
        dy = _inorm_bwd(y_cl, sy, gs, False) if ctx.pre_norm else gs
        return dx, dy, None


def _as_cl(x: torch.Tensor):
    """(B, C, *S) -> (B, V, C) view when x is bf16 with dense channels-last strides, else None."""
    B, C = x.shape[:2]
    if x.dtype != torch.bfloat16:
        return None
    x_cl = x.movedim(1, -1).reshape(B, -1, C)
    return x_cl if x_cl.is_contiguous() else None


def inorm_add_lrelu(x: torch.Tensor, r: torch.Tensor, r_pre_norm: bool) -> torch.Tensor | None:
    """UnetResBlock's tail lrelu(norm2(x) + r) (r = norm3(r) when r_pre_norm, else r as is) for bf16 channels-last
    (B, C, *S) tensors in one pass; None when the operands do not qualify (the caller keeps the unfused ops)."""
    if not x.is_cuda or x.shape != r.shape or x.shape[1] % 8 or x.shape[1] > 2048:
        return None
    xc, rc = _as_cl(x), _as_cl(r)
    if xc is None or rc is None or xc.data_ptr() % 16 or rc.data_ptr() % 16:
        return None
    B, C = x.shape[:2]
    z = _InormAddLrelu.apply(xc, rc, r_pre_norm)
    return z.view(B, *x.shape[2:], C).movedim(-1, 1)


def instance_norm_act(x: torch.Tensor, act: bool) -> torch.Tensor:
    """InstanceNorm{2,3}d(C) (affine=False, eps 1e-5) [+ LeakyReLU(0.01)] of a bf16 (B, C, *S) tensor, computed
    channels-last by the HIP kernels; returns (B, C, *S) bf16 with channels-last strides."""
    if not x.is_cuda:
        raise _lib.LciError("instance_norm_act runs on the GPU only; there is no CPU path")
    B, C = x.shape[:2]
    S = x.shape[2:]
    x_cl = x.movedim(1, -1).reshape(B, -1, C)
    if x_cl.dtype != torch.bfloat16:
        x_cl = x_cl.to(torch.bfloat16)
    x_cl = x_cl.contiguous()
    z = _InstanceNormAct.apply(x_cl, act)
    return z.view(B, *S, C).movedim(-1, 1)


# ------------------------------------------------------------------ transformer-block LayerNorm (+ autocast cast)
def _ln_fwd(x, weight, bias, eps, bf16_out):
    C = x.shape[-1]
    x2 = x.reshape(-1, C)
    rows = x2.shape[0]
    y = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16 if bf16_out else torch.float32)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    KernelTimer.run("ln_fwd", rows * C * (4 + y.element_size()), x, lambda: _lib.call(
        "lci_layernorm_fwd", x2.data_ptr(), weight.data_ptr(), bias.data_ptr(), y.data_ptr(), int(bf16_out),
        mean.data_ptr(), rstd.data_ptr(), rows, C, float(eps), _lib.stream_of(x)))
    return y, x2, mean, rstd


def _ln_bwd(x2, weight, mean, rstd, dy, dres, shape, want_bf16=False, dres2=None):
    """dx (f32, `shape`), dgamma, dbeta [, dx rounded to bf16 in the same kernel pass when want_bf16]; dres2: a second
    residual gradient (a recorded hidden state's), summed with dres inside the kernel."""
    rows, C = x2.shape
    bf = dy.dtype == torch.bfloat16
    dy = (dy if bf else dy.float()).contiguous()
    if dy.data_ptr() % 16:   # a contiguous view at a storage offset: the kernel's vector loads need 8/16-B rows
        dy = dy.clone()
    def dense_f32(t):   # the kernel reads residual gradients as dense, 16-B aligned f32 (rows, C) arrays
        if t is None:
            return None
        t = t.float().contiguous()
        return t.clone() if t.data_ptr() % 16 else t

    dres, dres2 = dense_f32(dres), dense_f32(dres2)
    if dres is None:   # a lone second residual gradient takes the first slot
        dres, dres2 = dres2, None
    dx = torch.empty(rows, C, device=x2.device, dtype=torch.float32)
    dxb = torch.empty(rows, C, device=x2.device, dtype=torch.bfloat16) if want_bf16 else None
    nblk = _lib.load().lci_layernorm_bwd_blocks(rows)
    part = torch.empty(nblk, 2, C, device=x2.device, dtype=torch.float32)
    KernelTimer.run("ln_bwd", rows * C * (8 + dy.element_size() + (4 if dres is not None else 0) + (2 if want_bf16 else 0)),
                    x2, lambda: _lib.call("lci_layernorm_bwd", x2.data_ptr(), dy.data_ptr(), int(bf), weight.data_ptr(),
                                          mean.data_ptr(), rstd.data_ptr(), _lib.ptr(dres), _lib.ptr(dres2),
                                          dx.data_ptr(), _lib.ptr(dxb), part.data_ptr(), rows, C, _lib.stream_of(x2)))
    s = part.sum(0)
    if want_bf16:
        return dx.view(shape), s[0], s[1], dxb.view(shape)
    return dx.view(shape), s[0], s[1]


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, bf16_out):
        y, x2, mean, rstd = _ln_fwd(x, weight, bias, eps, bf16_out)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, weight, mean, rstd = ctx.saved_tensors
        dx, dw, db = _ln_bwd(x2, weight, mean, rstd, dy, None, ctx.shape)
        return dx, dw, db, None, None


class _ResidualLayerNorm(torch.autograd.Function):
    """(h, t, y) = (x, x, LN(x)) for a block `x + f(LN(x))`: the backward adds the residual path's gradient dh into
    the LN input gradient inside the HIP kernel, instead of autograd accumulating the two in a separate pass; t is
    a second alias of x for a consumer outside the block (a recorded hidden state), whose gradient is summed in the
    same kernel."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps, bf16_out):
        y, x2, mean, rstd = _ln_fwd(x, weight, bias, eps, bf16_out)
        ctx.save_for_backward(x2, weight, mean, rstd)
        ctx.shape = x.shape
        ctx.set_materialize_grads(False)   # an unused output arrives as None, not as a zeros tensor
        return x.view_as(x), x.view_as(x), y

    @staticmethod
    def backward(ctx, dh, dt, dy):
        x2, weight, mean, rstd = ctx.saved_tensors
        if dy is None:   # LN output unused: the residual gradients pass straight through
            if dh is None or dt is None:
                return (dh if dt is None else dt), None, None, None, None
            return dh + dt, None, None, None, None
        dx, dw, db = _ln_bwd(x2, weight, mean, rstd, dy, dh, ctx.shape, dres2=dt)
        return dx, dw, db, None, None


class _AddResidualLayerNorm(torch.autograd.Function):
    """(x, y) = (h + a, LN(h + a)) for the middle of a block `h + a -> norm2 -> ...`: the residual add runs inside
    the LN forward kernel (no separate add pass), the backward is the residual LN backward on x (dh = dx,
    da = dx in a's dtype)."""

    @staticmethod
    def forward(ctx, h, a, weight, bias, eps, bf16_out):
        C = h.shape[-1]
        h2 = h.reshape(-1, C)
        a2 = a.reshape(-1, C)
        rows = h2.shape[0]
        xsum = torch.empty(rows, C, device=h.device, dtype=torch.float32)
        y = torch.empty(h.shape, device=h.device, dtype=torch.bfloat16 if bf16_out else torch.float32)
        mean = torch.empty(rows, device=h.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        KernelTimer.run("ln_add_fwd", rows * C * (8 + a.element_size() + y.element_size()), h, lambda: _lib.call(
            "lci_layernorm_add_fwd", h2.data_ptr(), a2.data_ptr(), int(a.dtype == torch.bfloat16), xsum.data_ptr(),
            weight.data_ptr(), bias.data_ptr(), y.data_ptr(), int(bf16_out), mean.data_ptr(), rstd.data_ptr(), rows,
            C, float(eps), _lib.stream_of(h)))
        ctx.save_for_backward(xsum, weight, mean, rstd)
        ctx.shape = h.shape
        ctx.adtype = a.dtype
        ctx.set_materialize_grads(False)
        return xsum.view(h.shape), xsum.view(h.shape), y   # the stream, and an alias for a hidden-state tap

    @staticmethod
    def backward(ctx, dx_out, dt, dy):
        xsum, weight, mean, rstd = ctx.saved_tensors
        if dy is None:
            dx, dw, db = (dx_out if dt is None else (dt if dx_out is None else dx_out + dt)), None, None
        elif ctx.adtype == torch.bfloat16:   # the bf16 branch gradient written by the same kernel pass
            dx, dw, db, da = _ln_bwd(xsum, weight, mean, rstd, dy, dx_out, ctx.shape, want_bf16=True, dres2=dt)
            return dx, da, dw, db, None, None
        else:
            dx, dw, db = _ln_bwd(xsum, weight, mean, rstd, dy, dx_out, ctx.shape, dres2=dt)
        if dx is None:
            return None, None, None, None, None, None
        return dx, dx.to(ctx.adtype), dw, db, None, None


def add_residual_layer_norm(h, a, weight, bias, eps, bf16_out, tap=False):
    """(h + a, layer_norm(h + a)) with the add inside the HIP LN forward; h f32, a bf16 / f32 of h's shape.
    tap: (h + a, a second alias of it for a consumer outside the block, layer_norm(h + a)), the alias's gradient
    summed inside the LN backward kernel."""
    h = _ln_checks(h, weight, bias)
    ok = (ln_kernel_supports(h.shape[-1]) and a.shape == h.shape and a.dtype in (torch.bfloat16, torch.float32)
          and a.is_cuda)
    if ok:
        a = a.contiguous()
        ok = a.data_ptr() % 16 == 0
    if not ok:
        x = h + a
        return residual_layer_norm(x, weight, bias, eps, bf16_out, tap)
    x, t, y = _AddResidualLayerNorm.apply(h, a, weight, bias, eps, bf16_out)
    return (x, t, y) if tap else (x, y)


def _ln_checks(x, weight, bias):
    _lib.require_gpu(weight, bias)
    if not x.is_cuda:
        raise _lib.LciError("layer_norm runs on the GPU only; there is no CPU path")
    if weight.dtype != torch.float32 or bias.dtype != torch.float32:
        raise _lib.LciError("layer_norm expects f32 affine parameters")
    return x.float().contiguous()


LN_MAX_C = 2048   # csrc/layernorm.hip LN_MAX_C


def ln_kernel_supports(C: int) -> bool:
    """The HIP LayerNorm covers C % 4 == 0, C <= 2048 (every ViT / Swin preset of the reference: ViT 384-1024,
    Swin stages up to 1536). Other widths (custom sizes only) run torch's own GPU layer_norm."""
    return C % 4 == 0 and C <= LN_MAX_C


def _torch_ln(x, weight, bias, eps, bf16_out):
    y = torch.nn.functional.layer_norm(x, (x.shape[-1],), weight, bias, eps)
    return y.to(torch.bfloat16) if bf16_out else y


def layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float, bf16_out: bool):
    """nn.LayerNorm over the last dim of an f32 tensor; bf16_out returns the bf16 rounding of the f32 result
    (what autocast hands the next Linear). HIP kernels (GPU tensors only; widths outside ln_kernel_supports run
    torch's GPU layer_norm)."""
    x = _ln_checks(x, weight, bias)
    if not ln_kernel_supports(x.shape[-1]):
        return _torch_ln(x, weight, bias, eps, bf16_out)
    return _LayerNorm.apply(x, weight, bias, eps, bf16_out)


def residual_layer_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, eps: float, bf16_out: bool,
                        tap: bool = False):
    """(x, layer_norm(x)) with the residual gradient fused into the LN backward (see _ResidualLayerNorm); tap: (x, a
    second alias of x, layer_norm(x)), the alias's gradient summed in the same kernel."""
    x = _ln_checks(x, weight, bias)
    if not ln_kernel_supports(x.shape[-1]):
        y = _torch_ln(x, weight, bias, eps, bf16_out)
        return (x, x, y) if tap else (x, y)
    h, t, y = _ResidualLayerNorm.apply(x, weight, bias, eps, bf16_out)
    return (h, t, y) if tap else (h, y)


# ------------------------------------------------------------------------------------- token-wise Linear
def linear_wgrad_supported(dy2: torch.Tensor, x2: torch.Tensor) -> bool:
    """Whether lci_linear_wgrad takes (dy2 (M, N), x2 (M, K)): bf16 CUDA row-major views with unit column stride,
    N, K and the row strides multiples of 8, 16-byte aligned, and a tile that fits (N, K)."""
    if not (dy2.is_cuda and x2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16):
        return False
    (M, N), K = dy2.shape, x2.shape[1]
    if dy2.stride(1) != 1 or x2.stride(1) != 1 or N % 8 or K % 8 or dy2.stride(0) % 8 or x2.stride(0) % 8:
        return False
    if dy2.data_ptr() % 16 or x2.data_ptr() % 16 or M == 0:
        return False
    return _lib.load().lci_linear_wgrad_splits(M, N, K) > 0


def linear_wgrad(dy2: torch.Tensor, x2: torch.Tensor, bias: bool):
    """dW (N, K) f32 = dy2^T x2 and db (N) f32 = column sums of dy2 (or None), by the HIP split-token kernel
    (per-split partials summed here)."""
    (M, N), K = dy2.shape, x2.shape[1]
    lib = _lib.load()
    ns = lib.lci_linear_wgrad_splits(M, N, K)
    if ns <= 0:
        raise _lib.LciError(f"linear_wgrad: unsupported shape N={N}, K={K}")
    part = torch.empty(ns, N, K, device=dy2.device, dtype=torch.float32)
    dbp = torch.empty(ns, N, device=dy2.device, dtype=torch.float32) if bias else None
    KernelTimer.run("linear_wgrad", 2.0 * M * N * K, dy2, lambda: _lib.call(
        "lci_linear_wgrad", dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), M, N, K, part.data_ptr(),
        _lib.ptr(dbp), _lib.stream_of(dy2)))
    return part.sum(0), (dbp.sum(0) if bias else None)


def _wgrad_tiny_k(dy2: torch.Tensor, x2: torch.Tensor, bias: bool):
    """dW (N, K) f32 = dy2^T x2 for K <= 4 input channels (the 1-channel image into a head's 1x1 residual conv, 2·10^6
    voxel rows at C3): lci_linear_small_bwd with the roles swapped (its "x" = dy2 (M, N <= 256), its "dy" = x2
    (M, K)) streams dy2 once; the K-padded GEMM hipBLASLt ran instead took 1.5 ms for this 96 x 8 output."""
    (M, N), K = dy2.shape, x2.shape[1]
    nt = _lib.load().lci_linear_small_threads()
    part = torch.empty(K * N + K, nt, device=dy2.device, dtype=torch.float32)
    w_unused = torch.zeros(K, N, device=dy2.device, dtype=torch.bfloat16)   # read only for dx, which is not asked
    KernelTimer.run("linear_wgrad_tiny", 2.0 * M * N * K, dy2, lambda: _lib.call(
        "lci_linear_small_bwd", dy2.data_ptr(), dy2.stride(0), w_unused.data_ptr(), x2.data_ptr(), None,
        part.data_ptr(), M, K, N, _lib.stream_of(dy2)))
    # the parameter's strides (DDP's bucket views); .contiguous() keeps (1, N) strides when K == 1, clone does not
    dw = part[:K * N].sum(1).view(K, N).t().clone(memory_format=torch.contiguous_format)
    return dw, (dy2.float().sum(0) if bias else None)


# csrc/gemm.hip for the bf16 projection GEMMs whose output width it takes (N % 384 == 0: every ViT-small / Mamba /
# Hyena projection and data gradient; N % 256 == 0: the decoders' ConvTranspose GEMMs); LCI_HIP_GEMM=0 routes them to
# hipBLASLt (A/B: profiles/r05_gemm_ab.txt)
HIP_GEMM = os.environ.get("LCI_HIP_GEMM", "1") == "1"


def gemm_bt_supported(x2: torch.Tensor, N: int, K: int) -> bool:
    """Whether lci_gemm_bt takes x2 (M, K) bf16 rows (unit column stride, 8-element row stride, 16-B aligned)."""
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and x2.dim() == 2 and x2.stride(1) == 1
            and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and x2.shape[0] > 0
            and bool(_lib.load().lci_gemm_bt_supported(N, K)))


GEMM_BT_MIN_TILES = 256   # one 256 x 384 output tile per CU at least


def gemm_bt_preferred(M: int, N: int) -> bool:
    """The product routing: lci_gemm_bt when its persistent grid has a tile for every CU. Below that (the Swin
    stage-3 / 4 projections: 4096 / 512 tokens, 16-48 tiles) its one-tile-per-CU walk leaves most of the chip idle
    and hipBLASLt's smaller / split-K tiles win (M = 4096 fc2: 0.056 vs 0.020 ms; C3 step 57.0 vs 54.2 ms with every
    supported shape on lci_gemm_bt; profiles/r05_gemm_ab.txt)."""
    return -(-M // 256) * (N // (384 if N % 384 == 0 else 256)) >= GEMM_BT_MIN_TILES


def gemm_bt(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """y (M, N) bf16 = x2 (M, K) . w^T + bias on csrc/gemm.hip (w (N, K) bf16, made contiguous; bias bf16 or None)."""
    M, K = x2.shape
    N = w.shape[0]
    w = w.contiguous()
    if bias is not None:
        bias = bias.contiguous()
    _lib.require_gpu(w, bias)
    y = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    KernelTimer.run("gemm_bt", 2.0 * M * N * K, x2, lambda: _lib.call(
        "lci_gemm_bt", x2.data_ptr(), x2.stride(0), w.data_ptr(), _lib.ptr(bias), y.data_ptr(), N, M, N, K,
        _lib.stream_of(x2)))
    return y


# csrc/gemm.hip's small / narrow kernel (round 6) for the GEMMs lci_gemm_bt does not take or fill: the Swin stage-3 / 4
# projections (4096 / 512 tokens) and the decoder heads' 96 / 192 / 288-wide 1x1 convolutions. Opt-in
# (LCI_SMALL_GEMM=1): against hipBLASLt it won on 5 of the 23 C3 shapes and lost up to 3x on the rest (K >= 192 at
# 2^18 - 2^21 rows, K >= 768 at 512 - 4096; profiles/r06_gemm_small.txt), and the C3 step went 48.8 -> 51.9 ms with
# it routed to every supported shape, so hipBLASLt keeps them.
SMALL_GEMM = os.environ.get("LCI_SMALL_GEMM", "0") == "1"


def gemm_small_supported(x2: torch.Tensor, N: int, K: int) -> bool:
    """Whether lci_gemm_bt_small takes x2 (M, K) bf16 rows (unit column stride, 8-element row stride, 16-B aligned)
    for N outputs: N % 32 == 0, K % 16 == 0."""
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and x2.dim() == 2 and x2.stride(1) == 1
            and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and x2.shape[0] > 0
            and bool(_lib.load().lci_gemm_bt_small_supported(N, K)))


def gemm_small(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """y (M, N) bf16 = x2 (M, K) . w^T + bias on lci_gemm_bt_small (w (N, K) bf16, made contiguous; bias bf16 or
    None); with `out` (an (M, N) bf16 matrix, unit column stride): out += bf16(x2 . w^T) in place (no bias)."""
    M, K = x2.shape
    N = w.shape[0]
    w = w.contiguous()
    if bias is not None:
        bias = bias.contiguous()
    _lib.require_gpu(w, bias)
    if out is not None:
        assert bias is None and out.shape == (M, N) and out.stride(1) == 1 and out.dtype == torch.bfloat16
        KernelTimer.run("gemm_bt_small", 2.0 * M * N * K, x2, lambda: _lib.call(
            "lci_gemm_bt_small_acc", x2.data_ptr(), x2.stride(0), w.data_ptr(), out.data_ptr(), out.stride(0), M, N, K,
            _lib.stream_of(x2)))
        return out
    y = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    KernelTimer.run("gemm_bt_small", 2.0 * M * N * K, x2, lambda: _lib.call(
        "lci_gemm_bt_small", x2.data_ptr(), x2.stride(0), w.data_ptr(), _lib.ptr(bias), y.data_ptr(), N, M, N, K,
        _lib.stream_of(x2)))
    return y


class _Linear(torch.autograd.Function):
    """y = x W^T + b with autocast's casts done here (x, W, b -> the autocast dtype, exactly what F.linear under
    autocast computes); the bf16 forward and data-gradient GEMMs on csrc/gemm.hip where it takes the shape (hipBLASLt
    otherwise), the weight / bias gradient on lci_linear_wgrad (f32 result, returned to the f32 parameters without
    the bf16 rounding the autocast GEMM would apply)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            xc, wc = x.to(dt), weight.to(dt)
            bc = bias.to(dt) if bias is not None else None
        else:
            xc, wc, bc = x, weight, bias
        N, K = wc.shape
        x2 = xc.reshape(-1, K) if xc.dim() != 2 else xc
        if HIP_GEMM and x2.dim() == 2 and gemm_bt_preferred(x2.shape[0], N) and gemm_bt_supported(x2, N, K):
            y = gemm_bt(x2, wc, bc).view(*xc.shape[:-1], N)
        elif SMALL_GEMM and x2.dim() == 2 and gemm_small_supported(x2, N, K):
            y = gemm_small(x2, wc, bc).view(*xc.shape[:-1], N)
        elif K == 1 and xc.is_cuda:
            # one input channel (the image into encoder1's 1x1 residual conv): an outer product, one stream; the
            # product of two bf16 values is exact in f32, so x w (+ b) rounds the same f32 value the GEMM does
            # (hipBLASLt: 0.40 ms at 2^21 x 96, C3)
            wv = wc.view(N)
            y = torch.addcmul(bc, xc, wv) if bc is not None else xc * wv
        else:
            with torch.autocast("cuda", enabled=False):
                y = torch.nn.functional.linear(xc, wc, bc)
        ctx.save_for_backward(xc, wc)
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        N, K = wc.shape
        dy2 = dy.reshape(-1, N)
        if dy2.stride(1) != 1:
            dy2 = dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if HIP_GEMM and dy2.dtype == wc.dtype and gemm_bt_preferred(dy2.shape[0], K) and gemm_bt_supported(dy2, K, N):
                dx = gemm_bt(dy2, wc.t()).view(*dy.shape[:-1], K)   # dX = dY . W = dY . (W^T)^T
            elif SMALL_GEMM and dy2.dtype == wc.dtype and gemm_small_supported(dy2, K, N):
                dx = gemm_small(dy2, wc.t()).view(*dy.shape[:-1], K)
            else:
                dx = (dy2 @ wc).view(*dy.shape[:-1], K)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            x2 = xc.reshape(-1, K)
            if K <= 4 and x2.dtype == torch.bfloat16 and pointwise_small_supported(dy2, K):
                dw, db = _wgrad_tiny_k(dy2, x2.contiguous(), ctx.has_bias)
                return dx, dw, db
            if K % 8 and x2.dtype == torch.bfloat16 and x2.is_cuda:
                # few input channels (the 1-channel image into a head's 1x1 residual conv): zero-pad to 8 columns
                x2 = torch.nn.functional.pad(x2, (0, 8 - K % 8))
            if linear_wgrad_supported(dy2, x2):
                dw, db = linear_wgrad(dy2, x2, ctx.has_bias)
                dw = dw[:, :K]
            else:
                dw = (dy2.t() @ x2).float()[:, :K]
                db = dy2.float().sum(0) if ctx.has_bias else None
        return dx, dw, db


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    return _Linear.apply(x, weight, bias)


def pointwise_small_supported(x2: torch.Tensor, N: int) -> bool:
    """lci_linear_small_*: x2 (M, K) bf16 CUDA rows (unit column stride, 16-B aligned), N <= 4, K % 8, K <= 256."""
    K = x2.shape[1]
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and 1 <= N <= 4 and K % 8 == 0 and K <= 256
            and x2.stride(1) == 1 and x2.stride(0) % 8 == 0 and x2.data_ptr() % 16 == 0 and x2.shape[0] > 0)


class _PointwiseSmall(torch.autograd.Function):
    """x2 (M, K) bf16 . w^T + b for N <= 4 output channels (autocast casts done here, as F.linear would)."""

    @staticmethod
    def forward(ctx, x2, weight, bias):
        M, K = x2.shape
        N = weight.shape[0]
        wc = weight.reshape(N, K).to(torch.bfloat16).contiguous()
        bc = bias.to(torch.bfloat16) if bias is not None else None
        y = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
        KernelTimer.run("pointwise_small_fwd", 0, x2, lambda: _lib.call(
            "lci_linear_small_fwd", x2.data_ptr(), x2.stride(0), wc.data_ptr(), _lib.ptr(bc), y.data_ptr(), M, N, K,
            _lib.stream_of(x2)))
        ctx.save_for_backward(x2, wc)
        ctx.has_bias, ctx.wshape = bias is not None, weight.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, wc = ctx.saved_tensors
        M, K = x2.shape
        N = wc.shape[0]
        dy = dy.to(torch.bfloat16).contiguous()
        nt = _lib.load().lci_linear_small_threads()
        part = torch.empty(N * K + N, nt, device=x2.device, dtype=torch.float32)
        dx = torch.empty(M, K, device=x2.device, dtype=torch.bfloat16) if ctx.needs_input_grad[0] else None
        KernelTimer.run("pointwise_small_bwd", 0, x2, lambda: _lib.call(
            "lci_linear_small_bwd", x2.data_ptr(), x2.stride(0), wc.data_ptr(), dy.data_ptr(), _lib.ptr(dx),
            part.data_ptr(), M, N, K, _lib.stream_of(x2)))
        g = part.sum(1)
        dw = g[:N * K].view(N, K).reshape(ctx.wshape)
        db = g[N * K:] if ctx.has_bias else None
        return dx, dw, db


def pointwise_small(x2: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None) -> torch.Tensor:
    return _PointwiseSmall.apply(x2, weight, bias)


# ------------------------------------------------------------------------------------------- optimizer step
def adam_step(params, grads, exp_avgs, exp_avg_sqs, steps, lr: float, beta1: float, beta2: float,
              weight_decay: float, eps: float, decoupled: bool, maximize: bool) -> None:
    """One Adam / AdamW update of f32 CUDA tensors in place by csrc/optim.hip (lci_adam_step, up to
    lci_adam_max_tensors() tensors per launch); `steps` are the per-tensor device step counts, already incremented
    (trainer_base.py:171-177 -> torch.optim.Adam / AdamW with optim_base.py:87-89's hyper-parameters)."""
    if not params:
        return
    lib = _lib.load()
    per = lib.lci_adam_max_tensors()
    for t in (*params, *grads, *exp_avgs, *exp_avg_sqs):
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise _lib.LciError("adam_step: f32 contiguous CUDA tensors only")
    st = _lib.stream_of(params[0])
    for i0 in range(0, len(params), per):
        sl = slice(i0, i0 + per)
        n = len(params[sl])
        arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])   # noqa: E731
        sizes = (ctypes.c_longlong * n)(*[t.numel() for t in params[sl]])
        _lib.call("lci_adam_step", arr(params[sl]), arr(grads[sl]), arr(exp_avgs[sl]), arr(exp_avg_sqs[sl]),
                  arr(steps[sl]), sizes, n, float(lr), float(beta1), float(beta2), float(weight_decay), float(eps),
                  int(decoupled), int(maximize), st)
