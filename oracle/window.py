"""Oracle: Swin shifted-window attention, CPU restatement. Test infrastructure only.

Index math (bit-exact, integer):
  window_partition / window_reverse      backbone_swin.py:135-197
  get_window_size                        backbone_swin.py:200-224
  relative_position_index (3-D and 2-D)  backbone_swin.py:268-308
  compute_mask (27 / 9 regions, -100)    backbone_swin.py:591-628
Floating point:
  WindowAttention.forward                backbone_swin.py:335-359
  SwinTransformerBlock.forward_part1     backbone_swin.py:435-487 (LN1 -> pad -> roll -> partition ->
                                          attn -> reverse -> roll back -> crop)
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def get_window_size(x_size, window_size, shift_size=None):
    ws = list(window_size)
    ss = list(shift_size) if shift_size is not None else None
    for i in range(len(x_size)):
        if x_size[i] <= window_size[i]:
            ws[i] = x_size[i]
            if ss is not None:
                ss[i] = 0
    return tuple(ws) if ss is None else (tuple(ws), tuple(ss))


def window_partition(x, ws):
    """(b, d, h, w, c) -> (b*nW, wd*wh*ww, c); window-major (b, d/wd, h/wh, w/ww), raster in window."""
    if x.ndim == 5:
        b, d, h, w, c = x.shape
        x = x.reshape(b, d // ws[0], ws[0], h // ws[1], ws[1], w // ws[2], ws[2], c)
        return x.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(-1, ws[0] * ws[1] * ws[2], c)
    b, h, w, c = x.shape
    x = x.reshape(b, h // ws[0], ws[0], w // ws[1], ws[1], c)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(-1, ws[0] * ws[1], c)


def window_reverse(windows, ws, dims):
    if len(dims) == 4:
        b, d, h, w = dims
        x = windows.reshape(b, d // ws[0], h // ws[1], w // ws[2], ws[0], ws[1], ws[2], -1)
        return x.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(b, d, h, w, -1)
    b, h, w = dims
    x = windows.reshape(b, h // ws[0], w // ws[1], ws[0], ws[1], -1)
    return x.permute(0, 1, 3, 2, 4, 5).reshape(b, h, w, -1)


def relative_position_index(ws) -> np.ndarray:
    """int64 (N, N) index into the ((2w-1)^dims, heads) bias table."""
    coords = np.stack(np.meshgrid(*[np.arange(w) for w in ws], indexing="ij")).reshape(len(ws), -1)
    rel = (coords[:, :, None] - coords[:, None, :]).transpose(1, 2, 0).astype(np.int64)
    for i, w in enumerate(ws):
        rel[:, :, i] += w - 1
    if len(ws) == 3:
        rel[:, :, 0] *= (2 * ws[1] - 1) * (2 * ws[2] - 1)
        rel[:, :, 1] *= 2 * ws[2] - 1
    else:
        rel[:, :, 0] *= 2 * ws[1] - 1
    return rel.sum(-1)


def region_ids(dims, ws, ss) -> np.ndarray:
    """Per-voxel region id (0..26 / 0..8) of compute_mask's img_mask (backbone_swin.py:604-621)."""
    img = np.zeros(dims, dtype=np.int64)
    cnt = 0
    sl = [(slice(-w), slice(-w, -s), slice(-s, None)) for w, s in zip(ws, ss)]
    if len(dims) == 3:
        for a in sl[0]:
            for b in sl[1]:
                for c in sl[2]:
                    img[a, b, c] = cnt
                    cnt += 1
    else:
        for a in sl[0]:
            for b in sl[1]:
                img[a, b] = cnt
                cnt += 1
    return img


def compute_mask(dims, ws, ss) -> torch.Tensor:
    """(nW, N, N) float32 mask: -100 where region ids differ, else 0."""
    img = torch.from_numpy(region_ids(dims, ws, ss)).float()[None, ..., None]
    mw = window_partition(img, ws).squeeze(-1)
    am = mw.unsqueeze(1) - mw.unsqueeze(2)
    return am.masked_fill(am != 0, -100.0).masked_fill(am == 0, 0.0)


def window_attention(x, mask, qkv_w, qkv_b, proj_w, proj_b, rpb_table, rp_index, num_heads):
    """WindowAttention.forward attention branch (backbone_swin.py:339-359)."""
    b, n, c = x.shape
    qkv = F.linear(x, qkv_w, qkv_b).reshape(b, n, 3, num_heads, c // num_heads).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0], qkv[1], qkv[2]
    q = q * (c // num_heads) ** -0.5
    attn = q @ k.transpose(-2, -1)
    idx = torch.as_tensor(rp_index)[:n, :n].reshape(-1)
    rpb = rpb_table[idx].reshape(n, n, -1).permute(2, 0, 1)
    attn = attn + rpb.unsqueeze(0)
    if mask is not None:
        nw = mask.shape[0]
        attn = attn.view(b // nw, nw, num_heads, n, n) + mask.unsqueeze(1).unsqueeze(0)
        attn = attn.view(-1, num_heads, n, n)
    attn = attn.softmax(-1).to(v.dtype)
    x = (attn @ v).transpose(1, 2).reshape(b, n, c)
    return F.linear(x, proj_w, proj_b)


def window_attention_core(q, k, v, rpb, mask, scale):
    """Core only: q,k,v (Bw, H, N, hd); rpb (H, N, N); mask (nW, N, N) or None."""
    attn = (q * scale) @ k.transpose(-2, -1) + rpb.unsqueeze(0)
    if mask is not None:
        bw, h, n, _ = attn.shape
        nw = mask.shape[0]
        attn = (attn.view(bw // nw, nw, h, n, n) + mask.unsqueeze(1).unsqueeze(0)).view(bw, h, n, n)
    return attn.softmax(-1) @ v


def swin_part1(x, ln_w, ln_b, ws_cfg, ss_cfg, attn_fn, mask_matrix):
    """SwinTransformerBlock.forward_part1 (backbone_swin.py:435-487), 3-D or 2-D channels-last input."""
    x = F.layer_norm(x, (x.shape[-1],), ln_w, ln_b)
    if x.ndim == 5:
        b, d, h, w, c = x.shape
        ws, ss = get_window_size((d, h, w), ws_cfg, ss_cfg)
        pads = [(ws[i] - s % ws[i]) % ws[i] for i, s in enumerate((d, h, w))]
        x = F.pad(x, (0, 0, 0, pads[2], 0, pads[1], 0, pads[0]))
        dims = [b, *x.shape[1:4]]
        sdims = (1, 2, 3)
    else:
        b, h, w, c = x.shape
        ws, ss = get_window_size((h, w), ws_cfg, ss_cfg)
        pads = [(ws[i] - s % ws[i]) % ws[i] for i, s in enumerate((h, w))]
        x = F.pad(x, (0, 0, 0, pads[1], 0, pads[0]))
        dims = [b, *x.shape[1:3]]
        sdims = (1, 2)
    shifted = any(s > 0 for s in ss)
    if shifted:
        x = torch.roll(x, shifts=tuple(-s for s in ss), dims=sdims)
    win = window_partition(x, ws)
    out = attn_fn(win, mask_matrix if shifted else None)
    out = window_reverse(out.reshape(-1, *ws, c), ws, dims)
    if shifted:
        out = torch.roll(out, shifts=tuple(ss), dims=sdims)
    if x.ndim == 5:
        return out[:, :d, :h, :w, :].contiguous()
    return out[:, :h, :w, :].contiguous()


def padded_dims(dims, ws):
    return [int(np.ceil(d / w)) * w for d, w in zip(dims, ws)]
