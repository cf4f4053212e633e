"""Phase timeline of the single-phase window-attention backward (win_attn_bwd1_kernel) from in-kernel timestamps.

Needs a variant library built with -DLCI_WIN_STAMPS (tools/build_variant.py stamps --define LCI_WIN_STAMPS=1
window.hip) loaded through LCI_LIB_PATH. Runs the C3 stage-1 / stage-3 window attention (128^3 p2, B 1, w 7) forward
+ backward twice and reads the stamps of the second backward: per workgroup (first 2048 in dispatch order) the
s_memrealtime (100 MHz) of kernel entry, setup done, prologue done, every step start, loop end, final barrier,
dK/dV stores done, end; slot 19 the CU. Prints phase medians and how the CU's consecutive workgroups overlap.
Usage (GPU box): LCI_LIB_PATH=build_variants/liblci_stamps.so python tools/r6_win_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from long_context_biomedical_imaging_amd import _lib, kernels  # noqa: E402

WG, NW, SL = 2048, 12, 20


def stamps():
    buf = np.zeros(WG * NW * SL, dtype=np.int64)
    fn = _lib.load().lci_debug_win_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    assert fn(buf.ctypes.data, buf.size) == 0
    return buf.reshape(WG, NW, SL)


def run(S, C, H, sh):
    w = 7
    qkv = torch.randn(1, S, S, S, 3 * C, device="cuda").to(torch.bfloat16).requires_grad_(True)
    bias = torch.randn(3 * C, device="cuda") * 0.1
    rpb = torch.randn(H, w ** 3, w ** 3, device="cuda") * 0.1
    for _ in range(2):
        o = kernels.window_attention_grid(qkv, bias, rpb, H, 32 ** -0.5, (w, w, w), (sh, sh, sh))
        torch.autograd.grad(o, qkv, torch.randn_like(o))
    torch.cuda.synchronize()
    st = stamps()
    nkb = (w ** 3 + 31) // 32
    nwg = min(WG, (-(-S // w)) ** 3 * H)
    st = st[:nwg, :nkb]
    t0 = st[:, :, 0].min()
    ent, setup, pro = st[:, :, 0], st[:, :, 1], st[:, :, 2]
    steps = st[:, :, 3:3 + nkb]
    loop_end, fin, dkv, end = st[:, :, 15], st[:, :, 16], st[:, :, 17], st[:, :, 18]
    us = lambda a: float(np.median(a)) / 100.0   # 100 MHz ticks -> us  # noqa: E731
    print(f"== S{S} C{C} H{H} shift {sh}: {nwg} workgroups x {nkb} waves (stamped)")
    print(f"  kernel span {(end.max() - t0) / 100:.1f} us; per workgroup (median over waves):")
    print(f"  setup {us(setup - ent):.2f}  prologue {us(pro - setup):.2f}  steps {us(loop_end - pro):.2f} "
          f"(per step {us(np.diff(steps, axis=2)):.2f}, first {us(steps[:, :, 0] - pro):.2f})  "
          f"final rmw+barrier {us(fin - loop_end):.2f}  dk/dv+pad {us(dkv - fin):.2f}  dq rows {us(end - dkv):.2f}  "
          f"total {us(end - ent):.2f}")
    # per-wave step spread: how far apart the waves of one workgroup run (counter-ordered RMW)
    spread = steps.max(axis=1) - steps.min(axis=1)
    print(f"  step-start spread across a workgroup's waves: median {us(spread):.2f} us")
    # per CU: consecutive workgroups' [entry, end] intervals -> idle gaps / overlap
    cu = st[:, 0, 19]
    gaps, conc = [], []
    for c in np.unique(cu):
        idx = np.where(cu == c)[0]
        s_ = ent[idx].min(axis=1)
        e_ = end[idx].max(axis=1)
        o = np.argsort(s_)
        s_, e_ = s_[o], e_[o]
        gaps += list(s_[1:] - e_[:-1])
        conc.append(len(idx))
    if gaps:
        g = np.array(gaps) / 100.0
        print(f"  per CU: {np.mean(conc):.1f} stamped workgroups; gap between consecutive workgroups median "
              f"{np.median(g):.2f} us (negative = overlap), min {g.min():.2f}, max {g.max():.2f}")


def main():
    torch.manual_seed(0)
    for S, C, H in ((64, 96, 3), (16, 384, 12)):
        for sh in (0, 3):
            run(S, C, H, sh)


if __name__ == "__main__":
    main()
