"""Price the one-kernel attention backward (dK/dV + dQ in one pass, dQ summed over key blocks) on MI355X.

A fused backward executes 10f MFMA work instead of today's 14f (f = B H L^2 d), but dQ must then be summed over the
L / KW key blocks that each hold one workgroup's dK/dV accumulators (KW keys per CU: 256 today; 512 = every register
of a CU). Every (key block, query tile) contributes a 64 x 64 f32 dQ partial: (L / KW) * L * 64 * 4 B
per (batch, head) written and read back once (partials + a reduction pass; an in-L2 hand-off moves the same bytes).
This measures that traffic's floor with plain torch streams (fill_ = write, sum(0) = read + small write) at the
metric shape and prints it beside the measured dQ kernel it would replace.

Usage (GPU box): python tools/attn_fused_price.py [--L 65536 --B 2 --H 6]
"""
import argparse
import json

import torch


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=65536)
    ap.add_argument("--B", type=int, default=2)
    ap.add_argument("--H", type=int, default=6)
    args = ap.parse_args()
    L, BH = args.L, args.B * args.H
    for kw in (256, 512, 1024):
        nkb = L // kw
        part = torch.empty(nkb, L, 64, device="cuda", dtype=torch.float32)     # one (batch, head)
        gb = part.numel() * 4 / 1e9
        t_w = timed(lambda: part.fill_(1.0))
        t_r = timed(lambda: part.sum(0))
        del part
        torch.cuda.empty_cache()
        print(json.dumps({"keys_per_workgroup": kw, "partials_gb_per_layer": round(gb * BH, 2),
                          "write_ms_per_layer": round(t_w * BH, 2), "reduce_ms_per_layer": round(t_r * BH, 2),
                          "write_gbs": round(gb / (t_w * 1e-3), 0), "reduce_read_gbs": round(gb / (t_r * 1e-3), 0),
                          "traffic_ms_per_layer": round((t_w + t_r) * BH, 2)}), flush=True)


if __name__ == "__main__":
    main()
