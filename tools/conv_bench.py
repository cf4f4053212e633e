"""Per-shape timing of the decoder-head conv kernels (csrc/conv.hip): forward, data gradient, weight gradient.

HIP events around each launch on the current stream, random bf16 data, channels-last. Prints one JSON line per
(shape, pass) with ms and TFLOP/s (2 * V * 27 * Cin * Cout per pass; 9 taps in 2-D).
Usage (GPU box): python tools/conv_bench.py [--set c3|c5|2d|all]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from long_context_biomedical_imaging_amd import kernels  # noqa: E402

SETS = {
    # Swin-tiny + SwinUNETR at 128^3 patch 2
    "c3": [((128, 128, 128), 96, 96), ((128, 128, 128), 192, 96), ((64, 64, 64), 96, 96), ((64, 64, 64), 192, 96),
           ((32, 32, 32), 192, 192), ((32, 32, 32), 384, 192), ((16, 16, 16), 384, 384)],
    # A/B mix of tile widths (NT = 1..4) at 128^3
    "mix": [((128, 128, 128), 96, 96), ((128, 128, 128), 192, 96), ((128, 128, 128), 256, 128),
            ((128, 128, 128), 512, 256), ((128, 128, 128), 64, 64), ((128, 128, 128), 64, 32)],
    # ViT + ViTUNETR at 256^3 patch 2: the whole decoder runs at full resolution (enhance_heads.py:221-224)
    "c5": [((256, 256, 256), 512, 256), ((256, 256, 256), 256, 256), ((256, 256, 256), 256, 128),
           ((256, 256, 256), 128, 128), ((256, 256, 256), 128, 64), ((256, 256, 256), 64, 64),
           ((256, 256, 256), 64, 32), ((256, 256, 256), 32, 32)],
    # ViT + ViTUNETR at 512^2 patch 2 (2-D: D = 1), full resolution likewise
    "2d": [((1, 512, 512), 512, 256), ((1, 512, 512), 256, 256), ((1, 512, 512), 256, 128),
           ((1, 512, 512), 128, 64), ((1, 512, 512), 64, 32), ((1, 512, 512), 32, 32)],
}


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="all")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fill", type=float, default=0.0, help="GB of device memory to hold in 1-GB blocks first")
    ap.add_argument("--only", default="")
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    args = ap.parse_args()
    hold = [torch.empty(1 << 30, dtype=torch.uint8, device="cuda") for _ in range(int(args.fill))]
    names = ["c3", "c5", "2d"] if args.set == "all" else args.set.split(",")
    dev = torch.device("cuda")
    for sname in names:
        for S, cin, cout in SETS[sname]:
            if args.only and f"{cin}-{cout}" != args.only:
                continue
            kd = 1 if S[0] == 1 else 3
            V = S[0] * S[1] * S[2]
            x = torch.randn(1, *S, cin, device=dev).bfloat16()
            dy = torch.randn(1, *S, cout, device=dev).bfloat16()
            w = (torch.randn(cout, kd * 9, cin, device=dev) * 0.05).bfloat16()
            wd = (torch.randn(cin, kd * 9, cout, device=dev) * 0.05).bfloat16()
            fl = 2.0 * V * kd * 9 * cin * cout
            for pas, fn in (("fwd", lambda: kernels.conv3_cl(x, w, kd)),
                            ("dgrad", lambda: kernels.conv3_cl(dy, wd, kd)),
                            ("wgrad", lambda: kernels.conv3_wgrad_cl(x, dy, kd))):
                if pas not in args.passes.split(","):
                    continue
                ms = timeit(fn, args.reps if V < 4_000_000 else 2)
                print(json.dumps({"fill": args.fill, "set": sname, "S": S, "cin": cin, "cout": cout, "pass": pas, "ms": round(ms, 3),
                                  "tflops": round(fl / ms / 1e9, 1)}), flush=True)
            del x, dy, w, wd
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
