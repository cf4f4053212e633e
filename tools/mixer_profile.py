"""Profile one token-mixer block fwd+bwd (torch.profiler, device time by op) at a BASELINE shape.

    python tools/mixer_profile.py mamba [--L 2097152 --B 1 --D 384]
    python tools/mixer_profile.py hyena [--L 262144 --B 2 --D 384]

Prints the ops by self device time (HIP kernels of liblci, hipBLASLt GEMMs, torch elementwise), so the glue around
the mixer kernels can be priced against the kernels themselves.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from long_context_biomedical_imaging_amd import hyena, mamba  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import use_tuned_gemms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mixer", choices=["mamba", "hyena"])
    ap.add_argument("--L", type=int, default=None)
    ap.add_argument("--B", type=int, default=None)
    ap.add_argument("--D", type=int, default=384)
    ap.add_argument("--rows", type=int, default=30)
    args = ap.parse_args()
    use_tuned_gemms()
    torch.manual_seed(0)
    if args.mixer == "mamba":
        L, B = args.L or (1 << 21), args.B or 1
        m = mamba.MambaVisionMixer(d_model=args.D, d_state=8, d_conv=3, expand=1).cuda()
    else:
        L, B = args.L or 262144, args.B or 2
        m = hyena.HyenaOperator(d_model=args.D, l_max=max(L, 66000), filter_order=64, num_heads=6, num_blocks=1,
                                short_filter_order=5, bidrectional=True, dropout=0.0, filter_dropout=0.0,
                                activation="id").cuda()
    x = torch.randn(B, L, args.D, device="cuda", requires_grad=True)
    g = torch.randn(B, L, args.D, device="cuda", dtype=torch.bfloat16)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.backward(g)

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=args.rows,
                                                            max_name_column_width=60))


if __name__ == "__main__":
    main()
