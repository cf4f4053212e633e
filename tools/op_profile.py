"""Attribute one training step's device time to torch ops (torch.profiler, grouped by input shape).

Usage (GPU box): python tools/op_profile.py <workload> [--size H W T] [--rows N]
Builds the bench workload (optionally at a smaller image size), runs 2 warm-up steps, profiles one step and prints
the top ops by self device time with their input shapes.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from long_context_biomedical_imaging_amd import config as lconfig  # noqa: E402
from long_context_biomedical_imaging_amd.model_base import EncoderDecoderModel  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import TrainStep, use_tuned_gemms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("--size", nargs=3, type=int, default=None, help="height width time")
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--ckpt", type=int, default=0)
    ap.add_argument("--rows", type=int, default=45)
    ap.add_argument("--stack", default="", help="comma-separated op names: print their time grouped by Python stack")
    args = ap.parse_args()
    extra = []
    if args.size:
        extra = ["--height", str(args.size[0]), "--width", str(args.size[1]), "--time", str(args.size[2])]
    dev = torch.device("cuda", 0)
    use_tuned_gemms()
    cfg = lconfig.parse_config(bench.WORKLOADS[args.workload] + ["--batch_size", str(args.batch)] + extra)
    torch.manual_seed(0)
    model = EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel,
                                cfg.no_out_channel).to(dev)
    if args.ckpt:
        model.encoder.checkpoint_blocks = args.ckpt
    ts = TrainStep(model, cfg, dev, ddp=False)
    x, y = bench.synthetic_batch(cfg, args.batch, dev, seed=1234)
    for _ in range(2):
        ts.step(x, y)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=bool(args.stack)) as prof:
        ts.step(x, y)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="self_cuda_time_total", row_limit=args.rows, max_name_column_width=40,
                   max_shapes_column_width=90))
    if args.stack:
        want = set(args.stack.split(","))
        for e in sorted(prof.key_averages(group_by_stack_n=6), key=lambda e: -e.self_device_time_total):
            if e.key in want and e.self_device_time_total > 0:
                print(f"{e.key} {e.self_device_time_total / 1e3:.2f} ms x{e.count}")
                for fr in e.stack[:6]:
                    print("     ", fr)


if __name__ == "__main__":
    main()
