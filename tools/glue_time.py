#!/usr/bin/env python3
"""Device time of every torch (aten) op of one training step, keyed by the module line (forward) or autograd node
(backward) that issued it: where the torch glue of a workload spends its time. liblci kernels are ctypes calls, not
aten ops, so they do not appear.

Each op is timed alone (the stream is synchronized before its start event), so a time includes ~5-10 us of launch
latency per kernel: rank with it, do not add it up against the bench line.

    python tools/glue_time.py swin_mamba_p2_128 [--rows 50]   (GPU box)
"""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from long_context_biomedical_imaging_amd import config as lconfig  # noqa: E402
from long_context_biomedical_imaging_amd.model_base import EncoderDecoderModel  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import TrainStep, synthetic_batch  # noqa: E402

SKIP = ("aten.view", "aten._unsafe_view", "aten.reshape", "aten.permute", "aten.t.", "aten.transpose",
        "aten.expand", "aten.as_strided", "aten.slice", "aten.select", "aten.unsqueeze", "aten.squeeze",
        "aten.detach", "aten.alias", "aten.empty", "aten.split", "aten.unbind", "aten.movedim", "aten.is_",
        "aten.sym_", "aten.lift", "aten._to_copy.default(cpu")


class Timed(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rec = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        key = str(func)
        if key.startswith(SKIP) or not any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
            return func(*args, **(kwargs or {}))
        node = torch._C._current_autograd_node()
        if node is not None:
            where = type(node).__name__
        else:
            fr = [f for f in traceback.extract_stack(limit=16) if "long_context_biomedical_imaging_amd" in f.filename]
            where = " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-2:][::-1]) if fr else "?"
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = func(*args, **(kwargs or {}))
        e1.record()
        shp = tuple(args[0].shape) if args and isinstance(args[0], torch.Tensor) else ()
        dt = str(args[0].dtype).replace("torch.", "") if args and isinstance(args[0], torch.Tensor) else ""
        self.rec.append((key, where, shp, dt, e0, e1))
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("--rows", type=int, default=50)
    ap.add_argument("--ckpt", type=int, default=None, help="checkpointed encoder blocks (default: bench.py's)")
    a = ap.parse_args()
    batch = 1 if a.workload in ("swin_p2_128", "vit_mamba_p2_256") else 2
    cfg = lconfig.parse_config(list(bench.WORKLOADS[a.workload]) + ["--batch_size", str(batch)])
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel, cfg.no_out_channel).to(dev)
    ckpt = a.ckpt if a.ckpt is not None else (10 if a.workload == "vit_mamba_p2_256" else 0)
    if ckpt:
        model.encoder.checkpoint_blocks = ckpt
    tr = TrainStep(model, cfg, dev, ddp=False)
    x, y = synthetic_batch(cfg, batch, dev, seed=1234)
    for _ in range(2):
        tr.step(x, y)
    torch.cuda.synchronize()
    mode = Timed()
    with mode:
        tr.step(x, y)
    torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    by_op = collections.defaultdict(float)
    total = 0.0
    for key, where, shp, dt, e0, e1 in mode.rec:
        ms = e0.elapsed_time(e1)
        agg[(key.split("(")[0], where, shp, dt)][0] += 1
        agg[(key.split("(")[0], where, shp, dt)][1] += ms
        by_op[key.split("(")[0]] += ms
        total += ms
    print(f"# {a.workload}: {len(mode.rec)} timed aten ops, {total:.2f} ms (incl. per-op launch latency)")
    for k, v in sorted(by_op.items(), key=lambda kv: -kv[1])[:15]:
        print(f"#   {v:8.3f} ms  {k}")
    for (k, where, shp, dt), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.rows]:
        print(f"{ms:8.3f} ms x{n:<3d} {k:34s} {dt:9s} {str(shp):30s} {where}")


if __name__ == "__main__":
    main()
