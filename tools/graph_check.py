#!/usr/bin/env python3
"""Eager vs HIP-graph training of one bench workload from the same seed: the loss of each step and the first
non-finite parameter, to find what a capture gets wrong.  python tools/graph_check.py <workload> [steps] (GPU box)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from long_context_biomedical_imaging_amd import config as lconfig  # noqa: E402
from long_context_biomedical_imaging_amd.model_base import EncoderDecoderModel  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import GraphedStep, TrainStep, synthetic_batch  # noqa: E402


def run(workload, steps, graphed):
    batch = 1 if workload in ("swin_p2_128", "vit_mamba_p2_256") else 2
    cfg = lconfig.parse_config(list(bench.WORKLOADS[workload]) + ["--batch_size", str(batch)])
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel, cfg.no_out_channel).to(dev)
    tr = TrainStep(model, cfg, dev, ddp=False)
    x, y = synthetic_batch(cfg, batch, dev, seed=1234)
    out = []

    def bad():
        for n, p in model.named_parameters():
            if not torch.isfinite(p).all():
                return n
        return None
    if graphed:
        gs = GraphedStep(tr, x, y, warmup=2)
        torch.cuda.synchronize()
        out.append(("after warmup + capture", None, bad()))
        for i in range(steps - 2):
            loss = gs.step()
            torch.cuda.synchronize()
            out.append((f"replay {i}", float(loss), bad()))
    else:
        for i in range(steps):
            loss = tr.step(x, y)
            torch.cuda.synchronize()
            out.append((f"eager {i}", float(loss), bad()))
    del tr, model
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    w = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    for g in (False, True):
        for row in run(w, steps, g):
            print(row, flush=True)
