"""Where the non-liblci GPU time of a training step goes (torch glue: casts, copies, reductions, optimizer).

    python tools/glue_profile.py --workload vit_hyena_p2_1024 [--rows 40] > gpurun_out/glue.txt

Builds the workload's model and TrainStep exactly as bench.py does, runs two warm-up steps, then one step under
torch.profiler (CPU + device activity, Python stacks) and prints the aten ops by self device time, grouped by input
shape and by the model-code stack that issued them. liblci kernels are launched through ctypes, so they do not
appear as aten ops: what is listed is exactly the torch-side work.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from long_context_biomedical_imaging_amd import config as lconfig  # noqa: E402
from long_context_biomedical_imaging_amd.model_base import EncoderDecoderModel  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import TrainStep, synthetic_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="vit_hyena_p2_1024")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--rows", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    batch = a.batch or (1 if a.workload in ("swin_p2_128", "vit_mamba_p2_256") else 2)
    cfg = lconfig.parse_config(bench.WORKLOADS[a.workload] + ["--batch_size", str(batch)])
    torch.manual_seed(0)
    model = EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel,
                                cfg.no_out_channel).to(dev)
    if a.workload == "vit_mamba_p2_256":
        model.encoder.checkpoint_blocks = 10
    tr = TrainStep(model, cfg, dev, ddp=False)
    x, y = synthetic_batch(cfg, batch, dev, seed=1234)
    for _ in range(2):
        tr.step(x, y)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        tr.step(x, y)
        torch.cuda.synchronize()
    key = "self_device_time_total"
    print(f"# {a.workload}: aten ops by self device time (one step), grouped by input shape")
    print(prof.key_averages(group_by_input_shape=True).table(sort_by=key, row_limit=a.rows, max_name_column_width=40,
                                                             max_shapes_column_width=70))
    print(f"# {a.workload}: grouped by the issuing stack (5 frames)")
    print(prof.key_averages(group_by_stack_n=5).table(sort_by=key, row_limit=a.rows, max_name_column_width=40,
                                                      max_src_column_width=110))


if __name__ == "__main__":
    main()
