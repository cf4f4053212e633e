#!/usr/bin/env python3
"""Headline benchmark: image-tokens/s fwd+bwd, ViT patch=2 at 512^2 (L = 65 536), 1..8 MI355X.

    python bench.py [--gpus N --steps K --warmup W]                (N = 1)
    torchrun --nproc-per-node N bench.py --gpus N ...               (N > 1; RCCL DDP)

A step = one DDP training step of the reference's segmentation model (trainer_base.py:157-182):
EncoderDecoderModel(ViT-small, p2, 512x512, 2-D) + ViTUNETR decoder, bf16 autocast, CrossEntropy loss,
backward (DDP gradient all-reduce over RCCL), Adam step — on synthetic U[0,1) images already on the GPU.
Throughput = (world * B * L) tokens / step time (max over ranks).

Also reported (rank 0): `roofline` of the dominant liblci kernel (HIP events over the timed region),
per-kernel breakdown, and `cpu_baseline` = the CPU oracle's forward on a bounded sample (N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from long_context_biomedical_imaging_amd import config as lconfig  # noqa: E402
from long_context_biomedical_imaging_amd import kernels  # noqa: E402
from long_context_biomedical_imaging_amd.model_base import EncoderDecoderModel  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import TrainStep, init_distributed, synthetic_batch  # noqa: E402

MFMA_BF16_PEAK_TFLOPS = 2500.0   # dense bf16, MI355X_MICROARCH.md chip table
HBM_PEAK_GBS = 8000.0

WORKLOADS = {
    # metric config: ViT-small, patch 2, 512x512 -> L = 65536 tokens per image
    "vit_p2_512": ["--encoder_name", "ViT", "--decoder_name", "ViTUNETR", "--task_type", "seg",
                   "--height", "512", "--width", "512", "--time", "1", "--no_in_channel", "1",
                   "--no_out_channel", "2", "--ViT.size", "small", "--ViT.patch_size", "1", "2", "2",
                   "--use_amp"],
}


def cpu_baseline(budget_s: float = 20.0):
    """Oracle (CPU restatement) forward of the same encoder, bounded sample, extrapolated per token.

    One 12-layer ViT-small layer at L = 65536 is: LN + qkv + out_proj + MLP over all tokens (timed on a
    4096-token slice, scaled x16) + attention (timed on `rows` query rows per head against all 65536 keys,
    scaled to all rows; rows are independent and equal work). tokens/s = L / (12 * t_layer).
    """
    from oracle import attention as oatt
    ncores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(ncores)
    L, D, H, dh, MLP = 65536, 384, 6, 64, 1536
    g = torch.Generator().manual_seed(0)
    w = {k: torch.randn(s, generator=g) * 0.02 for k, s in
         {"qkv": (3 * D, D), "out": (D, D), "l1": (MLP, D), "l2": (D, MLP)}.items()}
    x = torch.randn(1, 4096, D, generator=g)
    F = torch.nn.functional
    t0 = time.perf_counter()
    h = F.layer_norm(x, (D,))
    qkv = F.linear(h, w["qkv"])
    o = F.linear(qkv[..., :D], w["out"])
    h2 = F.layer_norm(x + o, (D,))
    _ = F.linear(F.gelu(F.linear(h2, w["l1"])), w["l2"])
    t_lin = (time.perf_counter() - t0) * (L / 4096)
    q = torch.randn(1, H, 1, dh, generator=g)
    k = torch.randn(1, H, L, dh, generator=g)
    v = torch.randn(1, H, L, dh, generator=g)
    rows, t_att, done = 256, 0.0, 0
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s * 0.8 and done < L:
        qs = q.expand(1, H, rows, dh).contiguous()
        t1 = time.perf_counter()
        oatt.attention_core(qs, k, v, dh ** -0.5)
        t_att += time.perf_counter() - t1
        done += rows
    t_layer = t_lin + t_att * (L / done)
    return {"value": round(L / (12 * t_layer), 1), "unit": "image-tokens/s (fwd only, fp32)", "cores": ncores,
            "kind": "port",
            "sample": f"oracle ViT-small encoder forward at L=65536, B=1: per layer, attention timed on {done} of "
                      f"65536 query rows per head (all keys) and the Linear/LN/MLP work on a 4096-token slice, "
                      f"both extrapolated linearly to the full layer, x12 layers"}


def profiled_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed PMC profile of this bench (profiles/traffic.json, written
    by tools/summarize_prof.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes), or None."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        prof = json.load(f)
    for name, d in prof.get("kernels", {}).items():
        if kernel + "_kernel" in name or name.endswith(kernel):
            return int(d["read_bytes"] + d["write_bytes"])
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2, help="images per GPU")
    ap.add_argument("--workload", default="vit_p2_512", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    args = ap.parse_args()

    rank, local, world = init_distributed()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    cfg = lconfig.parse_config(WORKLOADS[args.workload] + ["--batch_size", str(args.batch)])
    torch.manual_seed(0)
    model = EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel,
                                cfg.no_out_channel).to(device)
    trainer = TrainStep(model, cfg, device, ddp=world > 1)
    x, y = synthetic_batch(cfg, args.batch, device, seed=1234 + rank)
    L = model.encoder.patch_embedding.n_patches

    for _ in range(args.warmup):
        trainer.step(x, y)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kernels.KernelTimer.reset()
    kernels.KernelTimer.enabled = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = trainer.step(x, y)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernels.KernelTimer.enabled = False
    ksum = kernels.KernelTimer.summary()
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = t.item()
    loss_v = float(loss.item())

    if rank == 0:
        ms = 1000.0 * elapsed / args.steps
        tokens = world * args.batch * L * args.steps
        kern = {}
        for name, d in ksum.items():
            tf = d["work_per_call"] / (d["avg_ms"] * 1e-3) / 1e12 if d["work_per_call"] else None
            kern[name] = {"calls_per_step": d["calls"] / args.steps, "avg_ms": round(d["avg_ms"], 3),
                          "ms_per_step": round(d["total_ms"] / args.steps, 2),
                          "tflops": round(tf, 1) if tf else None}
        dom = max(ksum, key=lambda n: ksum[n]["total_ms"])
        dd = ksum[dom]
        ach = dd["work_per_call"] / (dd["avg_ms"] * 1e-3) / 1e12
        res = {
            "metric": "image-tokens/sec fwd+bwd, ViT patch=2 512^2 (L=65536), 1/2/4/8 MI355X",
            "value": round(tokens / elapsed, 1), "unit": "image-tokens/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic U[0,1) images, random-init weights",
            "config": {"workload": "ViT-small p2 512x512 2-D seg (ViTUNETR head), full attention",
                       "global_batch": world * args.batch, "seq_len": L, "parallelism": f"ddp{world}",
                       "per_gpu_batch": args.batch, "optimizer": cfg.optim_type, "loss": cfg.loss_func},
            "roofline": {"kernel": dom, "bound": "mfma", "achieved": round(ach, 1), "peak": MFMA_BF16_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(ach / MFMA_BF16_PEAK_TFLOPS, 4),
                         "traffic": profiled_traffic(dom), "traffic_source": "profiles/traffic.json",
                         "work_per_launch": dd["work_per_call"], "avg_launch_ms": round(dd["avg_ms"], 3)},
            "kernels": kern,
            "loss": round(loss_v, 5),
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_budget)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
