"""Find which Python frames issue the strided tensor copies (aten::copy_ / clone / contiguous) of a training step:
a bench workload at a reduced image size, one step under torch.profiler with stacks; prints the copy events whose
first input has at least MIN_NUMEL elements, grouped by (shape, frames), with counts.
Usage (GPU box): python tools/trace_copies.py vit_hyena_p2_1024 256"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from long_context_biomedical_imaging_amd import config as lconfig  # noqa: E402
from long_context_biomedical_imaging_amd.model_base import EncoderDecoderModel  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import TrainStep  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "vit_hyena_p2_1024"
size = sys.argv[2] if len(sys.argv) > 2 else "256"
args = list(bench.WORKLOADS[wl])
for k in ("--height", "--width"):
    if k in args:
        args[args.index(k) + 1] = size
BATCH = int(os.environ.get("TRACE_BATCH", "2"))
cfg = lconfig.parse_config(args + ["--batch_size", str(BATCH)])
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel, cfg.no_out_channel).to(dev)
if os.environ.get("TRACE_CKPT"):
    model.encoder.checkpoint_blocks = int(os.environ["TRACE_CKPT"])   # per-block activation checkpointing (C5)
ts = TrainStep(model, cfg, dev, ddp=False)
x, y = bench.synthetic_batch(cfg, BATCH, dev, seed=0)
ts.step(x, y)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as p:
    ts.step(x, y)
    torch.cuda.synchronize()
NAMES = set((os.environ.get("TRACE_OPS") or "aten::copy_,aten::clone,aten::contiguous").split(","))
MIN_NUMEL = int(os.environ.get("TRACE_MIN_NUMEL", 1 << 20))
agg = collections.Counter()
tm = collections.Counter()
for ev in p.events():
    if ev.name in NAMES and ev.input_shapes and ev.input_shapes[0]:
        n = 1
        for d in ev.input_shapes[0]:
            n *= d
        if n < MIN_NUMEL:
            continue
        st = [s for s in (ev.stack or []) if "site-packages" not in s and "torch/" not in s][:5]
        if not st:   # no Python frames recorded (ROCm builds): the enclosing ops instead
            par, up = ev.cpu_parent, []
            while par is not None and len(up) < 4:
                up.append(par.name)
                par = par.cpu_parent
            st = up
        key = (ev.name, str(ev.input_shapes[:2]), " <- ".join(st))
        agg[key] += 1
        tm[key] += ev.device_time_total
for key, t in tm.most_common(50):
    name, shp, st = key
    print(f"{t / 1e3:8.3f} ms {agg[key]:4d} {name} {shp} | {st}", flush=True)
