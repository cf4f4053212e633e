"""Find which autograd ops launch the large f32 elementwise adds of the ViT-Mamba (C5) backward: the C5 config at a
reduced volume (64^3 patch 2 -> L = 32768), per-block checkpointing as in bench.py, one training step under
torch.profiler; prints aten::add / add_ calls with their input shapes and the Python frames that issued them."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from long_context_biomedical_imaging_amd import config as lconfig  # noqa: E402
from long_context_biomedical_imaging_amd.model_base import EncoderDecoderModel  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import TrainStep  # noqa: E402

args = list(bench.WORKLOADS["vit_mamba_p2_256"])
for k in ("--height", "--width", "--time"):
    args[args.index(k) + 1] = "64"
cfg = lconfig.parse_config(args + ["--batch_size", "1"])
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel, cfg.no_out_channel).to(dev)
model.encoder.checkpoint_blocks = True
ts = TrainStep(model, cfg, dev, ddp=False)
x, y = bench.synthetic_batch(cfg, 1, dev, seed=0)
ts.step(x, y)
torch.cuda.synchronize()
with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], record_shapes=True, with_stack=True) as p:
    ts.step(x, y)
    torch.cuda.synchronize()
L = 32 ** 3
for ev in p.events():
    if ev.name in ("aten::add", "aten::add_") and ev.input_shapes and ev.input_shapes[0] and \
            len(ev.input_shapes[0]) >= 2 and ev.input_shapes[0][-2:] == [L, 384]:
        st = [s for s in (ev.stack or []) if "site-packages" not in s][:6]
        print(ev.name, ev.input_shapes, ev.input_types if hasattr(ev, "input_types") else "", "|", " <- ".join(st),
              flush=True)
