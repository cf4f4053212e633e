"""Which parameters get gradients whose strides differ from the parameter's (DDP's "Grad strides do not match
bucket view strides" warning under gradient_as_bucket_view): one micro-step of each test_ddp_model_gpu model."""
import sys
import torch
sys.path.insert(0, ".")
from tests.test_ddp_model_gpu import MODELS, COMMON, _batch  # noqa: E402
from long_context_biomedical_imaging_amd import config, model_base  # noqa: E402
from long_context_biomedical_imaging_amd.trainer import TrainStep  # noqa: E402

for name, (args, ckpt) in MODELS.items():
    cfg = config.parse_config(args + COMMON)
    torch.manual_seed(0)
    m = model_base.EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel,
                                       cfg.no_out_channel).cuda().train()
    ts = TrainStep(m, cfg, torch.device("cuda", 0), ddp=False)
    x, y = _batch(cfg, 0)
    ts.step(x.cuda(), y.cuda(), update=False)
    for n, p in m.named_parameters():
        if p.grad is not None and p.grad.stride() != p.stride():
            print(name, n, tuple(p.shape), "param", p.stride(), "grad", p.grad.stride())
    print(name, "done")
