"""Does any part of a model couple the samples of a batch? Runs the test_ddp_model_gpu models on a batch of 2 and on
each sample alone (same weights), under bf16 autocast and in fp32, and prints the per-sample output difference and
the parameter gradients that differ most between the batch-of-2 run and the sum of the single-sample runs (mean
loss: grad(B=2) = (grad(x0) + grad(x1)) / 2 exactly, up to rounding, when nothing couples the samples).
Also prints the intermediate hidden states' per-sample differences (forward hooks on the encoder's blocks).
Usage (GPU box): python tools/r6_batch_coupling.py [model ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_ddp_model_gpu import MODELS, COMMON, _batch  # noqa: E402
from long_context_biomedical_imaging_amd import config, model_base  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


def run(name, amp):
    args, ckpt = MODELS[name]
    cfg = config.parse_config(args + COMMON)
    torch.manual_seed(0)
    m = model_base.EncoderDecoderModel(cfg, cfg.encoder_name, cfg.decoder_name, cfg.no_in_channel,
                                       cfg.no_out_channel).cuda().train()
    if ckpt:
        m.encoder.checkpoint_blocks = True
    xs, ys = zip(*(_batch(cfg, r) for r in range(2)))
    feats = {}

    def hook(nm):
        def f(mod, inp, out):
            o = out[0] if isinstance(out, (tuple, list)) else out
            if torch.is_tensor(o):
                feats.setdefault(nm, []).append(o.detach().float().clone())
        return f
    hs = [mod.register_forward_hook(hook(nm)) for nm, mod in m.named_modules()
          if nm.count(".") <= 2 and nm and not isinstance(mod, (torch.nn.ModuleList, torch.nn.Sequential))]

    def step(x, y):
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = m(x.cuda())
            out = out[0] if isinstance(out, (tuple, list)) else out
            loss = torch.nn.functional.cross_entropy(out.float(), y.cuda())
        loss.backward()
        return out.detach().float(), {n: p.grad.detach().float().clone() for n, p in m.named_parameters()
                                      if p.grad is not None}
    feats.clear()
    o2, g2 = step(torch.cat(xs), torch.cat(ys))
    f2 = {k: v[0] for k, v in feats.items()}
    feats.clear()
    oa, ga = step(xs[0], ys[0])
    fa = {k: v[0] for k, v in feats.items()}
    feats.clear()
    ob, gb = step(xs[1], ys[1])
    fb = {k: v[0] for k, v in feats.items()}
    for h in hs:
        h.remove()
    print(f"== {name} amp={amp}: output rel diff sample0 {rel(o2[:1], oa):.2e} sample1 {rel(o2[1:], ob):.2e}")
    worst = []
    for k in f2:
        if k in fa and f2[k].shape[0] == 2 and fa[k].shape[0] == 1 and f2[k].shape[1:] == fa[k].shape[1:]:
            worst.append((max(rel(f2[k][:1], fa[k]), rel(f2[k][1:], fb[k])), k, tuple(fa[k].shape)))
    worst.sort(reverse=True)
    for w in worst[:8]:
        print(f"   hidden {w[1]} {w[2]}: {w[0]:.2e}")
    gd = []
    for n in g2:
        ref = (ga[n] + gb[n]) / 2
        gd.append((rel(g2[n], ref), n, ref.norm().item()))
    gd.sort(reverse=True)
    num = sum(((g2[n] - (ga[n] + gb[n]) / 2) ** 2).sum().item() for n in g2)
    den = sum((((ga[n] + gb[n]) / 2) ** 2).sum().item() for n in g2)
    print(f"   grads: global rel {(num / den) ** 0.5:.2e}; worst:")
    for d in gd[:10]:
        print(f"     {d[1]}: rel {d[0]:.2e} (|g| {d[2]:.2e})")


def main():
    names = sys.argv[1:] or sorted(MODELS)
    for nm in names:
        for amp in (False, True):
            run(nm, amp)


if __name__ == "__main__":
    main()
