"""One training step pinned to the reference (trainer/trainer_base.py:154-189 drives
forward, loss, backward and the optimizer step).

tests/golden/train_step.npz was produced by tools/gen_golden.py:train_step from the reference's own
ViT_with_alt_ops (backbone_vit.py:276-397, imported from /root/reference on CPU, fp32): a 2-layer ViT encoder
(16x16 image, patch 2, hidden 128, 2 heads) + mean-pooled Linear head, MSE loss, one SGD step (lr 0.1). It
holds the initial weights, the batch, the loss and, per parameter, (sum, sum|.|) after the step.

Here the same weights and batch go through this package's modules on the GPU (HIP patch embed, LayerNorm,
flash attention; fp32 model, bf16 attention operands inside the kernel) and torch.optim.SGD takes the step.
Tolerances (bf16 attention vs the reference's fp32 CPU attention): loss within 5e-3 relative; per parameter,
the update's signed sum -lr sum(g) within 2e-2 of lr sum|g| (the gradient's L1 mass) of the reference's, and
the post-step sum|w| within the same bound plus 1e-6 sum|w|.
"""
import numpy as np
import pytest
import torch

from golden_util import Golden

pytestmark = pytest.mark.gpu


def test_train_step_matches_reference_fixture():
    from long_context_biomedical_imaging_amd import backbone_vit
    g = Golden("train_step")
    torch.manual_seed(0)
    enc = backbone_vit.ViT_with_alt_ops(False, False, in_channels=1, img_size=(16, 16), patch_size=(2, 2),
                                        hidden_size=128, mlp_dim=256, num_layers=2, num_heads=2, dropout_rate=0.0,
                                        spatial_dims=2)
    head = torch.nn.Linear(128, 3)
    sd = g.sd()
    enc.load_state_dict({k[4:]: v for k, v in sd.items() if k.startswith("enc.")})
    head.load_state_dict({k[5:]: v for k, v in sd.items() if k.startswith("head.")})
    enc, head = enc.cuda().eval(), head.cuda()
    x, y = g.t("in/x").cuda(), g.t("in/y").cuda()
    pre = {**{f"enc.{k}": v.detach().double().cpu().clone() for k, v in enc.state_dict().items()},
           **{f"head.{k}": v.detach().double().cpu().clone() for k, v in head.state_dict().items()}}
    named = [(f"enc.{n}", p) for n, p in enc.named_parameters()] + [(f"head.{n}", p) for n, p in head.named_parameters()]
    opt = torch.optim.SGD([p for _, p in named], lr=0.1)
    loss = torch.nn.functional.mse_loss(head(enc(x)[-1].mean(1)), y)
    loss.backward()
    grads = {n: p.grad.detach().double().cpu().clone() for n, p in named}
    opt.step()
    ref_loss = g.scalar("out/loss")
    assert abs(loss.item() - ref_loss) <= 5e-3 * abs(ref_loss), (loss.item(), ref_loss)
    post = {**{f"enc.{k}": v for k, v in enc.state_dict().items()}, **{f"head.{k}": v for k, v in head.state_dict().items()}}
    checked = 0
    for name, w in post.items():
        key = f"post_sum/{name}"
        if not g.has(key):
            continue
        ref_sum, ref_abs = np.asarray(g.z[key], dtype=np.float64)
        w = w.detach().double().cpu()
        l1 = 0.1 * grads[name].abs().sum().item() if name in grads else 0.0
        tol = 2e-2 * l1 + 1e-9
        d_ours, d_ref = w.sum().item() - pre[name].sum().item(), ref_sum - pre[name].sum().item()
        assert abs(d_ours - d_ref) <= tol, f"{name}: update sum {d_ours:.6g} vs reference {d_ref:.6g}"
        assert abs(w.abs().sum().item() - ref_abs) <= tol + 1e-6 * ref_abs, f"{name}: sum|w|"
        checked += 1
    assert checked == len(named)
