"""Training BatchNorm + ReLU of UperNet's PSP bottleneck / FPN fusion (seg_heads.py:26-31, :60-63 and the 3-D
:158-163, :192-195) on the HIP kernels (kernels.batch_norm_relu: instance-norm reduction over the whole batch,
lci_bn_relu_fwd / _bwd_reduce / _bwd_apply) against torch's f32 batch_norm + relu of the same bf16 input.

Forward: within 1e-5 of |y| max (the statistics are combined in f64 from per-chunk f32 sums, torch uses Welford in
f32); running mean / var after the update within 1e-5 relative (momentum, unbiased variance). Backward: the input
gradient is rounded to the input's bf16 (as autocast's cast back would): rel-L2 <= 4e-3 of torch's f32 gradient;
weight / bias gradients rel-L2 <= 1e-4.
"""
import pytest
import torch
import torch.nn.functional as F

from golden_util import rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(2, 384, 66, 70), (2, 96, 17, 15), (1, 8, 5, 7), (2, 64, 9, 11, 13)])
def test_batch_norm_relu_vs_torch(shape):
    from long_context_biomedical_imaging_amd import kernels
    torch.manual_seed(sum(shape))
    C = shape[1]
    mf = torch.channels_last if len(shape) == 4 else torch.channels_last_3d
    x = (torch.randn(*shape, device="cuda") * 2 + 0.5).to(torch.bfloat16).to(memory_format=mf)
    bn = (torch.nn.BatchNorm2d if len(shape) == 4 else torch.nn.BatchNorm3d)(C).cuda().train()
    with torch.no_grad():
        bn.weight.copy_(1 + 0.2 * torch.randn(C))
        bn.bias.copy_(0.2 * torch.randn(C))
        bn.running_mean.copy_(0.1 * torch.randn(C))
        bn.running_var.copy_(1 + 0.1 * torch.rand(C))
    ref_bn = (torch.nn.BatchNorm2d if len(shape) == 4 else torch.nn.BatchNorm3d)(C).cuda().train()
    ref_bn.load_state_dict(bn.state_dict())
    assert kernels.batch_norm_relu_supported(x, bn)
    x1 = x.detach().clone().requires_grad_(True)
    x2 = x.detach().clone().requires_grad_(True)
    y1 = kernels.batch_norm_relu(x1, bn)
    y2 = F.relu(ref_bn(x2.float()))
    assert y1.dtype == torch.float32 and y1.shape == y2.shape
    assert (y1 - y2).abs().max().item() <= 1e-5 * y2.abs().max().item()
    assert rel_err(bn.running_mean, ref_bn.running_mean) < 1e-5
    assert rel_err(bn.running_var, ref_bn.running_var) < 1e-5
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1
    g = torch.randn(y2.shape, device="cuda")
    y1.backward(g)
    y2.backward(g)
    assert x1.grad.dtype == torch.bfloat16
    assert rel_err(x1.grad, x2.grad) < 4e-3
    assert rel_err(bn.weight.grad, ref_bn.weight.grad) < 1e-4
    assert rel_err(bn.bias.grad, ref_bn.bias.grad) < 1e-4
