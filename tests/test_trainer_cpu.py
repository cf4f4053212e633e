"""TrainStep semantics of the reference's step loop (trainer/trainer_base.py:154-182), on torch-only models (CPU):
gradient accumulation over `iters_to_accumulate` micro-batches, grad-norm clipping, and the batch-of-1 duplication."""
import copy

import pytest
import torch

from long_context_biomedical_imaging_amd import config
from long_context_biomedical_imaging_amd.trainer import TrainStep


def _cfg(*extra):
    return config.parse_config(["--optim_type", "sgd", "--optim.lr", "0.1", "--loss_func", "MSE", *extra])


def _mlp():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 4))


def test_accumulation_matches_one_full_batch():
    """N accumulated half-batches (loss / N each, one optimizer step at the end of the window) land on the same
    weights as one step on the full batch; in between no update happens (trainer_base.py:169-179)."""
    g = torch.Generator().manual_seed(3)
    x, y = torch.randn(8, 8, generator=g), torch.randn(8, 4, generator=g)
    full = _mlp()
    TrainStep(full, _cfg(), torch.device("cpu"), ddp=False).step(x, y)
    acc = _mlp()
    w0 = [p.detach().clone() for p in acc.parameters()]
    ts = TrainStep(acc, _cfg("--iters_to_accumulate", "2"), torch.device("cpu"), ddp=False)
    ts.step(x[:4], y[:4])
    for a, b in zip(acc.parameters(), w0):
        assert torch.equal(a, b), "no optimizer step inside an accumulation window"
    ts.step(x[4:], y[4:])
    for a, b in zip(acc.parameters(), full.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
    assert ts.micro == 0


def test_clip_grad_norm():
    """--clip_grad_norm c: the update is lr * g * c / ||g|| when ||g|| > c (trainer_base.py:173-175)."""
    g = torch.Generator().manual_seed(4)
    x, y = 10 * torch.randn(8, 8, generator=g), 10 * torch.randn(8, 4, generator=g)
    ref = _mlp()
    loss = torch.nn.functional.mse_loss(ref(x), y)
    loss.backward()
    gn = torch.sqrt(sum((p.grad ** 2).sum() for p in ref.parameters()))
    assert gn > 0.5
    want = [p.detach() - 0.1 * p.grad * (0.5 / (gn + 1e-6)) for p in ref.parameters()]
    m = _mlp()
    TrainStep(m, _cfg("--clip_grad_norm", "0.5"), torch.device("cpu"), ddp=False).step(x, y)
    for a, b in zip(m.parameters(), want):
        torch.testing.assert_close(a.detach(), b, rtol=1e-5, atol=1e-6)


class _BNNet(torch.nn.Module):
    """Pools to one value per channel before a BatchNorm, like UperNet's PSP bin-1 stage (seg_heads.py)."""

    def __init__(self):
        super().__init__()
        self.conv = torch.nn.Conv2d(1, 4, 3, padding=1)
        self.bn = torch.nn.BatchNorm2d(4)
        self.head = torch.nn.Conv2d(4, 1, 1)

    def forward(self, x):
        p = self.bn(torch.nn.functional.adaptive_avg_pool2d(self.conv(x), 1))
        return self.head(p).expand(-1, -1, x.shape[2], x.shape[3])


def test_batch_of_one_duplicated_for_batchnorm():
    """A batch of 1 trains (duplicated to 2, trainer_base.py:160-164) where plain BatchNorm training raises, and the
    step equals the explicit duplicate's."""
    torch.manual_seed(0)
    net = _BNNet()
    x, y = torch.rand(1, 1, 6, 6), torch.rand(1, 1, 6, 6)
    with pytest.raises(ValueError):
        copy.deepcopy(net).train()(x)
    a, b = copy.deepcopy(net), copy.deepcopy(net)
    ts = TrainStep(a, _cfg(), torch.device("cpu"), ddp=False)
    assert ts.dup_batch1
    ts.step(x, y)
    TrainStep(b, _cfg(), torch.device("cpu"), ddp=False).step(torch.cat([x, x]), torch.cat([y, y]))
    for p, q in zip(a.state_dict().values(), b.state_dict().values()):
        assert torch.equal(p, q)


def test_batch_of_one_without_batchnorm_not_duplicated():
    """Without a BatchNorm the duplicate is the identity (mean loss over two equal samples), so it is skipped."""
    m = _mlp()
    ts = TrainStep(m, _cfg(), torch.device("cpu"), ddp=False)
    assert not ts.dup_batch1
    x, y = torch.randn(1, 8), torch.randn(1, 4)
    ref = _mlp()
    TrainStep(ref, _cfg(), torch.device("cpu"), ddp=False).step(torch.cat([x, x]), torch.cat([y, y]))
    ts.step(x, y)
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)
