"""trainer.GraphedStep: the training step captured into one HIP graph and replayed (bench.py's mode for the
host-bound Swin workloads) must train exactly like the eager TrainStep: same weights after the same number of steps
(the liblci kernels are deterministic; fused Adam's capturable form keeps its step count on the device, so the bias
corrections are evaluated there in f32 instead of on the host: agreement to 1e-5 relative, not bitwise)."""
import pytest
import torch


def _run(graphed, steps=4):
    from long_context_biomedical_imaging_amd import backbone_swin, config
    from long_context_biomedical_imaging_amd.trainer import GraphedStep, TrainStep
    torch.manual_seed(0)
    model = torch.nn.Sequential(
        backbone_swin.BasicLayer(False, False, dim=64, depth=2, num_heads=2, window_size=(4, 4, 4),
                                 drop_path=[0.0, 0.0], downsample=None)).cuda()
    cfg = config.parse_config(["--optim_type", "adam", "--optim.lr", "1e-3", "--loss_func", "MSE", "--use_amp"])
    ts = TrainStep(model, cfg, torch.device("cuda"), ddp=False)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 64, 6, 8, 8, generator=g).cuda()
    y = torch.randn(2, 64, 6, 8, 8, generator=g).cuda()
    if graphed:
        gs = GraphedStep(ts, x, y, warmup=2)    # 2 eager warm-up steps, then replays
        for _ in range(steps - 2):
            loss = gs.step()
    else:
        for _ in range(steps):
            loss = ts.step(x, y)
    torch.cuda.synchronize()
    return float(loss), [p.detach().float().cpu() for p in model.parameters()]


@pytest.mark.gpu
def test_graphed_step_matches_eager():
    l0, w0 = _run(False)
    l1, w1 = _run(True)
    assert abs(l0 - l1) <= 1e-5 * max(1.0, abs(l0))
    for a, b in zip(w0, w1):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max()
