"""lci_adam_step (csrc/optim.hip) through trainer.LciAdam / LciAdamW against torch's fused Adam / AdamW, the
optimizer the reference's trainer steps (trainer_base.py:171-177, optim_base.py:87-89)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

# sizes: tiny / ragged / one chunk / several chunks / unaligned tail; 45 tensors = two launches of <= 40
SIZES = [1, 3, 7, 384, 2047, 2048, 2049, 4096 + 5, 65536 + 3, 147456] * 4 + [1536, 384 * 1536, 96, 8, 9]


def _params(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.randn(n, device="cuda", generator=g) for n in SIZES]


@pytest.mark.parametrize("adamw,wd", [(False, 0.0), (False, 0.01), (True, 0.05)])
def test_lci_adam_matches_torch_fused(adamw, wd):
    from long_context_biomedical_imaging_amd.trainer import LciAdam, LciAdamW
    p_ref, p_lci = _params(1), _params(1)
    kw = dict(lr=3e-4, betas=(0.9, 0.95), weight_decay=wd, eps=1e-8)
    ref = (torch.optim.AdamW if adamw else torch.optim.Adam)([torch.nn.Parameter(p) for p in p_ref], fused=True, **kw)
    lci = (LciAdamW if adamw else LciAdam)([torch.nn.Parameter(p) for p in p_lci], **kw)
    g = torch.Generator(device="cuda").manual_seed(7)
    for _ in range(5):
        for a, b in zip(ref.param_groups[0]["params"], lci.param_groups[0]["params"]):
            gr = torch.randn(a.shape, device="cuda", generator=g)
            a.grad, b.grad = gr.clone(), gr.clone()
        ref.step()
        lci.step()
    worst = 0.0
    for a, b in zip(ref.param_groups[0]["params"], lci.param_groups[0]["params"]):
        sa, sb = ref.state[a], lci.state[b]
        assert float(sa["step"]) == float(sb["step"]) == 5.0
        for x, y in ((a, b), (sa["exp_avg"], sb["exp_avg"]), (sa["exp_avg_sq"], sb["exp_avg_sq"])):
            d = ((x - y).abs() / (x.abs() + 1e-30)).max().item()
            worst = max(worst, d)
    # the same formulas in the same precisions; only FMA contraction may differ: one f32 ulp
    assert worst <= 2.0 ** -22, f"max relative difference {worst:.3e}"


def test_lci_adam_state_dict_is_torch_compatible():
    from long_context_biomedical_imaging_amd.trainer import LciAdam
    ps = [torch.nn.Parameter(p) for p in _params(2)[:5]]
    lci = LciAdam(ps, lr=1e-3)
    for p in ps:
        p.grad = torch.ones_like(p)
    lci.step()
    ref = torch.optim.Adam([torch.nn.Parameter(p.detach().clone()) for p in ps], lr=1e-3, fused=True)
    ref.load_state_dict(lci.state_dict())
    assert set(ref.state_dict()["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
    assert torch.equal(ref.state_dict()["state"][3]["exp_avg"], lci.state_dict()["state"][3]["exp_avg"])


def test_lci_adam_graph_capture_replays():
    """The step (device step counts, bias corrections on the device) captured once and replayed = eager steps."""
    from long_context_biomedical_imaging_amd.trainer import LciAdam
    p_e, p_g = _params(3)[:12], _params(3)[:12]
    pe = [torch.nn.Parameter(p) for p in p_e]
    pg = [torch.nn.Parameter(p) for p in p_g]
    oe, og = LciAdam(pe, lr=1e-3, betas=(0.9, 0.95)), LciAdam(pg, lr=1e-3, betas=(0.9, 0.95))
    grads = [torch.randn_like(p) for p in pe]
    for p, gr in zip(pe, grads):
        p.grad = gr.clone()
    for p, gr in zip(pg, grads):
        p.grad = gr.clone()
    oe.step()
    og.step()   # state initialised outside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        og.step()
    for _ in range(3):
        graph.replay()
        oe.step()
    torch.cuda.synchronize()
    for a, b in zip(pe, pg):
        assert torch.equal(a, b)
    assert float(og.state[pg[0]]["step"]) == 4.0   # 1 eager step + 3 replays (the capture itself runs nothing)


def test_lci_adam_under_grad_scaler_skips_inf_and_unscales():
    """under torch.amp.GradScaler (the reference's loop, trainer_base.py:116,171-182) LciAdam must unscale
    the gradients and skip a step whose gradients hold an inf, like torch's fused Adam it derives from."""
    from long_context_biomedical_imaging_amd.trainer import LciAdam
    p_ref, p_lci = _params(3)[:12], _params(3)[:12]
    kw = dict(lr=1e-3, betas=(0.9, 0.95), eps=1e-8)
    ref = torch.optim.Adam([torch.nn.Parameter(p) for p in p_ref], fused=True, **kw)
    lci = LciAdam([torch.nn.Parameter(p) for p in p_lci], **kw)
    s_ref = torch.amp.GradScaler("cuda", init_scale=1024.0)
    s_lci = torch.amp.GradScaler("cuda", init_scale=1024.0)
    g = torch.Generator(device="cuda").manual_seed(11)
    for it in range(4):
        for a, b in zip(ref.param_groups[0]["params"], lci.param_groups[0]["params"]):
            gr = torch.randn(a.shape, device="cuda", generator=g) * s_ref.get_scale()
            if it == 2 and a.numel() > 4:
                gr[3] = float("inf")                     # an overflowed step: both must skip it
            a.grad, b.grad = gr.clone(), gr.clone()
        before = [b.detach().clone() for b in lci.param_groups[0]["params"]]
        one = torch.ones((), device="cuda")
        s_ref.scale(one)                                 # (a scaled loss: initialises the scalers' scale tensors)
        s_lci.scale(one)
        s_ref.step(ref)
        s_lci.step(lci)
        s_ref.update()
        s_lci.update()
        if it == 2:
            assert all(torch.equal(x, b) for x, b in zip(before, lci.param_groups[0]["params"])), "inf step applied"
    assert s_ref.get_scale() == s_lci.get_scale() == 512.0
    for a, b in zip(ref.param_groups[0]["params"], lci.param_groups[0]["params"]):
        assert torch.isfinite(b).all()
        assert float(ref.state[a]["step"]) == float(lci.state[b]["step"]) == 3.0
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)
