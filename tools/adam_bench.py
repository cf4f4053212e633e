import torch, time, sys
sys.path.insert(0, '.')
from long_context_biomedical_imaging_amd.trainer import LciAdam
from long_context_biomedical_imaging_amd import kernels
torch.manual_seed(0)
for sizes in ([1_500_000] * 40, [62_000_000 // 200] * 200, [16_000_000] * 4):
    ps = [torch.nn.Parameter(torch.randn(n, device='cuda')) for n in sizes]
    for p in ps: p.grad = torch.randn_like(p)
    for name, opt in (("torch_fused", torch.optim.Adam(ps, lr=1e-3, fused=True)), ("lci", LciAdam(ps, lr=1e-3))):
        for _ in range(3): opt.step()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20): opt.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 20 * 1e3
        n = sum(sizes)
        print(name, len(sizes), n, f"{ms:.3f} ms", f"{n * 28 / ms / 1e9:.2f} TB/s", flush=True)
    del ps
