"""Multi-process data-parallel step: world_size 2, gloo.

CPU test: the TrainStep/DDP plumbing on a torch-only model — gradients are averaged across ranks and the
post-step weights are identical on every rank and equal to a single-process step on the concatenated batch.
GPU test: two ranks on one GPU (gloo carries the all-reduce) training a ViT block through the HIP kernels.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg():
    from long_context_biomedical_imaging_amd import config
    return config.parse_config(["--optim_type", "sgd", "--optim.lr", "0.1", "--loss_func", "MSE"])


def _cpu_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from long_context_biomedical_imaging_amd.trainer import TrainStep
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 4))
    ts = TrainStep(model, _cfg(), torch.device("cpu"), ddp=True)
    g = torch.Generator().manual_seed(100 + rank)
    x, y = torch.randn(4, 8, generator=g), torch.randn(4, 4, generator=g)
    ts.step(x, y)
    q.put((rank, [p.detach().numpy().copy() for p in model.parameters()]))  # by value
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_two_ranks_cpu_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for a, b in zip(res[0], res[1]):
        assert (a == b).all()
    # single-process reference: mean of per-rank losses == loss on the concatenated batch (equal batch sizes)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 4))
    xs, ys = [], []
    for r in range(2):
        g = torch.Generator().manual_seed(100 + r)
        xs.append(torch.randn(4, 8, generator=g))
        ys.append(torch.randn(4, 4, generator=g))
    loss = torch.nn.functional.mse_loss(model(torch.cat(xs)), torch.cat(ys))
    loss.backward()
    with torch.no_grad():
        for p in model.parameters():
            p -= 0.1 * p.grad
    for a, b in zip(res[0], model.parameters()):
        assert torch.allclose(torch.from_numpy(a), b, atol=1e-6)


def _gpu_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from long_context_biomedical_imaging_amd import backbone_vit
    from long_context_biomedical_imaging_amd.trainer import TrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = torch.nn.Sequential(backbone_vit.TransformerBlock(False, False, 128, 256, 2),
                                backbone_vit.TransformerBlock(False, True, 128, 256, 2)).to(dev)
    cfg = _cfg()
    cfg.use_amp = True
    ts = TrainStep(model, cfg, dev, ddp=True)
    g = torch.Generator().manual_seed(7 + rank)
    x = torch.randn(2, 300, 128, generator=g).to(dev)
    y = torch.randn(2, 300, 128, generator=g).to(dev)
    loss = ts.step(x, y)
    torch.cuda.synchronize()
    q.put((rank, float(loss), [p.detach().float().cpu().numpy().copy() for p in model.parameters()]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_ddp_two_ranks_gpu_kernels():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, loss, params = q.get(timeout=300)
        res[r] = params
        assert loss == loss  # finite
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for a, b in zip(res[0], res[1]):
        assert (a == b).all()


def _bench_worker(rank, world, port, q):
    """One rank of bench.py's timing harness (timed_steps) around a DDP step on CPU/gloo: rank 1 is made slower,
    so the reported time must be the max over ranks, and the weights must stay identical across ranks."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LCI_DIST_BACKEND="gloo")   # CPU ranks even on a GPU box
    import bench
    from long_context_biomedical_imaging_amd.trainer import TrainStep, init_distributed
    r, local, w = init_distributed()          # the harness's own rendezvous path (gloo without a GPU)
    assert (r, w) == (rank, world) and dist.is_initialized()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.GELU(), torch.nn.Linear(16, 4))
    ts = TrainStep(model, _cfg(), torch.device("cpu"), ddp=True)
    g = torch.Generator().manual_seed(100 + rank)
    x, y = torch.randn(4, 8, generator=g), torch.randn(4, 4, generator=g)

    def step():
        if rank == 1:
            time.sleep(0.05)
        return ts.step(x, y)

    t0 = time.perf_counter()
    elapsed, loss = bench.timed_steps(step, 4, 1, world, torch.device("cpu"), rank)
    mine = time.perf_counter() - t0
    q.put((rank, elapsed, mine, float(loss), [p.detach().numpy().copy() for p in model.parameters()]))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_harness_two_ranks_cpu_gloo():
    """bench.py's N > 1 path rehearsed on CPU (world size 2, gloo): barrier-bracketed timing, max over ranks,
    DDP gradient all-reduce keeping the replicas identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (e, m, l, w) for r, e, m, l, w in (q.get(timeout=180) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    e0, e1 = res[0][0], res[1][0]
    assert e0 == e1, "every rank reports the same (max) time"
    assert e0 >= 4 * 0.05, "the slow rank's 4 timed steps bound the reported time"
    for a, b in zip(res[0][3], res[1][3]):
        assert (a == b).all()


def _rccl_worker(port, q):
    """One rank on backend "nccl" (= RCCL on ROCm): the DDP gradient all-reduce and bench.timed_steps' barrier /
    MAX all-reduce run through RCCL itself (world size 1: a one-GPU box cannot host two RCCL ranks)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import bench
    from long_context_biomedical_imaging_amd import backbone_vit
    from long_context_biomedical_imaging_amd.trainer import TrainStep
    t = torch.arange(1024, device=dev, dtype=torch.float32)
    dist.all_reduce(t)
    ok_ar = bool(torch.equal(t, torch.arange(1024, device=dev, dtype=torch.float32)))
    res = []
    for ddp in (True, False):
        torch.manual_seed(0)
        model = torch.nn.Sequential(backbone_vit.TransformerBlock(False, False, 128, 256, 2),
                                    backbone_vit.TransformerBlock(False, True, 128, 256, 2)).to(dev)
        cfg = _cfg()
        cfg.use_amp = True
        ts = TrainStep(model, cfg, dev, ddp=ddp)
        g = torch.Generator().manual_seed(7)
        x = torch.randn(2, 300, 128, generator=g).to(dev)
        y = torch.randn(2, 300, 128, generator=g).to(dev)
        if ddp:
            elapsed, loss = bench.timed_steps(lambda: ts.step(x, y), 2, 1, 1, dev, 0)
            dist.barrier()                                     # the harness's N > 1 collectives, on RCCL
            tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = tt.item()
        else:
            for _ in range(3):
                loss = ts.step(x, y)
        torch.cuda.synchronize()
        res.append([p.detach().float().cpu().numpy().copy() for p in model.parameters()])
    q.put((ok_ar, float(loss), float(elapsed), res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_ddp_rccl_backend_gpu():
    """The N > 1 launch path's collective backend executed on the GPU: DDP over RCCL (world size 1) takes 3 SGD
    steps (1 warm-up + 2 timed by bench.timed_steps) and must land on the same weights as the same 3 steps without
    DDP (the all-reduce of one rank is the identity; every kernel on this path is deterministic)."""
    import numpy as np
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    ok_ar, loss, elapsed, (w_ddp, w_ref) = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert ok_ar and loss == loss and elapsed > 0
    for a, b in zip(w_ddp, w_ref):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)


def test_bench_gpus2_launch_cpu():
    """`python bench.py --gpus 2` outside torchrun starts the two ranks itself (torch.distributed.run child, 127.0.0.1
    rendezvous) and the rank-0 line reports both: the N-rank launch path end to end, on the torch-only rehearsal
    workload over gloo (no GPU here)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LCI_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--workload", "rehearsal",
                        "--steps", "3", "--warmup", "1", "--batch", "2"], capture_output=True, text=True, env=env,
                       timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["dist_backend"] == "gloo"
    assert line["config"]["global_batch"] == 4 and line["config"]["parallelism"] == "ddp2"
    assert line["value"] > 0 and line["steps"] == 3
