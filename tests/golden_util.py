"""Helpers to read tests/golden/*.npz (written by tools/gen_golden.py from the reference)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Golden:
    def __init__(self, name):
        self.name = name
        self.z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)

    def t(self, key, dtype=torch.float32):
        a = self.z[key]
        t = torch.from_numpy(np.array(a))
        return t.to(dtype) if t.is_floating_point() else t

    def has(self, key):
        return key in self.z.files

    def sd(self):
        return {k[3:]: self.t(k) if self.z[k].dtype.kind == "f" else torch.from_numpy(np.array(self.z[k]))
                for k in self.z.files if k.startswith("sd/")}

    def outs(self):
        n = len([k for k in self.z.files if k.startswith("out/") and k[4:].isdigit()])
        return [self.t(f"out/{i}") for i in range(n)]

    def scalar(self, key):
        return self.z[key].item()


def cotangents(outs, seed=123):
    """Same cotangents as tools/gen_golden.py:fwd_bwd (seeded N(0,1), one per output, in order)."""
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(o.shape, generator=g) for o in outs]


def assert_close(a, b, rtol, atol, what=""):
    a = a.detach().float().cpu()
    b = b.detach().float().cpu()
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol)
    if bad.any():
        i = int(torch.argmax((err - tol).flatten()))
        raise AssertionError(f"{what}: {int(bad.sum())}/{a.numel()} elements out of tolerance; worst "
                             f"err={err.flatten()[i].item():.3e} at {i}, ref={b.flatten()[i].item():.4e}, "
                             f"max|err|={err.max().item():.3e}, max|ref|={b.abs().max().item():.3e}")


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
