"""ORACLE / TEST INFRASTRUCTURE ONLY: ctypes binding of oracle/scan_ref.c (fp64 selective scan, fwd + bwd).

The C restatement follows mamba-ssm 1.2.0.post1 `selective_scan_ref` semantics as called at
model/models/mamba.py:125-134 (see the header of scan_ref.c); it exists so the GPU scan can be checked at the
C5 sequence length (L = 2^21) where the Python restatement (oracle/selective_scan.py) would take minutes. It is
cross-checked against that restatement in tests/test_oracle_golden.py. Only tests/ may import this module.

    build()                        gcc -O2 -fopenmp -> oracle/_build/libscan_ref.so (no -ffast-math: exact libm)
    scan_fwd(u, delta, A, B, C, D, delta_bias) -> y                        (channels-last, one batch element)
    scan_bwd(u, delta, A, B, C, D, delta_bias, dy) -> du, ddelta, dA, dD, ddelta_bias, dB, dC
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "scan_ref.c")
LIB = os.path.join(HERE, "_build", "libscan_ref.so")
_lib = None


_CMD = ["gcc", "-O2", "-fopenmp", "-fPIC", "-shared", SRC, "-o", LIB, "-lm"]


def _key() -> str:
    """Staleness key: sha256 of scan_ref.c + the compile line (copied trees have unreliable mtimes)."""
    h = hashlib.sha256(open(SRC, "rb").read())
    h.update(" ".join(_CMD).encode())
    return h.hexdigest()


def build(force: bool = False) -> str:
    key_path = LIB + ".key"
    key = _key()
    stale = not os.path.exists(LIB) or not os.path.exists(key_path) or open(key_path).read().strip() != key
    if force or stale:
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(_CMD, check=True)
        with open(key_path, "w") as f:
            f.write(key)
    return LIB


def _load():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.scan_ref_fwd.restype = ctypes.c_int
        _lib.scan_ref_bwd.restype = ctypes.c_int
    return _lib


def _f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _threads():
    omp = os.environ.get("OMP_NUM_THREADS", "")
    n = len(os.sched_getaffinity(0))
    return max(1, min(n, int(omp))) if omp.isdigit() and int(omp) > 0 else n


def scan_fwd(u, delta, A, Bm, Cm, D, dbias):
    """u, delta (L, Dx); Bm, Cm (L, N); A (Dx, N); D, dbias (Dx). Returns y (L, Dx) f64."""
    u, delta, Bm, Cm = _f32(u), _f32(delta), _f32(Bm), _f32(Cm)
    A, D, dbias = _f64(A), _f64(D), _f64(dbias)
    L, Dx = u.shape
    N = A.shape[1]
    y = np.empty((L, Dx), dtype=np.float64)
    rc = _load().scan_ref_fwd(_p(u), _p(delta), _p(Bm), _p(Cm), _p(A), _p(D), _p(dbias), ctypes.c_longlong(L),
                              Dx, N, ctypes.c_longlong(Dx), ctypes.c_longlong(N), _p(y))
    assert rc == 0, rc
    return y


def scan_bwd(u, delta, A, Bm, Cm, D, dbias, dy):
    u, delta, Bm, Cm, dy = _f32(u), _f32(delta), _f32(Bm), _f32(Cm), _f32(dy)
    A, D, dbias = _f64(A), _f64(D), _f64(dbias)
    L, Dx = u.shape
    N = A.shape[1]
    du = np.empty((L, Dx))
    dd = np.empty((L, Dx))
    dA = np.empty((Dx, N))
    dD = np.empty(Dx)
    db = np.empty(Dx)
    dB = np.empty((L, N))
    dC = np.empty((L, N))
    rc = _load().scan_ref_bwd(_p(u), _p(delta), _p(Bm), _p(Cm), _p(A), _p(D), _p(dbias), _p(dy),
                              ctypes.c_longlong(L), Dx, N, ctypes.c_longlong(Dx), ctypes.c_longlong(N), _p(du),
                              _p(dd), _p(dA), _p(dD), _p(db), _p(dB), _p(dC), _threads())
    assert rc == 0, rc
    return du, dd, dA, dD, db, dB, dC
