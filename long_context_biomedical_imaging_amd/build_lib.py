"""Build liblci.so (all HIP kernels + C-ABI) in-tree with hipcc for gfx950.

    python -m long_context_biomedical_imaging_amd.build_lib [--jobs N] [--force]

One object per source (parallel, rebuilt when its content key changes), then one shared library that carries
the sources' hash (lci_build_hash). The library links the HIP runtime by
soname (libamdhip64.so.7), so inside a process that already imported torch it binds to the same
runtime torch uses.
"""
from __future__ import annotations

import argparse
import hashlib
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "liblci.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HEADER = os.path.join(INCLUDE, "lci.h")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
         "-munsafe-fp-atomics"]
# Device code: MFMA accumulators in ordinary VGPRs (gfx950's unified register file) instead of AGPRs, which
# otherwise cost v_accvgpr_read/write copies around every softmax rescale and lower occupancy.
DEVICE_FLAGS = ["-Xarch_device", "-mllvm=-amdgpu-mfma-vgpr-form"]
# Softmax kernels: no NaN-quieting canonicalisation (v_max x,x) in front of every fmaxf on MFMA results;
# attention: no SLP packing of f32 multiplies into v_pk_mul_f32 (needs aligned pairs -> moves + alignbit).
FILE_FLAGS = {"attention.hip": ["-fno-honor-nans", "-fno-slp-vectorize"], "window.hip": ["-fno-honor-nans"]}


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _read(path):
    with open(path, "rb") as f:
        return f.read()


def source_hash() -> str:
    """sha256 over every kernel/ABI source, the shared headers, the public header and the build flags.

    Staleness is keyed on content, not mtimes (a copied tree keeps no meaningful mtimes). The hash is compiled
    into the library (lci_build_hash()) and _lib.load() refuses a liblci.so whose hash differs from the sources
    next to it, so a stale binary can never be used silently (on the GPU box the driver runs without building).
    """
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".hpp")))
    for f in files:
        h.update(f.encode() + b"\0" + _read(os.path.join(CSRC, f)) + b"\0")
    h.update(_read(HEADER))
    h.update(repr((FLAGS, DEVICE_FLAGS, sorted(FILE_FLAGS.items()))).encode())
    return h.hexdigest()[:32]


def _obj(src):
    return os.path.join(CSRC, "build", os.path.basename(src) + ".o")


def _obj_key(src, full_hash):
    """Per-object content key: the source, the shared headers and the flags (abi.cpp also embeds the full hash)."""
    h = hashlib.sha256(_read(src))
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hpp"):
            h.update(_read(os.path.join(CSRC, f)))
    h.update(repr((FLAGS, DEVICE_FLAGS, FILE_FLAGS.get(os.path.basename(src)))).encode())
    if os.path.basename(src) == "abi.cpp":
        h.update(full_hash.encode())
    return h.hexdigest()


def _stale(obj, key):
    stamp = obj + ".key"
    return not (os.path.exists(obj) and os.path.exists(stamp) and _read(stamp).decode() == key)


def _compile(src, force, full_hash):
    obj = _obj(src)
    key = _obj_key(src, full_hash)
    if not force and not _stale(obj, key):
        return obj, None, False
    cmd = [HIPCC, *FLAGS, *(DEVICE_FLAGS if src.endswith(".hip") else []), *FILE_FLAGS.get(os.path.basename(src), []),
           "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", f'-DLCI_BUILD_HASH="{full_hash}"', "-I", INCLUDE,
               "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}", True
    with open(obj + ".key", "w") as f:
        f.write(key)
    return obj, None, True


def build(jobs: int | None = None, force: bool = False, verbose: bool = True) -> str:
    os.makedirs(os.path.join(CSRC, "build"), exist_ok=True)
    srcs = sources()
    full_hash = source_hash()
    jobs = jobs or min(8, os.cpu_count() or 1)
    with cf.ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(lambda s: _compile(s, force, full_hash), srcs))
    errs = [e for _, e, _ in res if e]
    if errs:
        raise RuntimeError("liblci build failed:\n" + "\n".join(errs))
    objs = [o for o, _, _ in res]
    stamp = LIB + ".key"
    if force or any(rebuilt for _, _, rebuilt in res) or not os.path.exists(LIB) or not os.path.exists(stamp) \
            or _read(stamp).decode() != full_hash:
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"liblci link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        with open(stamp, "w") as f:
            f.write(full_hash)
    if verbose:
        print(f"built {LIB} from {len(srcs)} sources (hash {full_hash})", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.force)
