"""Build liblci.so (all HIP kernels + C-ABI) in-tree with hipcc for gfx950.

    python -m long_context_biomedical_imaging_amd.build_lib [--jobs N] [--force]

One object per source (parallel), then one shared library. The library links the HIP runtime by
soname (libamdhip64.so.7), so inside a process that already imported torch it binds to the same
runtime torch uses.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "liblci.so")
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


def _obj(src):
    return os.path.join(CSRC, "build", os.path.basename(src) + ".o")


def _stale(src, obj):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src, os.path.abspath(__file__)] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".hpp")]
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, force):
    obj = _obj(src)
    if not force and not _stale(src, obj):
        return obj, None
    cmd = [HIPCC, *FLAGS, *(DEVICE_FLAGS if src.endswith(".hip") else []), *FILE_FLAGS.get(os.path.basename(src), []),
           "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(jobs: int | None = None, force: bool = False, verbose: bool = True) -> str:
    os.makedirs(os.path.join(CSRC, "build"), exist_ok=True)
    srcs = sources()
    jobs = jobs or min(8, os.cpu_count() or 1)
    with cf.ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(lambda s: _compile(s, force), srcs))
    errs = [e for _, e in res if e]
    if errs:
        raise RuntimeError("liblci build failed:\n" + "\n".join(errs))
    objs = [o for o, _ in res]
    if force or not os.path.exists(LIB) or any(os.path.getmtime(o) > os.path.getmtime(LIB) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"liblci link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB} from {len(srcs)} sources", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.force)
