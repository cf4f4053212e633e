#!/usr/bin/env python3
"""Build a liblci variant for a same-box A/B (tools/lib_ab.sh): the current objects with some sources swapped for
another revision's (or compiled with extra flags), linked into build_variants/liblci_<name>.so.

    python tools/build_variant.py old --rev HEAD conv.hip          # conv.hip as committed, the rest as in the tree
    python tools/build_variant.py p1 --define LCI_CONV_PROBE=1 conv.hip
    python tools/build_variant.py new                              # the tree's library as is

The variant keeps the tree's ABI version (lci_abi_version) so _lib.load() accepts it under LCI_LIB_PATH; it is never
the library the tests or bench.py load by default. With --rev, the revision's include/lci.h must declare the same
LCI_ABI_VERSION as the tree's: objects built from sources of another ABI (other argument lists behind the same
symbols) are refused instead of being linked under the tree's version stamp.
"""
import argparse
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from long_context_biomedical_imaging_amd import build_lib as b  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("sources", nargs="*", help="csrc file names to rebuild for the variant")
    ap.add_argument("--rev", default=None, help="git revision to take those sources from (default: the tree)")
    ap.add_argument("--define", action="append", default=[], help="extra -D for those sources")
    a = ap.parse_intermixed_args()
    if a.rev and a.sources:
        def abi(text):
            m = re.search(r"^#define LCI_ABI_VERSION (\d+)", text, re.M)
            return int(m.group(1)) if m else None
        rev_h = subprocess.run(["git", "-C", ROOT, "show", f"{a.rev}:include/lci.h"], check=True,
                               capture_output=True, text=True).stdout
        with open(b.HEADER) as fh:
            tree = abi(fh.read())
        if abi(rev_h) != tree:
            sys.exit(f"build_variant: {a.rev} declares LCI_ABI_VERSION {abi(rev_h)}, the tree {tree}: refusing to link "
                     "its objects under the tree's ABI stamp")
    b.build(verbose=False)
    out_dir = os.path.join(ROOT, "build_variants")
    os.makedirs(out_dir, exist_ok=True)
    out = os.path.join(out_dir, f"liblci_{a.name}.so")
    if not a.sources:
        shutil.copy(b.LIB, out)
        print(out)
        return
    objs = [b._obj(s) for s in b.sources()]
    tmp = tempfile.mkdtemp()
    for f in a.sources:
        src = os.path.join(b.CSRC, f)
        if a.rev:
            text = subprocess.run(["git", "-C", ROOT, "show", f"{a.rev}:long_context_biomedical_imaging_amd/csrc/{f}"],
                                  check=True, capture_output=True).stdout
            src = os.path.join(tmp, f)
            with open(src, "wb") as fh:
                fh.write(text)
        obj = os.path.join(tmp, f + ".o")
        subprocess.run([b.HIPCC, *b.FLAGS, *b.DEVICE_FLAGS, *b.FILE_FLAGS.get(f, []), "-I", b.CSRC,
                        *[f"-D{d}" for d in a.define], "-c", src, "-o", obj], check=True, capture_output=True)
        objs = [obj if o == b._obj(os.path.join(b.CSRC, f)) else o for o in objs]
    subprocess.run([b.HIPCC, "-shared", "-fPIC", f"--offload-arch={b.ARCH}", *objs, "-o", out], check=True)
    shutil.rmtree(tmp)
    print(out)


if __name__ == "__main__":
    main()
