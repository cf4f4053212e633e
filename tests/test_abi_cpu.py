"""The C-ABI library loads on CPU-only hosts and exports every symbol include/lci.h declares; the Python
binding's argument lists match the header's (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "lci.h")


def _declared():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    decls = re.findall(r"^\s*(?:const\s+)?(?:char\*|int|long long)\s+(lci_\w+)\(([^;]*)\);", txt, flags=re.M)
    return {name: [a.strip() for a in args.replace("\n", " ").split(",") if a.strip() and a.strip() != "void"]
            for name, args in decls}


def _header_abi_version() -> int:
    m = re.search(r"#define\s+LCI_ABI_VERSION\s+(\d+)", open(HDR).read())
    assert m, "include/lci.h defines no LCI_ABI_VERSION"
    return int(m.group(1))


def test_abi_version_constants_agree():
    """include/lci.h, the Python binding and every `lci_abi_version() == N` literal in INTEGRATION.md agree."""
    from long_context_biomedical_imaging_amd import _lib
    v = _header_abi_version()
    assert _lib.ABI_VERSION == v
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    lits = re.findall(r"lci_abi_version\(\)\s*==\s*(\d+)", txt)
    assert lits, "INTEGRATION.md stub checks no ABI version"
    for n in lits:
        assert int(n) == v, f"INTEGRATION.md asserts ABI {n}, include/lci.h defines {v}"


def test_header_declares_entry_points():
    d = _declared()
    for must in ("lci_attn_fwd", "lci_attn_bwd", "lci_window_attn_fwd", "lci_window_attn_bwd",
                 "lci_selective_scan_fwd", "lci_selective_scan_bwd", "lci_fftconv_fwd", "lci_fftconv_bwd",
                 "lci_patch_embed_fwd", "lci_patch_embed_bwd", "lci_hyena_pre_fwd", "lci_dwconv_silu_fwd",
                 "lci_layernorm_fwd", "lci_layernorm_bwd", "lci_conv3_fwd", "lci_inorm_apply"):
        assert must in d, must


def test_library_exports_every_declared_symbol():
    from long_context_biomedical_imaging_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("liblci.so not built (python -m long_context_biomedical_imaging_amd.build_lib)")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), f"{name} declared in include/lci.h but not exported"
    assert _lib.load().lci_abi_version() == _lib.ABI_VERSION == _header_abi_version()


def test_python_binding_arity_matches_header():
    from long_context_biomedical_imaging_amd import _lib
    d = _declared()
    for name, argt in _lib.SIGNATURES.items():
        assert name in d, f"{name} bound in Python but not declared"
        assert len(argt) == len(d[name]), f"{name}: python {len(argt)} args, header {len(d[name])}"


def test_integration_doc_stubs_match_header():
    """Every `lib.<name>.argtypes = [...]` in INTEGRATION.md declares the header's argument count."""
    d = _declared()
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    stubs = re.findall(r"lib\.(lci_\w+)\.argtypes\s*=\s*\[([^\]]*)\]", txt)
    assert stubs, "INTEGRATION.md has no ctypes stub"
    for name, args in stubs:
        assert name in d, f"INTEGRATION.md binds {name}, not declared in include/lci.h"
        n = len([a for a in args.split(",") if a.strip()])
        assert n == len(d[name]), f"INTEGRATION.md {name}: {n} args, header {len(d[name])}"
