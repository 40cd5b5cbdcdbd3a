"""The C-ABI library loads and exports every symbol include/gaplac.h declares.
No compute calls here (this runs without a GPU)."""
import ctypes
import os
import re

from gaplac_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "gaplac.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gaplac_[a-z_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_native.EXPORTED) == syms


def test_abi_version_and_struct_layout():
    lib = _native.load()
    assert lib.gaplac_abi_version() == 1
    assert ctypes.sizeof(_native.Term) == 24
    assert _native.Term.param.offset == 8 and _native.Term.group.offset == 16


def test_ctx_create_reports_missing_device_without_crashing():
    try:
        import torch
        if torch.cuda.is_available():
            return
    except Exception:
        pass
    lib = _native.load()
    h = ctypes.c_void_p()
    assert lib.gaplac_ctx_create(0, ctypes.byref(h)) == _native.E_NODEVICE
    assert not h.value
    assert lib.gaplac_ctx_destroy(None) == 0
