"""CPU-side checks of the product library and host logic (no kernel launches):
librvz.so loads and exports every symbol include/rvz.h declares, the ctypes signature table
covers the header, and the host mirror refuses to run without a HIP device (no CPU fallback)."""
import os
import re
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rvz.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rvz_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import rvz
    lib = rvz.load()
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", rvz._lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rvz_[a-z0-9_]+)", out))
    assert set(syms) <= exported
    assert exported <= set(syms), exported - set(syms)   # nothing undeclared leaks


def test_ctypes_table_matches_header():
    import rvz
    assert set(rvz._lib.SIGNATURES) == set(declared_symbols())


def test_library_is_gfx950_code_object():
    import rvz
    blob = open(rvz._lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob      # the embedded offload bundle's target


def test_version_without_gpu():
    import rvz
    assert rvz.load().rvz_version() == 1


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_engine_fails_loudly_without_gpu():
    import rvz
    with pytest.raises(rvz.RvzError):
        rvz.Engine(4)
    with pytest.raises(RuntimeError):
        rvz.ReversiGame().get_valid_moves()
