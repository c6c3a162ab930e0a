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


def test_trunk_stamp_decoding():
    """bench.py's in-situ trunk duration: per launch row, last workgroup end minus first start
    (100 MHz ticks -> ms), evaluated boards from bits 56-63 of the end stamps; rows beyond the
    counter are ignored, a wrapped ring keeps every row."""
    import torch
    from rvz.measure import trunk_spans
    ring, grid = 4, 3
    st = torch.zeros(ring, grid, 2, dtype=torch.int64)
    # launch 0: starts 1000..1002, ends 31000..31002 -> span 30002 ticks; boards 2 + 2 + 1
    # launch 1: starts 5000, ends 15000 -> span 10000 ticks; boards 2 + 0 + 0
    for w in range(grid):
        st[0, w, 0] = 1000 + w
        st[0, w, 1] = (31000 + w) | ((2 if w < 2 else 1) << 56)
        st[1, w, 0] = 5000
        st[1, w, 1] = 15000 | ((2 if w == 0 else 0) << 56)
    st[2:] = 999999                      # rows past the counter: ignored
    r = trunk_spans(st, 2)
    assert r["launches"] == 2
    assert abs(r["ms"] - (30002 + 10000) / 2 / 1e5) < 1e-12
    assert r["rows"] == (5 + 2) / 2
    assert trunk_spans(st, 0) is None
    full = trunk_spans(st[:2], 7)         # wrapped: both rows kept
    assert full["launches"] == 7 and full["rows"] == 3.5


def test_alt_library_matches_its_header():
    """tools/alt/librvz_alt.so (the A/B and cross-check build) exports exactly what
    tools/alt/rvz_alt.h declares, its ctypes table covers the header, and the product library
    exports none of it (the alternatives are not on the product surface)."""
    import alt_eval
    hdr = open(os.path.join(ROOT, "tools", "alt", "rvz_alt.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    decl = set(re.findall(r"\b(rvz_[a-z0-9_]+)\s*\(", hdr))
    assert set(alt_eval.SIGNATURES) == decl
    out = subprocess.run(["nm", "-D", "--defined-only", alt_eval.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rvz_[a-z0-9_]+)", out))
    assert exported == decl, exported ^ decl
    alt_eval.load()
    assert not decl & set(declared_symbols())


def test_evaluator_entry_points_reject_a_misaligned_workspace():
    """the trunk's 64-bit unit-counter atomic and the heads' f32x4 row copies need a
    16-byte aligned workspace; a misaligned one is RVZ_EINVAL at the C-ABI (argument checks run
    before any HIP call, so this needs no GPU), never a device fault."""
    import rvz
    lib = rvz.load()
    EINVAL = -22
    params, blob, x, out = 0x10000, 0x20000, 0x30000, 0x40000   # never dereferenced
    for work in (0x50004, 0x50008):
        assert lib.rvz_resnet_trunk_h2(8, x, 64, params, blob, 64, 6, work, None) == EINVAL
        assert lib.rvz_resnet_heads_fc(8, work, 64, params, 64, 6, out, out, None) == EINVAL
        assert lib.rvz_resnet_fwd_h2(8, x, 64, params, blob, 64, 6, work, out, out,
                                     None) == EINVAL


def test_evaluator_width_rules_without_gpu():
    """The h2 widths at the C-ABI (argument checks only, no HIP call): 64 and 128 filters on both
    boards, 256 on 8x8; anything else is RVZ_EINVAL. rvz_resnet_h2_grid: one workgroup per board
    at 128 / 256 on 8x8 (two boards per unit at 64), plus 1/8 spare workgroups rounded to 8."""
    import rvz
    lib = rvz.load()
    EINVAL = -22
    assert lib.rvz_resnet_h2_grid(8, 256, 10) == 18 and lib.rvz_resnet_h2_grid(8, 128, 10) == 18
    assert lib.rvz_resnet_h2_grid(8, 64, 10) == 13
    for board, f in ((6, 256), (8, 192), (8, 32), (8, 512), (7, 64)):
        assert lib.rvz_resnet_h2_grid(board, f, 10) == EINVAL, (board, f)
    for f in (64, 128, 256):
        assert lib.rvz_resnet_h2_size(f, 3) > 0 and lib.rvz_resnet_params_size(8, f, 3) > 0
    assert lib.rvz_resnet_h2_size(192, 3) == EINVAL
    # a 6x6 trunk at 256 filters is refused before anything is launched
    p = 0x10000
    assert lib.rvz_resnet_trunk_h2(6, p, 4, p, p, 256, 1, p, None) == EINVAL
