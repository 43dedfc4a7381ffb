"""librn.so loads and exports every entry point declared in include/rn.h (no compute calls)."""
import ctypes as C
import os
import re

import pytest

from rn import lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(REPO, "include", "rn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"#ifdef RN_DIAG.*?#endif", "", src, flags=re.S)  # diagnostic build only
    return sorted(set(re.findall(r"\b(rn_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    names = declared()
    assert len(names) >= 25
    assert set(names) == set(L.SIGNATURES), set(names) ^ set(L.SIGNATURES)


def test_library_exports_everything():
    lib = L.load()
    for n in declared():
        assert hasattr(lib, n), n
    assert lib.rn_version() >= 100


def test_host_side_validation_and_errors():
    lib = L.load()
    d = L.ConvDesc(dtype=L.RN_BF16, n=2, h=56, w=56, c=64, c_real=64, k=64, k_pad=64, r=3, s=3, stride_h=1,
                   stride_w=1, pad_h=1, pad_w=1, groups=1)
    assert lib.rn_conv_desc_init(C.byref(d)) == 0 and (d.p, d.q) == (56, 56)
    d.c = 3
    assert lib.rn_conv_desc_init(C.byref(d)) == -1
    assert b"multiple of 8" in lib.rn_last_error()
    b = L.BNDesc(dtype=L.RN_BF16, m=1000, c=64, c_real=64, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    assert lib.rn_bn_workspace_bytes(C.byref(b)) > 64 * 4
    pd = L.PoolDesc(dtype=L.RN_BF16, n=2, h=112, w=112, c=64, r=3, s=3, stride_h=2, stride_w=2, pad_h=1, pad_w=1,
                    type=L.RN_POOL_MAX, global_pool=0)
    assert lib.rn_pool_desc_init(C.byref(pd)) == 0 and (pd.p, pd.q) == (56, 56)


def test_sgd_pack_work_table():
    """Host-side work table of rn_sgd_mom_update_pack: 4096-element chunks for tensors without a
    CRSK copy, 64 x 64 (k, c) tiles per tap for the others; every element covered exactly once."""
    import numpy as np
    lib = L.load()
    dt = np.dtype([("krsc", "<u8"), ("crsk", "<u8"), ("k", "<i4"), ("rs", "<i4"), ("creal", "<i4"),
                   ("c", "<i4"), ("kpad", "<i4"), ("pad", "<i4")])
    assert dt.itemsize == 40
    tab = np.zeros(3, dtype=dt)
    tab[1] = (1, 1, 100, 9, 70, 72, 104, 0)   # conv 3x3, ragged k and c
    tab[2] = (1, 0, 16, 49, 3, 8, 16, 0)      # stem: KRSC copy only -> chunks
    nums = np.array([5000, 100 * 9 * 70, 16 * 49 * 3], dtype=np.int64)
    work = np.zeros((64, 4), dtype=np.int32)
    P = lambda a: a.ctypes.data_as(C.c_void_p)
    n = lib.rn_sgd_pack_work(3, P(nums), P(tab), P(work), 64)
    assert n == 2 + 2 * 9 * 2 + 1, n
    w = work[:n]
    assert [tuple(r) for r in w[:2]] == [(0, 0, 0, 0), (0, 4096, 0, 0)]
    cover = np.zeros((100, 9, 70), dtype=np.int32)
    for t, k0, tap, c0 in w[w[:, 0] == 1]:
        cover[k0:k0 + 64, tap, c0:c0 + 64] += 1
    assert (cover == 1).all()
    assert lib.rn_sgd_pack_work(3, P(nums), P(tab), P(work), 4) == -1
    tab[1]["k"] = 99  # size mismatch is refused
    assert lib.rn_sgd_pack_work(3, P(nums), P(tab), P(work), 64) == -1


def test_diagnostic_modes_are_not_in_the_product_library():
    """the wrong-result diagnostics (rn_set_tuning 3 / 6 / 7, the checked SGD
    twin) exist only in the RN_DIAG build; librn.so refuses the keys and does not export the twin."""
    lib = L.load()
    assert not hasattr(lib, "rn_sgd_mom_update_pack_checked")
    for key in (3, 6, 7):
        assert lib.rn_set_tuning(key, 1) == -1
        assert b"diagnostic" in lib.rn_last_error()
        assert lib.rn_set_tuning(key, 0) == 0
    assert lib.rn_set_tuning(12, 0) == 0  # ordinary variant keys stay available


def test_grouped_layout_is_fixed_at_descriptor_init():
    """the grouped direct / block-diagonal choice (rn_set_tuning 15) is recorded in the
    descriptor by rn_conv_desc_init, so a later change of the key cannot make a launch read a copy
    packed in the other layout: the pack size of an initialised descriptor never changes."""
    lib = L.load()

    def desc():
        d = L.ConvDesc(dtype=L.RN_BF16, n=2, h=14, w=14, c=128, c_real=128, k=128, k_pad=128, r=3, s=3,
                       stride_h=1, stride_w=1, pad_h=1, pad_w=1, groups=32)
        assert lib.rn_conv_desc_init(C.byref(d)) == 0
        return d
    d = desc()
    assert d.grouped_direct == 1
    compact = lib.rn_conv_pack_numel(C.byref(d), 0)
    assert compact == 128 * 9 * 4
    try:
        assert lib.rn_set_tuning(15, 1) == 0
        assert lib.rn_conv_pack_numel(C.byref(d), 0) == compact  # the same descriptor keeps its layout
        d2 = desc()
        assert d2.grouped_direct == 0 and lib.rn_conv_pack_numel(C.byref(d2), 0) > compact
    finally:
        lib.rn_set_tuning(15, 0)
    d.groups = 1  # a dense conv is never direct
    assert lib.rn_conv_desc_init(C.byref(d)) == 0 and d.grouped_direct == 0


def test_loaded_library_is_tied_to_the_tree(tmp_path, monkeypatch):
    """the library carries a build id (a hash of csrc/*, include/rn.h and the flags,
    exported as rn_build_id); rn.lib.load() refuses one whose id differs from the tree's, so a stale
    prebuilt after a checkout or copy fails loudly. A touched source makes load(auto_build=False) fail."""
    from rn import build as B
    lib = L.load()
    assert lib.rn_build_id().decode() == B.source_hash() == B.library_build_id(L.LIB_PATH)
    assert not B.needs_build()
    # a touched source: one more dependency with new bytes changes the tree's id
    extra = tmp_path / "touched.h"
    extra.write_text("// edited\n")
    deps = B._deps
    monkeypatch.setattr(B, "_deps", lambda: deps() + [str(extra)])
    assert B.source_hash() != B.library_build_id(L.LIB_PATH) and B.needs_build()
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.delenv("RN_LIB_ALLOW_MISMATCH", raising=False)
    with pytest.raises(RuntimeError, match="built from other sources"):
        L.load(auto_build=False)
    # an explicit A/B override loads it anyway
    monkeypatch.setenv("RN_LIB_ALLOW_MISMATCH", "1")
    assert L.load(auto_build=False) is not None
