"""librn.so loads and exports every entry point declared in include/rn.h (no compute calls)."""
import ctypes as C
import os
import re

from rn import lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(REPO, "include", "rn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
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
