"""ctypes binding of librn.so, the C-ABI declared in include/rn.h.

Loading fails loudly (RuntimeError) when the library is missing: there is no CPU or
PyTorch fallback for any op of the training path.
"""
import ctypes as C
import os

from .build import LIB_PATH as _BUILT_LIB, build, library_build_id, needs_build, source_hash

# RN_LIB_PATH: load another build of the library (A/B of two builds in one GPU call); default the in-tree one.
# A library whose build id is not the tree's (rn/build.py: source_hash) is refused unless
# RN_LIB_ALLOW_MISMATCH=1 says the A/B is deliberate; the diagnostic build (librn_diag.so) is checked
# against the tree's diagnostic id.
LIB_PATH = os.environ.get("RN_LIB_PATH") or _BUILT_LIB

RN_BF16 = 0
RN_F32 = 1
RN_POOL_MAX = 0
RN_POOL_AVG = 1

_P = C.c_void_p
_i32 = C.c_int32
_i64 = C.c_int64
_f32 = C.c_float


class ConvDesc(C.Structure):
    _fields_ = [(n, _i32) for n in ("dtype", "n", "h", "w", "c", "c_real", "k", "k_pad", "r", "s", "stride_h",
                                   "stride_w", "pad_h", "pad_w", "groups", "p", "q",
                                   "grouped_direct")]


class BNDesc(C.Structure):
    _fields_ = [("dtype", _i32), ("m", _i64), ("c", _i32), ("c_real", _i32), ("eps", _f32), ("momentum", _f32),
                ("fix_gamma", _i32), ("relu", _i32), ("clip", _P),
                ("clip2", _P), ("dy2", _P), ("xmm", _P), ("xmm_blocks", _i64)]


class WQuantItem(C.Structure):
    _fields_ = [("master", _P), ("qw", _P), ("unit", _P), ("minmax", _P), ("w_codes", _P), ("w_crsk", _P),
                ("k", _i32), ("rs", _i32), ("c_real", _i32), ("c", _i32), ("k_pad", _i32), ("nbits", _i32)]


class PoolDesc(C.Structure):
    _fields_ = [(n, _i32) for n in ("dtype", "n", "h", "w", "c", "r", "s", "stride_h", "stride_w", "pad_h", "pad_w",
                                   "type", "global_pool", "p", "q")]


# name -> (restype, argtypes); every symbol declared in include/rn.h
SIGNATURES = {
    "rn_conv_desc_init": (_i32, [_P]),
    "rn_conv_fwd": (_i32, [_P, _P, _P, _P, _i32, _P, _P, _P]),
    "rn_conv_fwd_bnstats": (_i32, [_P, _P, _P, _P, _i32, _P, _P, _P, _P]),
    "rn_conv_bnstats_blocks": (_i64, [_P]),
    "rn_conv_bn_part_rows": (_i32, [_P, _i32]),
    "rn_conv_tile": (_i32, [_P, _i32]),
    "rn_conv_fwd_i8": (_i32, [_P, _P, _P, _P, _i32, _P, _P, _P, _P, _P]),
    "rn_conv_fwd_i8_mm": (_i32, [_P, _P, _P, _P, _i32, _P, _P, _P, _P, _P, _P, _P]),
    "rn_conv_weight_pack_i8": (_i32, [_P, _P, _P, _P, _P]),
    "rn_conv_fwd_x": (_i32, [_P, _P, _P, _P, _i32, _P, _P, _P, _P, _P, _P]),
    "rn_conv_bwd_filter_x": (_i32, [_P, _P, _P, _P, _P, _P, _P, _i64, _P]),
    "rn_bn_apply_add": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _i32, _P]),
    "rn_bn_reduce_blocks": (_i64, [_P]),
    "rn_relu_bwd_bnred": (_i32, [_P] * 11),
    "rn_conv_bwd_data_bnred": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _i32, _P, _P]),
    "rn_conv_bwd_data_bnred_clip": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _i32, _P, _P, _P]),
    "rn_conv_bwd_data_bnred_clip2": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rn_conv_bnred_blocks": (_i64, [_P]),
    "rn_bn_bwd_part": (_i32, [_P, _P, _i64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rn_bn_bwd_finalize": (_i32, [_P, _P, _i64, _P, _P, _P, _P, _P, _P, _P]),
    "rn_conv_bwd_data_bnapply": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _i32, _P]),
    "rn_conv_bwd_data": (_i32, [_P, _P, _P, _P, _P, _P]),
    "rn_conv_bwd_filter": (_i32, [_P, _P, _P, _P, _P]),
    "rn_conv_wgrad_ws_bytes": (_i64, [_P]),
    "rn_conv_bwd_filter_ws": (_i32, [_P, _P, _P, _P, _P, _i64, _P]),
    "rn_conv_wgrad_i8_supported": (_i32, [_P]),
    "rn_conv_wgrad_i8_ws_bytes": (_i64, [_P]),
    "rn_conv_bwd_filter_i8": (_i32, [_P, _P, _P, _P, _P, _P, _i64, _P]),
    "rn_conv_weight_numel": (_i64, [_P]),
    "rn_conv_pack_numel": (_i64, [_P, _i32]),
    "rn_conv_weight_pack": (_i32, [_P, _P, _P, _P, _P]),
    "rn_conv_weight_pack_multi": (_i32, [_P, _P, _P, _P, _i32, _P]),
    "rn_stem_prepare": (_i32, [_P, _P, _i32, _i32, _i32, _i32, _P, _i32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rn_stem_prepare_p4": (_i32, [_P, _P, _i32, _i32, _i32, _i32, _P, _i32, _i32, _i32, _i32, _i32, _P, _P, _P, _P,
                                  _P, _P, _P, _P, _P, _P]),
    "rn_stem_p4_supported": (_i32, [_P, _i32, _i32]),
    "rn_stem_weight_pack_p4": (_i32, [_P, _P, _P, _P]),
    "rn_stem_conv_fwd_p4": (_i32, [_P, _P, _P, _P, _i32, _i32, _P]),
    "rn_stem_conv_wgrad_p4": (_i32, [_P, _P, _P, _P, _i32, _i32, _P]),
    "rn_im2col_nchw": (_i32, [_P, _P, _P, _P, _P, _i32, _P]),
    "rn_im2col_nchw_quant": (_i32, [_P, _P, _P, _P, _P, _i32, _f32, _i32, _i32, _P, _P, _i32, _P]),
    "rn_stem_quant_clip_grad": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rn_stem_clip_supported": (_i32, [_P]),
    "rn_stem_clip_mask": (_i32, [_P, _P, _P, _P, _P, _P, _P]),
    "rn_stem_clip_wgrad_ws_bytes": (_i64, [_P]),
    "rn_stem_clip_wgrad": (_i32, [_P, _P, _P, _P, _P, _P, _i64, _P]),
    "rn_stem_clip_wgrad_chunk": (_i32, [_P, _P, _P, _P, _P, _P, _i64, _i32, _i32, _P]),
    "rn_stem_clip_dbeta": (_i32, [_P, _P, _P, _P, _P]),
    "rn_stem_shift_grad": (_i32, [_P, _P, _P, _P, _P, _P]),
    "rn_bn_workspace_bytes": (_i64, [_P]),
    "rn_bn_fwd_train": (_i32, [_P] * 13),
    "rn_bn_fwd_train_part": (_i32, [_P, _P, _i64, _i32, _i32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "rn_bn_fwd_infer": (_i32, [_P] * 10),
    "rn_bn_apply": (_i32, [_P] * 6),
    "rn_bn_bwd": (_i32, [_P] * 14),
    "rn_bn_bwd_apply_rows": (_i32, [_P] * 8 + [_i64, _i64, _P]),
    "rn_bn_bwd_global": (_i32, [_P] * 14),
    "rn_pool_desc_init": (_i32, [_P]),
    "rn_pool_fwd": (_i32, [_P, _P, _P, _P, _P]),
    "rn_pool_bwd": (_i32, [_P, _P, _P, _P, _P, _P]),
    "rn_pool_bwd_bnred": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _i32, _P, _P]),
    "rn_pool_bwd_bnred_blocks": (_i64, [_P]),
    "rn_softmax_output": (_i32, [_i32, _i32, _i32, _i32, _P, _P, _P, _P, _f32, _P, _P]),
    "rn_col_sum": (_i32, [_i32, _i64, _i32, _i32, _P, _P, _i32, _P]),
    "rn_sgd_mom_update": (_i32, [_i32, _P, _P, _P, _P, _P, _P, _P, _i32, _f32, _P, _f32, _f32, _f32, _P]),
    "rn_sgd_mom_update_pack": (_i32, [_i32, _P, _P, _P, _P, _P, _P, _P, _P, _i32, _i32, _f32, _P, _f32, _f32, _f32,
                                      _P]),
    "rn_sgd_pack_work": (_i32, [_i32, _P, _P, _P, _i32]),
    "rn_nchw_to_nhwc": (_i32, [_i32, _i32, _i32, _i32, _i32, _P, _P, _i32, _P]),
    "rn_cast": (_i32, [_i64, _P, _i32, _P, _i32, _P]),
    "rn_eltwise_add": (_i32, [_i64, _i32, _P, _P, _P, _i32, _P]),
    "rn_relu_bwd": (_i32, [_i64, _i32, _P, _P, _P, _P, _P]),
    "rn_quant_int8_fwd": (_i32, [_i32, _i64, _P, _P, _P, _i32, _i32, _f32, _i32, _i32, _P, _P]),
    "rn_quant_int8_fwd_codes": (_i32, [_i32, _i64, _P, _P, _P, _P, _P, _i32, _i32, _f32, _i32, _i32, _P, _P]),
    "rn_quant_int8_fwd_codes_bn": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _i32, _f32, _i32, _i32, _P, _P]),
    "rn_quant_int8_fwd_codes_bn2": (_i32, [_P, _P, _P, _P, _P, _P, _P, _P, _f32, _i32, _P, _P, _P, _P, _f32, _i32,
                                           _i32, _i32, _P, _P]),
    "rn_quant_int8_expand": (_i32, [_i32, _i64, _P, _P, _P, _P]),
    "rn_weight_quant_pack": (_i32, [_P, _i32, _i32, _P, _P]),
    "rn_quant_int8_bwd": (_i32, [_i32, _i64, _P, _P, _P, _P, _i32, _P, _P]),
    "rn_set_tuning": (_i32, [_i32, _i32]),
    "rn_last_error": (C.c_char_p, []),
    "rn_version": (_i32, []),
    "rn_build_id": (C.c_char_p, []),
    "rn_device_cu_count": (_i32, []),
    "rn_pool_fwd_x": (_i32, [_P] * 7),
    "rn_stem_conv_fwd_p4_bnstats": (_i32, [_P, _P, _P, _P, _i32, _i32, _P, _P]),
    "rn_stem_bnstats_blocks": (_i64, [_P, _i32, _i32]),
}

# include/rn.h's `#ifdef RN_DIAG` section: exported by the diagnostic build (librn_diag.so) only
DIAG_SIGNATURES = {
    "rn_sgd_mom_update_pack_checked": (_i32, [_i32, _P, _P, _P, _P, _P, _P, _P, _P, _i32, _i32, _f32, _f32, _f32, _P,
                                              _P, _P]),
}

_lib = None


class RNError(RuntimeError):
    pass


def load(auto_build=True):
    """Load librn.so (building it first if sources are newer and hipcc is present)."""
    global _lib
    if _lib is not None:
        return _lib
    if auto_build and LIB_PATH == _BUILT_LIB and os.path.exists("/opt/rocm/bin/hipcc") and needs_build():
        build()
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"librn.so not found at {LIB_PATH}: build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    # PyTorch-ROCm ships its own libamdhip64 (soname libamdhip64.so.7, DT_NEEDED "libamdhip64.so"):
    # load it first so that librn's libamdhip64.so.7 resolves to that same runtime. Loading librn
    # first pulls /opt/rocm's copy, torch then loads a second runtime, and librn's launches see no
    # device ("no ROCm-capable device is detected"). Importing torch does not initialise the GPU.
    import torch  # noqa: F401
    expect = source_hash(diag=os.path.basename(LIB_PATH) == "librn_diag.so")
    got = library_build_id(LIB_PATH)
    if got != expect and os.environ.get("RN_LIB_ALLOW_MISMATCH", "0") != "1":
        raise RuntimeError(f"{LIB_PATH} was built from other sources (build id {got}, tree {expect}): rebuild it "
                           "(`python -c 'import __graft_entry__ as g; g.build()'`), or set RN_LIB_ALLOW_MISMATCH=1 "
                           "for a deliberate A/B of another build")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in list(SIGNATURES.items()) + list(DIAG_SIGNATURES.items()):
        if (name in DIAG_SIGNATURES or LIB_PATH != _BUILT_LIB) and not hasattr(lib, name):
            continue  # (diagnostic-only symbols; an older build loaded for an A/B may lack new entries)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    # RN_DETERMINISTIC=1: bitwise reproducible weight gradients (rn_set_tuning 17)
    if os.environ.get("RN_DETERMINISTIC", "0") == "1":
        check(lib.rn_set_tuning(17, 1), "rn_set_tuning")
        _DETERMINISTIC[0] = True
    # RN_TUNE="key=value,..." selects kernel variants (rn_set_tuning; A/B measurements)
    for kv in filter(None, os.environ.get("RN_TUNE", "").split(",")):
        k, v = kv.split("=")
        check(lib.rn_set_tuning(int(k), int(v)), "rn_set_tuning")
        USER_TUNED.add(int(k))
        if int(k) == 17:
            _DETERMINISTIC[0] = int(v) == 1
    return lib


USER_TUNED = set()  # rn_set_tuning keys fixed by RN_TUNE: the executor leaves them alone
WGRAD_SPLIT_OVERLAPPED = 50  # rn_set_tuning 21 with the weight gradients on the side stream (percent of the chip)
_DETERMINISTIC = [False]  # rn_set_tuning 17 as set through this module (RN_DETERMINISTIC, RN_TUNE, call())


def set_wgrad_split(overlapped, pct=None):
    """rn_set_tuning 21 -- the share of the chip the split-M weight gradients size their grids for -- by how
    the executor runs them: `pct` (default 50 %) beside the data-gradient chain on the side stream
    (measured, DESIGN.md rounds 4-6), the whole chip when they run serialised on the compute stream
    (RN_WGRAD_STREAM=0). An RN_TUNE=21=... override wins. Launches clamp their split to the workspace the
    plan sized. The key is process-global and the split count fixes the fp32 summation order of the weight
    gradients, so outside the deterministic mode a serialised step (bench.py's calibration) does not give
    gradients bit-equal to an overlapped one; in the deterministic mode (rn_set_tuning 17) the key is
    pinned to the whole chip for every executor and step, so the split -- and the bits -- never change."""
    lib = load()
    if 21 not in USER_TUNED:
        v = 100 if (_DETERMINISTIC[0] or not overlapped) else (pct or WGRAD_SPLIT_OVERLAPPED)
        check(lib.rn_set_tuning(21, v), "rn_set_tuning")


def check(ret, what=""):
    if ret != 0:
        msg = _lib.rn_last_error().decode() if _lib is not None else "librn not loaded"
        raise RNError(f"{what}: {msg}")
    return ret


def call(name, *args):
    lib = load()
    ret = check(getattr(lib, name)(*args), name)
    if name == "rn_set_tuning" and int(args[0]) == 17:
        _DETERMINISTIC[0] = int(args[1]) == 1
        if 21 not in USER_TUNED:  # pinned to the whole chip in the mode (set_wgrad_split), else the library default
            check(lib.rn_set_tuning(21, 100 if _DETERMINISTIC[0] else WGRAD_SPLIT_OVERLAPPED), "rn_set_tuning")
    return ret


def ptr(t):
    """Device pointer of a torch tensor (or None)."""
    return None if t is None else C.c_void_p(t.data_ptr())
