"""Helpers for GPU parity tests: NCHW numpy <-> NHWC device tensors, direct C-ABI calls."""
import ctypes as C

import numpy as np
import torch

from rn import lib as L

BF16, F32 = L.RN_BF16, L.RN_F32


def tdt(dtype):
    return torch.bfloat16 if dtype == BF16 else torch.float32


def bf16_round(a):
    """Round an fp64/fp32 array to bf16 and back (RNE), as the device copy sees it."""
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16).to(torch.float32)
    return t.numpy().astype(np.float64)


def pad8(c):
    return (c + 7) // 8 * 8


def to_nhwc(x, dtype, dev, cpad=None):
    n, c, h, w = x.shape
    cpad = cpad or pad8(c)
    t = torch.zeros((n, h, w, cpad), dtype=torch.float32)
    t[..., :c] = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 2, 3, 1), dtype=np.float32))
    return t.to(tdt(dtype)).to(dev).contiguous()


def from_nhwc(t, c):
    a = t.float().cpu().numpy()
    return a[..., :c].transpose(0, 3, 1, 2).astype(np.float64)


def stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def conv_desc(dtype, n, c, h, w, k, r, s, stride, pad, c_real=None, groups=1):
    d = L.ConvDesc(dtype=dtype, n=n, h=h, w=w, c=pad8(c) if c_real is None else c, c_real=c if c_real is None else c_real,
                   k=k, k_pad=pad8(k), r=r, s=s, stride_h=stride, stride_w=stride, pad_h=pad, pad_w=pad, groups=groups)
    L.call("rn_conv_desc_init", C.byref(d))
    return d


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))
