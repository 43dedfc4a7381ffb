"""Int8 MFMA forward of quantized convolutions (rn_conv_fwd_i8, v_mfma_i32_16x16x64_i8) and the int8
codes of Quantization_int8 (rn_quant_int8_fwd_codes[_bn], rn_conv_weight_pack_i8).

The reference computes a quantized conv in fp32 on fake-quantized values (symbol/int8_api.py:120-151,
values code * unit, symbol/quant_ops.py:17-31, clip_grad_quantization_int8.py:37-54). On the integer
grid the sum of code products is exact; the kernel keeps it exact in int32 and applies unit_x * unit_w
once. Bars: the integer sums exactly (fp32 output with unit 1, |sum| < 2^24); with real units, fp32
output within 2 ulp-scale (4e-7 relative) of the fp64 value, bf16 output within bf16 rounding (2^-8);
codes and units bit-identical to the fake-quant values the same call writes (value == code * unit).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import ops
from rn import lib as L
from gpu_util import BF16, F32, conv_desc, from_nhwc, p, rel_err, stream, tdt, to_nhwc

pytestmark = pytest.mark.gpu

CASES = [
    # n, c, h, w, k, r, stride, pad  (c a multiple of 16)
    (2, 64, 14, 14, 64, 1, 1, 0),      # 64-column tile
    (2, 64, 14, 14, 256, 1, 1, 0),     # 224 x 128 / 256 tiles
    (2, 128, 14, 14, 128, 3, 1, 1),    # 3x3: 9 taps x one 128-deep K-tile
    (3, 256, 9, 7, 512, 3, 2, 1),      # strided 3x3, ragged M
    (2, 32, 8, 8, 24, 1, 1, 0),        # ragged K (24 columns), partial K-tile
    (1, 512, 7, 7, 2048, 1, 1, 0),     # stage-4 conv3 shape
    (2, 64, 56, 56, 256, 1, 1, 0),     # many tiles: persistent walk
]


def _codes(rng, shape, qmax=127):
    return rng.integers(-qmax, qmax + 1, size=shape)


def _run(gpu, case, y_dtype, ux, uw, res=None, part=None):
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(sum(case))
    xc = _codes(rng, (n, c, h, w))
    wc = _codes(rng, (k, c, r, r))
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    assert d.c % 16 == 0
    xd = torch.from_numpy(np.ascontiguousarray(xc.transpose(0, 2, 3, 1)).astype(np.int8)).to(gpu)
    wd = torch.from_numpy(np.ascontiguousarray(wc.transpose(0, 2, 3, 1)).astype(np.int8)).reshape(-1).to(gpu)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    y = torch.zeros((n, P, Q, d.k_pad), dtype=tdt(y_dtype), device=gpu)
    uxd = torch.tensor([ux], dtype=torch.float32, device=gpu)
    uwd = torch.tensor([uw], dtype=torch.float32, device=gpu)
    rd = to_nhwc(res, y_dtype, gpu) if res is not None else None
    L.call("rn_conv_fwd_i8", C.byref(d), p(xd), p(wd), p(y), y_dtype, p(rd), p(uxd), p(uwd), p(part), stream())
    torch.cuda.synchronize()
    exact = ops.conv2d_fwd(xc.astype(np.float64), wc.astype(np.float64), (st, st), (pd, pd))  # exact integers
    return d, from_nhwc(y, k), exact


@pytest.mark.parametrize("case", CASES)
def test_int8_conv_exact_integer_sums(gpu, case):
    _, y, exact = _run(gpu, case, F32, 1.0, 1.0)
    assert np.abs(exact).max() < 2 ** 24
    np.testing.assert_array_equal(y, exact)


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("y_dtype", [F32, BF16])
@pytest.mark.parametrize("persist", [512, 8], ids=["persist512", "persist8"])
def test_int8_conv_scaled_residual(gpu, case, y_dtype, persist):
    n, c, h, w, k, r, st, pd = case
    L.call("rn_set_tuning", 10, persist)
    try:
        P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
        res = np.random.default_rng(3).standard_normal((n, k, P, Q))
        if y_dtype == BF16:
            res = from_nhwc(to_nhwc(res, BF16, "cpu"), k)
        ux, uw = 0.0123, 0.00071
        _, y, exact = _run(gpu, case, y_dtype, ux, uw, res=res)
    finally:
        L.call("rn_set_tuning", 10, 512)
    ref = exact * (np.float64(np.float32(ux)) * np.float64(np.float32(uw))) + res
    assert rel_err(y, ref) < (4e-7 if y_dtype == F32 else 2 ** -8), rel_err(y, ref)


@pytest.mark.parametrize("case", [CASES[1], CASES[2], CASES[0]])
@pytest.mark.parametrize("y_dtype", [F32, BF16])
def test_int8_conv_bnstats_epilogue(gpu, case, y_dtype):
    """BatchNorm statistics partials of the int8 conv's stored output (rn_conv_bn_part_rows(d, 2))
    merged by rn_bn_fwd_train_part == the batch mean / variance of that output."""
    n, c, h, w, k, r, st, pd = case
    lib = L.load()
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    rows = lib.rn_conv_bn_part_rows(C.byref(d), 2)
    assert rows in (64, 224)  # per 64-row wave row (64-column tile) or per 224-row tile
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    nblk = -(-(n * P * Q) // rows)
    part = torch.zeros(nblk * 3 * d.k_pad, dtype=torch.float32, device=gpu)
    _, y, _ = _run(gpu, case, y_dtype, 0.01, 0.002, part=part)
    bd = L.BNDesc(dtype=y_dtype, m=n * P * Q, c=d.k_pad, c_real=k, eps=1e-5, momentum=0.9, fix_gamma=0, relu=0)
    f = lambda a: torch.tensor(np.pad(a, (0, d.k_pad - k)), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(np.ones(k)), f(np.zeros(k)), f(np.zeros(k)), f(np.ones(k))
    sm, si, sc, sh = [torch.zeros(d.k_pad, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    ydev = to_nhwc(y, y_dtype, gpu, d.k_pad)
    yb = torch.zeros_like(ydev)
    L.call("rn_bn_fwd_train_part", C.byref(bd), p(part), nblk, rows, d.k_pad, p(ydev), p(yb), p(g_d), p(b_d), p(mm),
           p(mv), p(sm), p(si), p(sc), p(sh), p(ws), stream())
    torch.cuda.synchronize()
    assert rel_err(sm.cpu().numpy()[:k], y.mean(axis=(0, 2, 3))) < 1e-5
    var = y.var(axis=(0, 2, 3))
    assert rel_err(1.0 / si.cpu().numpy()[:k] ** 2 - 1e-5, var) < 1e-4


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("is_weight", [0, 1])
def test_quant_codes_match_values(gpu, dtype, is_weight):
    """rn_quant_int8_fwd_codes: the fake-quantized output equals rn_quant_int8_fwd's, and equals
    code * unit (fp32; for bf16 its rounding); the EMA state updates as the plain call does."""
    rng = np.random.default_rng(7)
    n = 4096
    x = torch.tensor(rng.standard_normal(n) * 2.0, dtype=tdt(dtype), device=gpu)
    out1 = torch.zeros_like(x)
    out2 = torch.zeros_like(x)
    codes = torch.zeros(n, dtype=torch.int8, device=gpu)
    unit = torch.zeros(1, dtype=torch.float32, device=gpu)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    mm1 = torch.tensor([1.5], dtype=torch.float32, device=gpu)
    mm2 = mm1.clone()
    L.call("rn_quant_int8_fwd", dtype, n, p(x), p(out1), p(mm1), is_weight, 1, 0.99, 0, 8, p(ws), stream())
    L.call("rn_quant_int8_fwd_codes", dtype, n, p(x), p(out2), p(codes), p(unit), p(mm2), is_weight, 1, 0.99, 0, 8,
           p(ws), stream())
    torch.cuda.synchronize()
    assert torch.equal(out1, out2)
    assert torch.equal(mm1, mm2)
    u = unit.item()
    t = (x.abs().max().item() if is_weight else mm2.item())
    assert u == np.float32(np.float32(t) / np.float32(127))
    val = codes.cpu().numpy().astype(np.float32) * np.float32(u)
    want = torch.tensor(val).to(tdt(dtype)).float().numpy()
    np.testing.assert_array_equal(out2.float().cpu().numpy(), want)
    assert np.abs(codes.cpu().numpy()).max() <= 127


def test_weight_pack_i8(gpu):
    rng = np.random.default_rng(9)
    k, c, r = 40, 48, 3
    d = conv_desc(BF16, 1, c, 8, 8, k, r, r, 1, 1)
    wt = rng.standard_normal((k, c, r, r)).astype(np.float32)
    master = torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 2, 3, 1))).reshape(-1).to(gpu)
    qw = torch.zeros_like(master)
    unit = torch.zeros(1, dtype=torch.float32, device=gpu)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    L.call("rn_quant_int8_fwd_codes", F32, master.numel(), p(master), p(qw), None, p(unit), None, 1, 1, 0.99, 0, 8,
           p(ws), stream())
    wk8 = torch.zeros(k * r * r * d.c, dtype=torch.int8, device=gpu)
    L.call("rn_conv_weight_pack_i8", C.byref(d), p(master), p(unit), p(wk8), stream())
    torch.cuda.synchronize()
    codes = wk8.cpu().numpy().reshape(k, r, r, d.c)
    assert not codes[..., c:].any()
    u = np.float32(unit.item())
    qv = qw.cpu().numpy().reshape(k, r, r, c)
    np.testing.assert_array_equal(codes[..., :c].astype(np.float32) * u, qv)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("relu", [1, 0])
@pytest.mark.parametrize("m,c", [(3136, 64), (1001, 48), (98, 2048), (7, 16)])
def test_quant_codes_bn_fused(gpu, dtype, relu, m, c):
    """rn_quant_int8_fwd_codes_bn (the BatchNorm applied on load) == rn_bn_apply followed by
    rn_quant_int8_fwd_codes, bit for bit: values, codes, unit and the EMA state, training (max|y| and
    the EMA update) and inference (the moving threshold); c = 48 leaves threads of each block idle."""
    rng = np.random.default_rng(m + c)
    x = torch.tensor(rng.standard_normal((m, c)) * 3.0, dtype=tdt(dtype), device=gpu)
    sc = torch.tensor(rng.standard_normal(c) * 0.7, dtype=torch.float32, device=gpu)
    sh = torch.tensor(rng.standard_normal(c) * 0.5, dtype=torch.float32, device=gpu)
    d = L.BNDesc(dtype=dtype, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=relu)
    n = m * c
    y = torch.zeros_like(x)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    for train in (1, 0):
        outs = []
        # (deferred: codes only, then rn_quant_int8_expand -- the int8 graph's weight-gradient stream)
        for fused in (False, True, "deferred"):
            out = torch.full_like(x, float("nan"))
            codes = torch.zeros(n, dtype=torch.int8, device=gpu)
            unit = torch.zeros(1, dtype=torch.float32, device=gpu)
            mm = torch.tensor([2.5], dtype=torch.float32, device=gpu)
            if fused == "deferred":
                L.call("rn_quant_int8_fwd_codes_bn", C.byref(d), p(x), p(sc), p(sh), None, p(codes), p(unit), p(mm),
                       train, 0.99, 0, 8, p(ws), stream())
                torch.cuda.synchronize()
                assert torch.isnan(out.float()).all()
                L.call("rn_quant_int8_expand", dtype, n, p(codes), p(unit), p(out), stream())
            elif fused:
                L.call("rn_quant_int8_fwd_codes_bn", C.byref(d), p(x), p(sc), p(sh), p(out), p(codes), p(unit), p(mm),
                       train, 0.99, 0, 8, p(ws), stream())
            else:
                L.call("rn_bn_apply", C.byref(d), p(x), p(y), p(sc), p(sh), stream())
                L.call("rn_quant_int8_fwd_codes", dtype, n, p(y), p(out), p(codes), p(unit), p(mm), 0, train, 0.99,
                       0, 8, p(ws), stream())
            outs.append((out, codes, unit, mm))
        torch.cuda.synchronize()
        for a, b, e in zip(*outs):
            assert torch.equal(a, b) and torch.equal(a, e)
        assert ws[0].item() == 0.0  # the shared workspace's running max is left zero
        if train:
            yv = y.float()
            assert outs[1][3].item() != 2.5 and yv.abs().max().item() > 0


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("mode", [63, 119])
def test_quant_codes_bn_store_hints(gpu, dtype, mode):
    """rn_set_tuning 18 bit 8 (streaming hints) and bit 64 (write-through stores) change only the cache
    policy of rn_quant_int8_fwd_codes_bn: values, codes and unit equal the default (55) bit for bit."""
    m, c = 1001, 48
    rng = np.random.default_rng(11)
    x = torch.tensor(rng.standard_normal((m, c)) * 3.0, dtype=tdt(dtype), device=gpu)
    sc = torch.tensor(rng.standard_normal(c) * 0.7, dtype=torch.float32, device=gpu)
    sh = torch.tensor(rng.standard_normal(c) * 0.5, dtype=torch.float32, device=gpu)
    d = L.BNDesc(dtype=dtype, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    outs = []
    try:
        for md in (55, mode):
            L.call("rn_set_tuning", 18, md)
            out = torch.full_like(x, float("nan"))
            codes = torch.zeros(m * c, dtype=torch.int8, device=gpu)
            unit = torch.zeros(1, dtype=torch.float32, device=gpu)
            mm = torch.tensor([2.5], dtype=torch.float32, device=gpu)
            L.call("rn_quant_int8_fwd_codes_bn", C.byref(d), p(x), p(sc), p(sh), p(out), p(codes), p(unit), p(mm),
                   1, 0.99, 0, 8, p(ws), stream())
            torch.cuda.synchronize()
            outs.append((out, codes, unit, mm))
    finally:
        L.call("rn_set_tuning", 18, 55)  # the default
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert not torch.isnan(outs[1][0].float()).any()


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_quant_codes_bn_ties(gpu, dtype):
    """The fused quantizer forms the quotient v / unit as v * (1 / unit) and takes the exact division
    only near a half-integer: with unit = 2^-6 (threshold 127 * 2^-6, inference mode) every input
    (2k + 1) / 128 is an exact tie, which must round half away from zero as round(v / unit) does --
    codes and values bit for bit against rn_bn_apply + rn_quant_int8_fwd_codes and numpy."""
    k = np.arange(-130, 130)
    vals = (2 * k + 1) / 128.0                       # ties (+ a few past the clip at +-127 * 2^-6)
    m, c = 64, 16
    rng = np.random.default_rng(3)
    x = torch.tensor(rng.choice(vals, size=(m, c)), dtype=tdt(dtype), device=gpu)
    sc = torch.ones(c, dtype=torch.float32, device=gpu)
    sh = torch.zeros(c, dtype=torch.float32, device=gpu)
    d = L.BNDesc(dtype=dtype, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=0)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    outs = []
    for fused in (False, True):
        out = torch.zeros_like(x)
        codes = torch.zeros(m * c, dtype=torch.int8, device=gpu)
        unit = torch.zeros(1, dtype=torch.float32, device=gpu)
        mm = torch.tensor([127 / 64.0], dtype=torch.float32, device=gpu)
        if fused:
            L.call("rn_quant_int8_fwd_codes_bn", C.byref(d), p(x), p(sc), p(sh), p(out), p(codes), p(unit), p(mm),
                   0, 0.99, 0, 8, p(ws), stream())
        else:
            y = torch.zeros_like(x)
            L.call("rn_bn_apply", C.byref(d), p(x), p(y), p(sc), p(sh), stream())
            L.call("rn_quant_int8_fwd_codes", dtype, m * c, p(y), p(out), p(codes), p(unit), p(mm), 0, 0, 0.99,
                   0, 8, p(ws), stream())
        outs.append((out, codes, unit))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert outs[1][2].item() == 1 / 64.0
    xv = x.double().cpu().numpy()
    ref = np.sign(xv) * np.floor(np.abs(np.clip(xv, -127 / 64, 127 / 64)) * 64 + 0.5)  # half away from zero
    np.testing.assert_array_equal(outs[1][1].cpu().numpy().reshape(m, c), ref.astype(np.int8))


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("m,c", [(3136, 64), (1001, 48)])
def test_quant_codes_bn_pair(gpu, dtype, m, c):
    """rn_quant_int8_fwd_codes_bn2 (the two quantizers of one BN output, symbol/resnet_int8.py's first
    units: conv1 and the shortcut) == rn_bn_apply + rn_quant_int8_fwd_codes twice, bit for bit: both
    quantizers' values, codes, units and EMA states (different states, decays and nbits)."""
    rng = np.random.default_rng(m + c + 1)
    x = torch.tensor(rng.standard_normal((m, c)) * 3.0, dtype=tdt(dtype), device=gpu)
    sc = torch.tensor(rng.standard_normal(c) * 0.7, dtype=torch.float32, device=gpu)
    sh = torch.tensor(rng.standard_normal(c) * 0.5, dtype=torch.float32, device=gpu)
    d = L.BNDesc(dtype=dtype, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    n = m * c
    y = torch.zeros_like(x)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    qs = [(2.5, 0.99, 8), (1.25, 0.9, 4)]  # (minmax state, ema decay, nbits) of the two quantizers
    for train in (1, 0):
        res = []
        for fused in (False, True):
            bufs = [(torch.full_like(x, float("nan")), torch.zeros(n, dtype=torch.int8, device=gpu),
                     torch.zeros(1, dtype=torch.float32, device=gpu),
                     torch.tensor([mm0], dtype=torch.float32, device=gpu)) for mm0, _, _ in qs]
            if fused:
                (o1, c1, u1, m1), (o2, c2, u2, m2) = bufs
                L.call("rn_quant_int8_fwd_codes_bn2", C.byref(d), p(x), p(sc), p(sh), p(o1), p(c1), p(u1), p(m1),
                       qs[0][1], qs[0][2], p(o2), p(c2), p(u2), p(m2), qs[1][1], qs[1][2], train, 0, p(ws), stream())
            else:
                L.call("rn_bn_apply", C.byref(d), p(x), p(y), p(sc), p(sh), stream())
                for (o, cd, u, mm), (_, dec, nb) in zip(bufs, qs):
                    L.call("rn_quant_int8_fwd_codes", dtype, n, p(y), p(o), p(cd), p(u), p(mm), 0, train, dec, 0, nb,
                           p(ws), stream())
            res.append(bufs)
        torch.cuda.synchronize()
        for b0, b1 in zip(*res):
            for a, b in zip(b0, b1):
                assert torch.equal(a, b)
        assert ws[0].item() == 0.0
        assert not torch.equal(res[1][0][1], res[1][1][1])  # (8 and 4 bits: different codes)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("use_global", [False, True])
def test_bn_backward_quant_pair_fold(gpu, dtype, use_global):
    """The two quantizers of one BN+ReLU output folded into its backward (rn_bn_desc.clip / clip2 / dy2):
    rn_bn_bwd[_global] == two rn_quant_int8_bwd summing into one buffer followed by rn_bn_bwd[_global]
    without clips, bit for bit (dx, dgamma, dbeta); rn_bn_bwd_part refuses dy2."""
    n, c, h, w = 3, 96, 13, 11
    rng = np.random.default_rng(41)
    xb = rng.standard_normal((n, c, h, w)) * 1.5 + 0.3
    lib = L.load()
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    g_d, b_d = f(rng.uniform(0.5, 1.5, c)), f(rng.standard_normal(c) * 0.2)
    mm, mv = f(rng.standard_normal(c) * 0.1), f(rng.uniform(0.8, 1.2, c))
    sm, si, sc, sh = [torch.zeros(c, dtype=torch.float32, device=gpu) for _ in range(4)]
    bd = L.BNDesc(dtype=dtype, m=n * h * w, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    xbd = to_nhwc(xb, dtype, gpu)
    act = torch.zeros_like(xbd)
    if use_global:
        L.call("rn_bn_fwd_infer", C.byref(bd), p(xbd), p(act), p(g_d), p(b_d), p(mm), p(mv), p(sc), p(sh), stream())
    else:
        L.call("rn_bn_fwd_train", C.byref(bd), p(xbd), p(act), p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc),
               p(sh), p(ws), stream())
    torch.cuda.synchronize()
    a_np = from_nhwc(act, c)
    t1, t2 = (float(np.quantile(a_np[a_np > 0], qq)) for qq in (0.6, 0.85))
    tq1, tq2 = (torch.tensor([t], dtype=torch.float32, device=gpu) for t in (t1, t2))
    dy1, dy2 = (to_nhwc(rng.standard_normal((n, c, h, w)), dtype, gpu) for _ in range(2))
    zf = lambda: torch.zeros(c, dtype=torch.float32, device=gpu)
    bwd = "rn_bn_bwd_global" if use_global else "rn_bn_bwd"
    stats = (p(mm), p(mv)) if use_global else (p(sm), p(si))
    g = torch.zeros_like(xbd)
    L.call("rn_quant_int8_bwd", dtype, act.numel(), p(act), p(dy2), p(g), p(tq2), 0, None, stream())
    L.call("rn_quant_int8_bwd", dtype, act.numel(), p(act), p(dy1), p(g), p(tq1), 0, p(g), stream())
    dx0, dg0, db0 = torch.zeros_like(xbd), zf(), zf()
    L.call(bwd, C.byref(bd), p(xbd), p(g), p(dx0), None, p(g_d), *stats, p(sc), p(sh), p(dg0), p(db0), p(ws), stream())
    bdp = L.BNDesc(dtype=dtype, m=n * h * w, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1,
                   clip=tq1.data_ptr(), clip2=tq2.data_ptr(), dy2=dy2.data_ptr())
    dx1, dg1, db1 = torch.zeros_like(xbd), zf(), zf()
    L.call(bwd, C.byref(bdp), p(xbd), p(dy1), p(dx1), None, p(g_d), *stats, p(sc), p(sh), p(dg1), p(db1), p(ws),
           stream())
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1) and torch.equal(dg0, dg1) and torch.equal(db0, db1)
    pos = act > 0
    assert ((g == 0) & pos).float().sum().item() > 0.05 * pos.float().sum().item()  # the clips bit
    part = torch.zeros(64, dtype=torch.float32, device=gpu)
    assert lib.rn_bn_bwd_part(C.byref(bdp), p(part), 1, p(xbd), p(dy1), p(dx1), None, p(g_d), p(sm), p(si), p(sc),
                              p(sh), p(dg1), p(db1), p(ws), stream()) != 0


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_weight_quant_pack_batched(gpu, dtype):
    """rn_weight_quant_pack (every weight quantizer in three launches) == per weight
    rn_quant_int8_fwd_codes + rn_conv_weight_pack (CRSK) + rn_conv_weight_pack_i8, bit for bit: the
    fake-quantized copies, units, threshold states, int8 codes and data-gradient copies; an unaligned
    master (a flat parameter buffer's offset) and items without codes / copies (stem, fc)."""
    rng = np.random.default_rng(5)
    # (k, c, r, nbits, int8 conv): 1x1 / 3x3 / ragged channels (c_real < c) / an fc-like item
    shapes = [(64, 64, 1, 8, True), (48, 40, 3, 8, True), (24, 16, 3, 4, True), (10, 20, 1, 8, False)]
    total = sum(k * c * r * r for k, c, r, _, _ in shapes) + 1
    master = torch.tensor(rng.standard_normal(total) * 0.1, dtype=torch.float32, device=gpu)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    items, refs, off = [], [], 1  # (offset 1: a master not 16-byte aligned)
    for k, c, r, nb, i8 in shapes:
        n = k * c * r * r
        wm = master[off:off + n]
        off += n
        d = conv_desc(dtype, 2, c, 8, 8, k, r, r, 1, r // 2)
        bufs = {}
        for tag in ("a", "b"):
            bufs[tag] = dict(qw=torch.zeros(n, device=gpu), unit=torch.zeros(1, device=gpu),
                             mm=torch.zeros(1, device=gpu),
                             codes=torch.zeros(k * r * r * d.c, dtype=torch.int8, device=gpu) if i8 else None,
                             wc=torch.zeros(d.c * r * r * d.k_pad, dtype=tdt(dtype), device=gpu) if i8 else None)
        a = bufs["a"]
        L.call("rn_quant_int8_fwd_codes", F32, n, p(wm), p(a["qw"]), None, p(a["unit"]), p(a["mm"]), 1, 1, 0.99, 0,
               nb, p(ws), stream())
        if i8:
            L.call("rn_conv_weight_pack", C.byref(d), p(a["qw"]), None, p(a["wc"]), stream())
            L.call("rn_conv_weight_pack_i8", C.byref(d), p(wm), p(a["unit"]), p(a["codes"]), stream())
        b = bufs["b"]
        items.append(L.WQuantItem(master=wm.data_ptr(), qw=b["qw"].data_ptr(), unit=b["unit"].data_ptr(),
                                  minmax=b["mm"].data_ptr(), w_codes=b["codes"].data_ptr() if i8 else None,
                                  w_crsk=b["wc"].data_ptr() if i8 else None, k=k, rs=r * r, c_real=c,
                                  c=d.c, k_pad=d.k_pad, nbits=nb))
        refs.append(bufs)
    arr = (L.WQuantItem * len(items))(*items)
    dev = torch.frombuffer(bytearray(arr), dtype=torch.uint8).to(gpu)
    # the shared workspace as the executor hands it over after a forward: the activation quantizers
    # leave their thresholds in ws[1..2] (they were taken as weight maxima)
    ws[1:3] = 1e3
    L.call("rn_weight_quant_pack", p(dev), len(items), dtype, p(ws), stream())
    torch.cuda.synchronize()
    assert not ws[:len(items)].any()
    for bufs in refs:
        for key in ("qw", "unit", "mm", "codes", "wc"):
            if bufs["a"][key] is not None:
                assert torch.equal(bufs["a"][key], bufs["b"][key]), key
    assert refs[0]["b"]["unit"].item() > 0


@pytest.mark.parametrize("case", [CASES[1], CASES[2], CASES[0], CASES[3]])
def test_int8_conv_block_extremes_feed_quantizer_max(gpu, case):
    """rn_conv_fwd_i8_mm: the same output and BatchNorm partials as rn_conv_fwd_i8, plus per block and
    channel the max of the stored output (the min where the sign vector -- the consuming BN's gamma --
    is negative); with them in rn_bn_desc.xmm the BN+ReLU-on-load quantizer (rn_quant_int8_fwd_codes_bn)
    takes max|y| from the extremes instead of a pass over x -- and writes bit-identical values,
    codes, unit and EMA state."""
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(sum(case) + 5)
    lib = L.load()
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    rows = lib.rn_conv_bn_part_rows(C.byref(d), 2)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    m = n * P * Q
    nblk = -(-m // rows)
    xd = torch.from_numpy(rng.integers(-127, 128, (n, h, w, d.c)).astype(np.int8)).to(gpu)
    wd = torch.from_numpy(rng.integers(-127, 128, (k, r, r, d.c)).astype(np.int8)).reshape(-1).to(gpu)
    ux, uw = (torch.tensor([u], dtype=torch.float32, device=gpu) for u in (0.011, 0.0007))
    # BN scale with both signs (its gamma's sign), shift
    sc = torch.tensor(rng.standard_normal(d.k_pad) * 0.02, dtype=torch.float32, device=gpu)
    sh = torch.tensor(rng.standard_normal(d.k_pad) * 0.5, dtype=torch.float32, device=gpu)
    sc[k:] = 0
    sh[k:] = 0
    sgn = sc.clone()
    outs = []
    for mm in (False, True):
        y = torch.zeros((m, d.k_pad), dtype=torch.bfloat16, device=gpu)
        part = torch.zeros(nblk * 3 * d.k_pad, dtype=torch.float32, device=gpu)
        pmm = torch.full((nblk * d.k_pad,), float("nan"), dtype=torch.float32, device=gpu) if mm else None
        if mm:
            L.call("rn_conv_fwd_i8_mm", C.byref(d), p(xd), p(wd), p(y), BF16, None, p(ux), p(uw), p(part), p(pmm),
                   p(sgn), stream())
        else:
            L.call("rn_conv_fwd_i8", C.byref(d), p(xd), p(wd), p(y), BF16, None, p(ux), p(uw), p(part), stream())
        outs.append((y, part, pmm))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    yv = outs[1][0].float().cpu().numpy()
    pmm = outs[1][2].cpu().numpy().reshape(nblk, d.k_pad)
    pad = nblk * rows - m
    yb = np.concatenate([yv, np.full((pad, d.k_pad), np.nan, np.float32)]).reshape(nblk, rows, d.k_pad)
    neg = sgn.cpu().numpy()[:k] < 0
    want = np.where(neg[None, :], np.nanmin(yb, axis=1)[:, :k], np.nanmax(yb, axis=1)[:, :k])
    np.testing.assert_array_equal(pmm[:, :k], want)
    # the quantizer of relu(bn(y)): max from the extremes == max from a pass over y
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    res = []
    for mm in (False, True):
        bd = L.BNDesc(dtype=BF16, m=m, c=d.k_pad, c_real=k, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1,
                      xmm=outs[1][2].data_ptr() if mm else None, xmm_blocks=nblk if mm else 0)
        out = torch.zeros_like(outs[0][0])
        codes = torch.zeros(m * d.k_pad, dtype=torch.int8, device=gpu)
        unit = torch.zeros(1, dtype=torch.float32, device=gpu)
        mmst = torch.tensor([1.0], dtype=torch.float32, device=gpu)
        L.call("rn_quant_int8_fwd_codes_bn", C.byref(bd), p(outs[0][0]), p(sc), p(sh), p(out), p(codes), p(unit),
               p(mmst), 1, 0.99, 1, 8, p(ws), stream())
        res.append((out, codes, unit, mmst))
    torch.cuda.synchronize()
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert res[1][3].item() > 0  # (first batch: the state is the max itself)


def test_weight_quant_pack_batched_multistep(gpu, monkeypatch):
    """The int8 graph (symbol/resnet_int8.py, one unit per stage) for three bf16 QAT steps with the
    batched weight quantizer (RN_WQUANT_BATCH=1, the default) and with one call per weight (=0):
    after steps 2 and 3 -- repacks that follow a forward whose activation quantizers left their
    thresholds in the shared workspace -- every fake-quantized weight, weight unit, int8 weight code,
    data-gradient copy and minmax state is bit-identical, and so are the outputs (the
    batched form took the stale thresholds as weight maxima from step 2 on)."""
    import mxnet as mx
    from oracle import net as onet
    from rn import graphs
    from step_util import oracle_state
    cfg = ([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16)
    g = onet.resnet_int8(*cfg)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    runs = []
    for batched in ("1", "0"):
        monkeypatch.setenv("RN_WQUANT_BATCH", batched)
        mod = mx.mod.Module(graphs.resnet_int8(*cfg), context=[mx.gpu(0)], precision="bfloat16")
        mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", label.shape)])
        mod.init_params(arg_params={k: v.astype(np.float32) for k, v in args.items()},
                        aux_params={k: v.astype(np.float32) for k, v in aux.items()}, allow_missing=True)
        mod.init_optimizer(kvstore="device", optimizer="sgd",
                           optimizer_params={"learning_rate": 0.05, "wd": 1e-4, "momentum": 0.9})
        batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
        probs = []
        for _ in range(3):
            mod.forward(batch, is_train=True)
            probs.append(mod.get_outputs()[0].asnumpy().copy())
            mod.backward()
            mod.update()
        ex = mod.executor
        assert ex._wq_batch == (batched == "1")
        state = {}
        for op in ex.plan.ops:
            if getattr(op, "qweight", None) is None:
                continue
            for attr in ("qw", "wunit", "wk8", "wc"):
                t = getattr(op, attr, None)
                if t is not None:
                    state[(op.weight, attr)] = t.detach().cpu().clone()
        torch.cuda.synchronize()
        st = {k: v.asnumpy() for k, v in mod.get_params()[1].items() if k.endswith("_minmax")}
        runs.append((probs, state, st))
    (p1, s1, m1), (p0, s0, m0) = runs
    assert len(s1) >= 4 * 5 and set(s1) == set(s0)
    for k in s1:
        assert torch.equal(s1[k], s0[k]), k
    assert set(m1) == set(m0) and any(k.endswith("_weight_minmax") for k in m1)
    for k in m1:
        np.testing.assert_array_equal(m1[k], m0[k], err_msg=k)
    for a, b in zip(p1, p0):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("case", [
    (3, 64, 56, 56, 64, 3, 1, 1),      # the quantized stage-1 conv2 (several bands per workgroup)
    (5, 64, 9, 13, 64, 3, 1, 1),       # a last band of one output row
    (1, 64, 7, 7, 64, 3, 1, 1),        # fewer pixels than one band
    (40, 64, 20, 56, 64, 3, 1, 1),     # the widest row, many bands per workgroup
])
def test_int8_conv3x3_band(gpu, case):
    """conv3x3c64_band_i8_kernel (the int8 image-band forward of a 3x3 / stride-1 / pad-1 64 -> 64
    layer, default; rn_set_tuning 26 = 1 the int8 implicit-GEMM tile): exact integer sums (f32 path of the
    tile vs the oracle) and the bf16 output bit-identical to the tile's, both scaling the same int32 sums."""
    n, c, h, w, k, r, st, pd = case
    ux, uw = 0.0123, 0.00071
    outs = []
    try:
        for mode in (0, 1):
            L.call("rn_set_tuning", 26, mode)
            _, y, exact = _run(gpu, case, BF16, ux, uw)
            outs.append(y)
    finally:
        L.call("rn_set_tuning", 26, 0)
    np.testing.assert_array_equal(outs[0], outs[1])
    ref = exact * (np.float64(np.float32(ux)) * np.float64(np.float32(uw)))
    assert rel_err(outs[0], ref) < 2 ** -8
