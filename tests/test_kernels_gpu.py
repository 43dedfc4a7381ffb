"""Per-kernel parity of librn against the numpy oracle (oracle/ops.py) on the GPU.

Tolerances (max |err| / max |ref|):
  fp32 path: 2e-5 (exact-fp32 MFMA products, fp32 accumulation order differs from fp64)
  bf16 path: 1.5e-2 (oracle fed the same bf16-rounded inputs; output rounded to bf16 = 2^-8)
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import ops
from rn import lib as L
from gpu_util import BF16, F32, bf16_round, conv_desc, from_nhwc, p, pad8, rel_err, stream, tdt, to_nhwc

pytestmark = pytest.mark.gpu

TOL = {F32: 2e-5, BF16: 1.5e-2}

CONV_CASES = [
    # n, c, h, w, k, r, stride, pad
    (2, 64, 14, 14, 64, 1, 1, 0),
    (2, 64, 14, 14, 128, 3, 1, 1),
    (3, 32, 13, 11, 48, 3, 2, 1),
    (2, 64, 14, 14, 256, 1, 2, 0),
    (2, 128, 7, 7, 24, 3, 1, 1),
    (4, 16, 9, 9, 40, 5, 2, 2),
    (2, 8, 16, 16, 16, 7, 2, 3),
    (1, 256, 4, 4, 1000, 1, 1, 0),
]


def _conv_data(case, seed):
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, c, h, w))
    wt = rng.standard_normal((k, c, r, r)) / np.sqrt(c * r * r)
    return x, wt


def _master_krsc(wt, dev):
    return torch.from_numpy(np.ascontiguousarray(wt.transpose(0, 2, 3, 1), dtype=np.float32)).reshape(-1).to(dev)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd(gpu, dtype, case):
    n, c, h, w, k, r, st, pd = case
    x, wt = _conv_data(case, 1)
    if dtype == BF16:
        x, wt = bf16_round(x), bf16_round(wt)
    res = np.random.default_rng(2).standard_normal((n, k) + ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd)))
    if dtype == BF16:
        res = bf16_round(res)
    ref = ops.conv2d_fwd(x, wt, (st, st), (pd, pd)) + res
    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd)
    xd = to_nhwc(x, dtype, gpu)
    wk = torch.zeros(k * r * r * d.c, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), None, stream())
    y = torch.zeros((n, d.p, d.q, d.k_pad), dtype=tdt(dtype), device=gpu)
    rd = to_nhwc(res, dtype, gpu)
    L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(y), dtype, p(rd), None, stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(y, k), ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_bwd(gpu, dtype, case):
    n, c, h, w, k, r, st, pd = case
    x, wt = _conv_data(case, 3)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = np.random.default_rng(4).standard_normal((n, k, P, Q))
    if dtype == BF16:
        x, wt, dy = bf16_round(x), bf16_round(wt), bf16_round(dy)
    dx_ref, dw_ref = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd))
    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd)
    xd = to_nhwc(x, dtype, gpu)
    dyd = to_nhwc(dy, dtype, gpu)
    wc = torch.zeros(d.c * r * r * d.k_pad, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), None, p(wc), stream())
    dx = torch.zeros((n, h, w, d.c), dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(dx), None, stream())
    dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dyd), p(dw), stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(dx, c), dx_ref) < TOL[dtype]
    dw_h = dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2)
    assert rel_err(dw_h, dw_ref) < (TOL[dtype] if dtype == F32 else 5e-3)


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_stem_im2col_and_shift_grad(gpu, dtype):
    """conv0 as im2col + 1x1 GEMM (with bn_data affine) and d(beta) without the stem dgrad."""
    n, c, h, w, k, r, st, pd = 2, 3, 20, 18, 16, 7, 2, 3
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, (n, c, h, w))
    wt = rng.standard_normal((k, c, r, r)) * 0.1
    scale = np.array([1.5, 0.5, 2.0])
    shift = np.array([0.1, -0.2, 0.3])
    xa = x * scale[None, :, None, None] + shift[None, :, None, None]
    if dtype == BF16:
        xa, wt = bf16_round(xa), bf16_round(wt)
    ref = ops.conv2d_fwd(xa, wt, (st, st), (pd, pd))
    P, Q = ref.shape[2:]
    kc = 160
    d1 = conv_desc(dtype, n, kc, P, Q, k, 1, 1, 1, 0, c_real=r * r * c)
    dfull = conv_desc(dtype, n, 8, h, w, k, r, r, st, pd, c_real=c)
    xd = torch.from_numpy(x.astype(np.float32)).to(gpu)
    sc = torch.tensor(scale, dtype=torch.float32, device=gpu)
    sh = torch.tensor(shift, dtype=torch.float32, device=gpu)
    cols = torch.zeros(n * P * Q * kc, dtype=tdt(dtype), device=gpu)
    L.call("rn_im2col_nchw", C.byref(dfull), p(xd), p(sc), p(sh), p(cols), kc, stream())
    master = _master_krsc(wt, gpu)
    wk = torch.zeros(k * kc, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d1), p(master), p(wk), None, stream())
    y = torch.zeros((n, P, Q, pad8(k)), dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_fwd", C.byref(d1), p(cols), p(wk), p(y), dtype, None, None, stream())
    # wgrad through the cols matrix, d(shift) via rn_stem_shift_grad
    dy = rng.standard_normal((n, k, P, Q))
    if dtype == BF16:
        dy = bf16_round(dy)
    dx_ref, dw_ref = ops.conv2d_bwd(xa, wt, dy, (st, st), (pd, pd))
    dshift_ref = dx_ref.sum(axis=(0, 2, 3))
    dyd = to_nhwc(dy, dtype, gpu)
    dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter", C.byref(d1), p(cols), p(dyd), p(dw), stream())
    dbeta = torch.zeros(c, dtype=torch.float32, device=gpu)
    ws = torch.zeros(P * Q * pad8(k) + P * r * k + k * r * r, dtype=torch.float32, device=gpu)
    L.call("rn_stem_shift_grad", C.byref(dfull), p(dyd), p(master), p(dbeta), p(ws), stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(y, k), ref) < TOL[dtype]
    assert rel_err(dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2), dw_ref) < \
        (TOL[dtype] if dtype == F32 else 5e-3)
    assert rel_err(dbeta.cpu().numpy(), dshift_ref) < (1e-4 if dtype == F32 else 5e-3)


BN_CASES = [(4, 64, 9, 9, False, True), (2, 24, 5, 7, True, False), (8, 256, 4, 4, False, False),
            (2, 2048, 2, 2, False, True)]


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("relu", [False, True])
def test_bn_streaming_hint_variants(gpu, dtype, relu):
    """rn_set_tuning 18 (nontemporal stores / loads in the BatchNorm passes) changes only the cache
    policy: rn_bn_fwd_train's y and rn_bn_bwd's reduction and dx (with the residual add) are
    bit-identical for every mask value (bit 32: the apply passes' write-through stores)."""
    n, c, h, w = 4, 200, 9, 13
    rng = np.random.default_rng(61)
    x = rng.standard_normal((n, c, h, w)) * 2 + 0.5
    dy = rng.standard_normal((n, c, h, w))
    add = rng.standard_normal((n, c, h, w))
    gamma, beta = rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.1
    d = L.BNDesc(dtype=dtype, m=n * h * w, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=int(relu))
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=gpu)
    xd, dyd, addd = to_nhwc(x, dtype, gpu), to_nhwc(dy, dtype, gpu), to_nhwc(add, dtype, gpu)
    ws = torch.zeros(L.load().rn_bn_workspace_bytes(C.byref(d)) // 4 + 16, dtype=torch.float32, device=gpu)
    outs = []
    try:
        for mode in (0, 1, 2, 3, 6, 7, 32, 34, 55):
            L.call("rn_set_tuning", 18, mode)
            g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
            sm, si, sc, sh = [torch.zeros(c, dtype=torch.float32, device=gpu) for _ in range(4)]
            yd, dxd = torch.zeros_like(xd), torch.zeros_like(xd)
            dg, db = torch.zeros(c, dtype=torch.float32, device=gpu), torch.zeros(c, dtype=torch.float32, device=gpu)
            L.call("rn_bn_fwd_train", C.byref(d), p(xd), p(yd), p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc),
                   p(sh), p(ws), stream())
            L.call("rn_bn_bwd", C.byref(d), p(xd), p(dyd), p(dxd), p(addd), p(g_d), p(sm), p(si), p(sc), p(sh),
                   p(dg), p(db), p(ws), stream())
            torch.cuda.synchronize()
            outs.append((yd.cpu(), dxd.cpu(), dg.cpu(), db.cpu()))
    finally:
        L.call("rn_set_tuning", 18, 55)  # the default
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
    assert outs[0][0].abs().sum() > 0 and outs[0][1].abs().sum() > 0


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", BN_CASES)
def test_bn_relu(gpu, dtype, case):
    n, c, h, w, fix_gamma, relu = case
    rng = np.random.default_rng(6)
    x = rng.standard_normal((n, c, h, w)) * 2 + 0.5
    gamma = rng.uniform(0.5, 1.5, c)
    beta = rng.standard_normal(c) * 0.1
    dy = rng.standard_normal((n, c, h, w))
    if dtype == BF16:
        x, dy = bf16_round(x), bf16_round(dy)
    eps, mom = 1e-5, 0.9
    y_ref, cache = ops.bn_train_fwd(x, gamma, beta, eps, fix_gamma)
    if relu:
        dz = ops.relu_bwd(dy, ops.relu_fwd(y_ref))
        y_ref = ops.relu_fwd(y_ref)
    else:
        dz = dy
    dx_ref, dg_ref, db_ref = ops.bn_train_bwd(dz, cache, fix_gamma)
    mm_ref, mv_ref = ops.bn_moving_update(np.zeros(c), np.ones(c), cache[3], cache[4], mom)
    cp = pad8(c)
    d = L.BNDesc(dtype=dtype, m=n * h * w, c=cp, c_real=c, eps=eps, momentum=mom, fix_gamma=int(fix_gamma),
                 relu=int(relu))
    f = lambda a: torch.tensor(np.pad(a, (0, cp - c)), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
    sm, si, sc, sh = [torch.zeros(cp, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(L.load().rn_bn_workspace_bytes(C.byref(d)) // 4 + 16, dtype=torch.float32, device=gpu)
    xd = to_nhwc(x, dtype, gpu)
    yd = torch.zeros_like(xd)
    L.call("rn_bn_fwd_train", C.byref(d), p(xd), p(yd), p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc), p(sh),
           p(ws), stream())
    dyd = to_nhwc(dy, dtype, gpu)
    dxd = torch.zeros_like(xd)
    addd = to_nhwc(np.ones_like(x), dtype, gpu)
    dg, db = torch.zeros(cp, dtype=torch.float32, device=gpu), torch.zeros(cp, dtype=torch.float32, device=gpu)
    L.call("rn_bn_bwd", C.byref(d), p(xd), p(dyd), p(dxd), p(addd), p(g_d), p(sm), p(si), p(sc), p(sh), p(dg), p(db),
           p(ws), stream())
    # rn_bn_bwd with dx = NULL (reductions, dgamma / dbeta) + dx in row chunks: the same bits
    dx2 = torch.zeros_like(xd)
    dg2, db2 = torch.zeros_like(dg), torch.zeros_like(db)
    L.call("rn_bn_bwd", C.byref(d), p(xd), p(dyd), None, None, p(g_d), p(sm), p(si), p(sc), p(sh), p(dg2), p(db2),
           p(ws), stream())
    m, step = n * h * w, max(1, (n * h * w) // 3)  # (cp = 8k channels: every row starts on 16 bytes)
    for r0 in range(0, m, step):
        L.call("rn_bn_bwd_apply_rows", C.byref(d), p(xd), p(dyd), p(dx2), p(addd), p(sc), p(sh), p(ws), r0,
               min(step, m - r0), stream())
    torch.cuda.synchronize()
    assert torch.equal(dx2, dxd) and torch.equal(dg2, dg) and torch.equal(db2, db)
    tol = TOL[dtype]
    assert rel_err(from_nhwc(yd, c), y_ref) < tol
    assert rel_err(mm.cpu().numpy()[:c], mm_ref) < 1e-4
    assert rel_err(mv.cpu().numpy()[:c], mv_ref) < 1e-4
    assert rel_err(from_nhwc(dxd, c), dx_ref + 1.0) < (tol if dtype == F32 else 3e-2)
    assert rel_err(db.cpu().numpy()[:c], db_ref) < (1e-4 if dtype == F32 else 1e-2)
    if fix_gamma:
        assert np.all(dg.cpu().numpy() == 0)
    else:
        assert rel_err(dg.cpu().numpy()[:c], dg_ref) < (1e-4 if dtype == F32 else 1e-2)


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_maxpool_and_gap(gpu, dtype):
    rng = np.random.default_rng(7)
    n, c, h, w = 2, 16, 11, 12
    # many ties (post-ReLU zeros) to pin the first-max gradient rule
    x = np.maximum(rng.standard_normal((n, c, h, w)), 0)
    x = np.round(x * 4) / 4
    y_ref, arg = ops.maxpool_fwd(x, (3, 3), (2, 2), (1, 1))
    dy = rng.standard_normal(y_ref.shape)
    if dtype == BF16:
        dy = bf16_round(dy)
    dx_ref = ops.maxpool_bwd(dy, arg, x.shape, (3, 3), (2, 2), (1, 1))
    d = L.PoolDesc(dtype=dtype, n=n, h=h, w=w, c=pad8(c), r=3, s=3, stride_h=2, stride_w=2, pad_h=1, pad_w=1,
                   type=L.RN_POOL_MAX, global_pool=0)
    L.call("rn_pool_desc_init", C.byref(d))
    xd = to_nhwc(x, dtype, gpu)
    yd = torch.zeros((n, d.p, d.q, pad8(c)), dtype=tdt(dtype), device=gpu)
    am = torch.zeros(yd.numel(), dtype=torch.uint8, device=gpu)
    L.call("rn_pool_fwd", C.byref(d), p(xd), p(yd), p(am), stream())
    dyd = to_nhwc(dy, dtype, gpu)
    dxd = torch.zeros_like(xd)
    L.call("rn_pool_bwd", C.byref(d), p(dyd), p(am), p(dxd), None, stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(yd, c), y_ref) == 0.0
    assert rel_err(from_nhwc(dxd, c), dx_ref) < TOL[dtype]
    # global average pool
    g = L.PoolDesc(dtype=dtype, n=n, h=h, w=w, c=pad8(c), type=L.RN_POOL_AVG, global_pool=1)
    L.call("rn_pool_desc_init", C.byref(g))
    yg = torch.zeros((n, 1, 1, pad8(c)), dtype=tdt(dtype), device=gpu)
    L.call("rn_pool_fwd", C.byref(g), p(xd), p(yg), None, stream())
    dyg = rng.standard_normal((n, c, 1, 1))
    dxg = torch.zeros_like(xd)
    L.call("rn_pool_bwd", C.byref(g), p(to_nhwc(dyg, dtype, gpu)), None, p(dxg), None, stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(yg, c), ops.avgpool_global_fwd(x)) < TOL[dtype]
    dyg_r = bf16_round(dyg) if dtype == BF16 else dyg
    assert rel_err(from_nhwc(dxg, c), ops.avgpool_global_bwd(dyg_r, x.shape)) < TOL[dtype]


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("shape", [(3, 20, 11, 12), (2, 64, 56, 56), (4, 2048, 7, 7)])
def test_pool_bnrelu_on_load(gpu, dtype, shape):
    """rn_pool_fwd_x (the producing BatchNorm+ReLU applied to each loaded element: the stem's bn0 -> relu0
    -> max pool and the final bn1 -> relu1 -> global pool, symbol/resnet.py:94-97,111-113) == rn_bn_apply
    followed by rn_pool_fwd, BIT FOR BIT: the pooled values and the max pool's tap indices (many ReLU
    zeros: the first-max rule on ties), padded channels included."""
    n, c, h, w = shape
    rng = np.random.default_rng(71)
    x = rng.standard_normal((n, c, h, w)) * 1.5 + 0.2
    cp = pad8(c)
    sc = np.zeros(cp)
    sh = np.zeros(cp)
    sc[:c] = rng.uniform(0.3, 1.5, c) * np.where(rng.random(c) < 0.2, -1, 1)  # a few negative scales
    sh[:c] = rng.standard_normal(c) * 0.5
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=gpu)
    scd, shd = f(sc), f(sh)
    xd = to_nhwc(x, dtype, gpu)
    bd = L.BNDesc(dtype=dtype, m=n * h * w, c=cp, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    act = torch.zeros_like(xd)
    L.call("rn_bn_apply", C.byref(bd), p(xd), p(act), p(scd), p(shd), stream())
    for kind in ("max", "gap") if h * w <= 255 else ("max",):  # (the global pool's window: <= 255 taps)
        if kind == "max":
            d = L.PoolDesc(dtype=dtype, n=n, h=h, w=w, c=cp, r=3, s=3, stride_h=2, stride_w=2, pad_h=1, pad_w=1,
                           type=L.RN_POOL_MAX, global_pool=0)
        else:
            d = L.PoolDesc(dtype=dtype, n=n, h=h, w=w, c=cp, type=L.RN_POOL_AVG, global_pool=1)
        L.call("rn_pool_desc_init", C.byref(d))
        y0 = torch.full((n, d.p, d.q, cp), float("nan"), dtype=tdt(dtype), device=gpu)
        y1 = torch.full_like(y0, float("nan"))
        a0 = torch.full((y0.numel(),), 255, dtype=torch.uint8, device=gpu)
        a1 = torch.full_like(a0, 255)
        am = (lambda t: p(t)) if kind == "max" else (lambda t: None)
        L.call("rn_pool_fwd", C.byref(d), p(act), p(y0), am(a0), stream())
        L.call("rn_pool_fwd_x", C.byref(d), p(xd), p(y1), am(a1), p(scd), p(shd), stream())
        torch.cuda.synchronize()
        iv = torch.int16 if dtype == BF16 else torch.int32
        assert torch.equal(y0.view(iv), y1.view(iv)), kind
        if kind == "max":
            assert torch.equal(a0, a1)
            assert (y1.float() == 0).any()  # ReLU zeros: ties in the windows


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_softmax_output(gpu, dtype):
    rng = np.random.default_rng(8)
    b, ncls, ld = 37, 1000, 1000
    z = rng.standard_normal((b, ncls)) * 3
    lab = rng.integers(0, ncls, b).astype(np.float32)
    lab[0] = np.argmax(z[0])
    prob_ref = ops.softmax_output_fwd(z)
    g_ref = ops.softmax_output_bwd(prob_ref, lab)
    zd = torch.tensor(z, dtype=torch.float32, device=gpu)
    ld_ = torch.tensor(lab, dtype=torch.float32, device=gpu)
    prob = torch.zeros((b, ncls), dtype=torch.float32, device=gpu)
    dl = torch.zeros((b, ld), dtype=tdt(dtype), device=gpu)
    stats = torch.zeros(4, dtype=torch.float32, device=gpu)
    L.call("rn_softmax_output", dtype, b, ncls, ld, p(zd), p(ld_), p(prob), p(dl), C.c_float(1.0), p(stats), stream())
    torch.cuda.synchronize()
    assert rel_err(prob.cpu().numpy(), prob_ref) < 1e-5
    assert rel_err(dl.float().cpu().numpy(), g_ref) < (1e-5 if dtype == F32 else 1e-2)
    st = stats.cpu().numpy()
    assert abs(st[0] - ops.cross_entropy(prob_ref, lab)) < 1e-3 * b
    top1 = (np.argmax(z, 1) == lab).sum()
    top5 = sum(lab[i] in np.argsort(z[i])[-5:] for i in range(b))
    assert st[1] == top1 and st[2] == top5


def test_sgd_momentum(gpu):
    rng = np.random.default_rng(9)
    sizes = [7, 64, 1000, 3]
    names = ["a_weight", "a_beta", "fc_weight", "fc_bias"]
    offs = np.cumsum([0] + [((s + 3) // 4) * 4 for s in sizes])[:-1]
    total = int(offs[-1] + sizes[-1] + 4)
    w = rng.standard_normal(total).astype(np.float32)
    g = rng.standard_normal(total).astype(np.float32)
    m = rng.standard_normal(total).astype(np.float32) * 0.1
    wd = np.array([ops.wd_mult_for(n) * 1e-4 for n in names], dtype=np.float32)
    wr, mr = w.astype(np.float64).copy(), m.astype(np.float64).copy()
    for o, s, d in zip(offs, sizes, wd):
        ops.sgd_mom_update(wr[o:o + s], g[o:o + s].astype(np.float64), mr[o:o + s], 0.1, float(d), 0.9, 1 / 256.)
    t = lambda a, dt=torch.float32: torch.tensor(a, dtype=dt, device=gpu)
    # keep every device table alive until the kernel has run (no temporaries behind raw pointers)
    wd_, gd, md = t(w), t(g), t(m)
    offs_d, sizes_d, wds_d = t(offs, torch.int64), t(sizes, torch.int64), t(wd)
    L.call("rn_sgd_mom_update", len(sizes), p(offs_d), p(sizes_d), p(wds_d), p(wd_),
           p(gd), p(md), None, F32, C.c_float(0.1), None, C.c_float(0.9), C.c_float(1 / 256.), C.c_float(-1.0),
           stream())
    torch.cuda.synchronize()
    for o, s in zip(offs, sizes):
        assert rel_err(wd_.cpu().numpy()[o:o + s], wr[o:o + s]) < 1e-6
        assert rel_err(md.cpu().numpy()[o:o + s], mr[o:o + s]) < 1e-5


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_sgd_update_pack(gpu, dtype):
    """rn_sgd_mom_update_pack = rn_sgd_mom_update followed by rn_conv_weight_pack of every dense
    conv / FC tensor, bit for bit (padding entries of the copies untouched)."""
    rng = np.random.default_rng(11)
    # (name, conv desc args or None): a 3x3 conv with padded channels, the stem (c=8 over 3), an FC
    # with a ragged output count, a BN gamma
    specs = [("c3_weight", (dtype, 2, 24, 5, 5, 40, 3, 3, 1, 1)), ("g_gamma", None),
             ("stem_weight", (dtype, 2, 8, 9, 9, 16, 7, 7, 2, 3, 3)), ("fc_weight", (dtype, 2, 64, 1, 1, 1000, 1, 1, 1, 0))]
    descs, sizes = [], []
    for nm, a in specs:
        if a is None:
            descs.append(None)
            sizes.append(40)
            continue
        d = conv_desc(*a[:10], c_real=a[10] if len(a) > 10 else None)
        descs.append(d)
        sizes.append(int(d.k * d.r * d.s * d.c_real))
    offs = np.cumsum([0] + [((s + 3) // 4) * 4 for s in sizes])[:-1]
    total = int(offs[-1] + sizes[-1] + 4)
    t = lambda a, dt=torch.float32: torch.tensor(a, dtype=dt, device=gpu)
    w, g, m = (rng.standard_normal(total).astype(np.float32) for _ in range(3))
    wd = np.array([1e-4, 0.0, 1e-4, 1e-4], dtype=np.float32)
    offs_d, sizes_d, wds_d = t(offs, torch.int64), t(sizes, torch.int64), t(wd)
    tab = np.zeros(len(specs), dtype=[("krsc", "<u8"), ("crsk", "<u8"), ("k", "<i4"), ("rs", "<i4"),
                                      ("creal", "<i4"), ("c", "<i4"), ("kpad", "<i4"), ("pad", "<i4")])
    outs = []
    for i, d in enumerate(descs):
        if d is None:
            outs.append(None)
            continue
        # copies prefilled with a sentinel: the padding must keep it
        pair = [torch.full((int(L.load().rn_conv_pack_numel(C.byref(d), j)),), 7.0, dtype=tdt(dtype), device=gpu)
                for j in (0, 1)]
        ref = [x.clone() for x in pair]
        outs.append((pair, ref))
        tab[i] = (pair[0].data_ptr(), pair[1].data_ptr(), d.k, d.r * d.s, d.c_real, d.c, d.k_pad, 0)
    tab_d = torch.from_numpy(tab.view(np.uint8).copy()).to(gpu)
    work = np.zeros((4096, 4), dtype=np.int32)
    nwork = L.load().rn_sgd_pack_work(len(specs), np.asarray(sizes, np.int64).ctypes.data_as(C.c_void_p),
                                      tab.ctypes.data_as(C.c_void_p), work.ctypes.data_as(C.c_void_p), 4096)
    assert nwork > 0
    work_d = torch.from_numpy(work[:nwork].copy()).to(gpu)
    args = lambda wv, mv: (p(offs_d), p(sizes_d), p(wds_d), p(wv), p(gd), p(mv))
    gd = t(g)
    w1, m1, w2, m2 = t(w), t(m), t(w), t(m)
    sc = (C.c_float(0.05), None, C.c_float(0.9), C.c_float(1 / 128.), C.c_float(-1.0), stream())
    L.call("rn_sgd_mom_update", len(specs), *args(w1, m1), None, F32, *sc)
    for i, d in enumerate(descs):
        if d is not None:
            ref = outs[i][1]
            L.call("rn_conv_weight_pack", C.byref(d), C.c_void_p(w1.data_ptr() + 4 * int(offs[i])), p(ref[0]),
                   p(ref[1]), stream())
    L.call("rn_sgd_mom_update_pack", len(specs), *args(w2, m2), p(tab_d), p(work_d), nwork, dtype, *sc)
    torch.cuda.synchronize()
    assert torch.equal(w1, w2) and torch.equal(m1, m2)
    for o in outs:
        if o is None:
            continue
        pair, ref = o
        # reference pack zero-fills the padding; the fused kernel leaves the sentinel there
        for a, b in zip(pair, ref):
            pad = b == 0
            assert torch.equal(a[~pad], b[~pad])
            assert bool((a[pad] == 7.0).all())


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_quant_int8(gpu, dtype):
    rng = np.random.default_rng(10)
    n = 4096
    w = rng.standard_normal(n)
    if dtype == BF16:
        w = bf16_round(w)
    wq_ref, _ = ops.quant_int8_weight(w)
    xd = torch.tensor(w, dtype=tdt(dtype), device=gpu)
    out = torch.zeros_like(xd)
    ws = torch.zeros(4096, dtype=torch.float32, device=gpu)
    L.call("rn_quant_int8_fwd", dtype, n, p(xd), p(out), None, 1, 1, C.c_float(0.99), 1, 8, p(ws), stream())
    torch.cuda.synchronize()
    tol = 1e-6 if dtype == F32 else 1e-2
    assert rel_err(out.float().cpu().numpy(), wq_ref) < tol
    # activation: EMA state, clip and masked STE
    x = rng.standard_normal(n) * 3
    if dtype == BF16:
        x = bf16_round(x)
    mm = torch.tensor([2.0], dtype=torch.float32, device=gpu)
    xq_ref, mm_ref = ops.quant_int8_act(x, 2.0, True, False)
    xd = torch.tensor(x, dtype=tdt(dtype), device=gpu)
    L.call("rn_quant_int8_fwd", dtype, n, p(xd), p(out), p(mm), 0, 1, C.c_float(0.99), 0, 8, p(ws), stream())
    dy = rng.standard_normal(n)
    dx = torch.zeros_like(xd)
    L.call("rn_quant_int8_bwd", dtype, n, p(xd), p(torch.tensor(dy, dtype=tdt(dtype), device=gpu)), p(dx), p(mm), 0,
           None, stream())
    torch.cuda.synchronize()
    assert abs(mm.item() - mm_ref) < 1e-5 * abs(mm_ref)
    assert rel_err(out.float().cpu().numpy(), xq_ref) < tol
    dyr = bf16_round(dy) if dtype == BF16 else dy
    assert rel_err(dx.float().cpu().numpy(), ops.quant_int8_act_bwd(dyr, x, mm_ref)) < tol


GCONV_CASES = [
    # n, c, h, w, k, r, stride, pad, groups -- ResNeXt-50 32x4d conv2 shapes at small spatial size
    (2, 128, 9, 9, 128, 3, 1, 1, 32),   # 4 channels per group
    (2, 256, 10, 10, 256, 3, 2, 1, 32),  # 8 per group, stride 2 (dgrad parity classes)
    (2, 512, 6, 6, 512, 3, 1, 1, 32),   # 16 per group
    (1, 1024, 5, 5, 1024, 3, 2, 1, 32),  # 32 per group
    (2, 128, 6, 6, 256, 1, 1, 0, 2),    # 64 -> 128 per group (block inside one group)
]


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", GCONV_CASES)
def test_grouped_conv(gpu, dtype, case):
    """Grouped convolution (symbol/resnext.py:23-25) fwd / dgrad / wgrad vs the oracle."""
    n, c, h, w, k, r, st, pd, g = case
    rng = np.random.default_rng(11)
    x = rng.standard_normal((n, c, h, w))
    wt = rng.standard_normal((k, c // g, r, r)) / np.sqrt(c // g * r * r)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = rng.standard_normal((n, k, P, Q))
    if dtype == BF16:
        x, wt, dy = bf16_round(x), bf16_round(wt), bf16_round(dy)
    y_ref = ops.conv2d_fwd(x, wt, (st, st), (pd, pd), g)
    dx_ref, dw_ref = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd), g)
    d = L.ConvDesc(dtype=dtype, n=n, h=h, w=w, c=c, c_real=c, k=k, k_pad=k, r=r, s=r, stride_h=st, stride_w=st,
                   pad_h=pd, pad_w=pd, groups=g)
    L.call("rn_conv_desc_init", C.byref(d))
    lib = L.load()
    wk = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 0), dtype=tdt(dtype), device=gpu)
    wc = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 1), dtype=tdt(dtype), device=gpu)
    master = _master_krsc(wt, gpu)
    assert master.numel() == lib.rn_conv_weight_numel(C.byref(d))
    L.call("rn_conv_weight_pack", C.byref(d), p(master), p(wk), p(wc), stream())
    xd, dyd = to_nhwc(x, dtype, gpu), to_nhwc(dy, dtype, gpu)
    y = torch.zeros((n, P, Q, k), dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(y), dtype, None, None, stream())
    dx = torch.zeros((n, h, w, c), dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(dx), None, stream())
    dw = torch.zeros(master.numel(), dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dyd), p(dw), stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(y, k), y_ref) < TOL[dtype]
    assert rel_err(from_nhwc(dx, c), dx_ref) < TOL[dtype]
    dw_h = dw.cpu().numpy().reshape(k, r, r, c // g).transpose(0, 3, 1, 2)
    assert rel_err(dw_h, dw_ref) < (TOL[dtype] if dtype == F32 else 5e-3)


@pytest.mark.parametrize("case", [
    (2, 128, 9, 9, 128, 3, 1, 1, 32),     # 4 per group (stage 1), fwd + dgrad direct
    (3, 128, 15, 13, 128, 3, 1, 1, 32),   # ragged rows (13 = 3 blocks of 4 pixels + 1)
    (2, 256, 10, 10, 256, 3, 2, 1, 32),   # 8 per group, stride 2: direct forward, block-diagonal dgrad
    (2, 256, 7, 11, 256, 3, 1, 1, 32),    # 8 per group, stride 1
    (2, 128, 12, 12, 128, 3, 2, 1, 32),   # 4 per group, stride 2 (the transposed stride-2 data gradient too)
    (2, 128, 11, 13, 128, 3, 2, 1, 32),   # stride 2, odd input sizes
    (2, 512, 6, 7, 512, 3, 1, 1, 32),     # 16 per group (stage 3)
    (2, 512, 9, 9, 512, 3, 2, 1, 32),     # 16 per group, stride 2
    (1, 64, 5, 5, 64, 3, 1, 1, 8),        # 8 per group, fewer channels than a wave has lanes
])
def test_grouped_conv_direct(gpu, case):
    """The direct grouped kernels (rn_set_tuning 15 = 0: v_dot2_f32_bf16 over 16-byte channel chunks,
    compact weight copies; 4 per group, and 8 per group at stride 2 forward) vs the oracle and vs the
    block-diagonal 64-column tiles (15 = 1): forward and data gradient with an add_src (the residual /
    gradient accumulation operand), both within one bf16 rounding of the fp64 values. (8 per group at
    stride 1 and 16 per group run the block-diagonal tiles either way.)"""
    n, c, h, w, k, r, st, pd, g = case
    rng = np.random.default_rng(13)
    x = bf16_round(rng.standard_normal((n, c, h, w)))
    wt = bf16_round(rng.standard_normal((k, c // g, r, r)) / np.sqrt(c // g * r * r))
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = bf16_round(rng.standard_normal((n, k, P, Q)))
    ya = bf16_round(rng.standard_normal((n, k, P, Q)))
    xa = bf16_round(rng.standard_normal((n, c, h, w)))
    d = L.ConvDesc(dtype=BF16, n=n, h=h, w=w, c=c, c_real=c, k=k, k_pad=k, r=r, s=r, stride_h=st, stride_w=st,
                   pad_h=pd, pad_w=pd, groups=g)
    L.call("rn_conv_desc_init", C.byref(d))
    lib = L.load()
    master = _master_krsc(wt, gpu)
    xd, dyd, yad, xad = (to_nhwc(v, BF16, gpu) for v in (x, dy, ya, xa))
    outs = {}
    for mode in (0, 1):
        L.call("rn_set_tuning", 15, mode)
        try:
            L.call("rn_conv_desc_init", C.byref(d))  # (the layout is recorded in the descriptor at init)
            assert d.grouped_direct == (1 if mode == 0 and (c // g == 4 or (c // g == 8 and st == 2)) else 0)
            if mode == 0:
                if c // g == 4 or (c // g == 8 and st == 2):  # the direct forward: compact [c/8][9][8][G] copy
                    assert lib.rn_conv_pack_numel(C.byref(d), 0) == c * 9 * (c // g)
                    assert lib.rn_conv_tile(C.byref(d), 0) == 0
            wk = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 0), dtype=torch.bfloat16, device=gpu)
            wc = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 1), dtype=torch.bfloat16, device=gpu)
            L.call("rn_conv_weight_pack", C.byref(d), p(master), p(wk), p(wc), stream())
            y = torch.zeros((n, P, Q, k), dtype=torch.bfloat16, device=gpu)
            dx = torch.zeros((n, h, w, c), dtype=torch.bfloat16, device=gpu)
            L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(y), BF16, p(yad), None, stream())
            L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(dx), p(xad), stream())
            torch.cuda.synchronize()
        finally:
            L.call("rn_set_tuning", 15, 0)
        outs[mode] = (from_nhwc(y, k), from_nhwc(dx, c))
    y_ref = ops.conv2d_fwd(x, wt, (st, st), (pd, pd), g) + ya
    dx_ref = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd), g)[0] + xa
    for mode in (0, 1):
        assert np.abs(outs[mode][0] - y_ref).max() <= 2 ** -7 * np.abs(y_ref).max(), mode
        assert np.abs(outs[mode][1] - dx_ref).max() <= 2 ** -7 * np.abs(dx_ref).max(), mode
    assert rel_err(outs[0][0], outs[1][0]) < 4e-3 and rel_err(outs[0][1], outs[1][1]) < 4e-3


GBN_CASES = [
    # n, c, h, w, stride, groups: ResNeXt-50 32x4d conv2 (3x3, pad 1) at small spatial size
    (2, 128, 9, 9, 1, 32),     # 4 per group: direct data gradient (stride 1)
    (3, 128, 15, 13, 1, 32),   # ragged pixel lanes
    (2, 128, 12, 12, 2, 32),   # 4 per group, stride 2: the transposed stride-2 direct data gradient
    (2, 256, 11, 13, 2, 32),   # 8 per group, stride 2: direct (transposed) data gradient
    (2, 256, 7, 11, 1, 32),    # 8 per group, stride 1: block-diagonal tile (GD)
    (2, 512, 6, 7, 1, 32),     # 16 per group: GD tile
    (1, 1024, 5, 5, 2, 32),    # 32 per group, stride 2: GD tile over parity classes
]


@pytest.fixture(params=[0, 2], ids=["gd_auto", "gd_s2"])
def gd_tune(request):
    """rn_set_tuning 13 (block-diagonal grouped tile): 0 auto; 2 also the stride-2 data gradients."""
    L.call("rn_set_tuning", 13, request.param)
    yield request.param
    L.call("rn_set_tuning", 13, 0)


@pytest.mark.parametrize("case", GBN_CASES)
def test_grouped_dgrad_bn_backward_fusion(gpu, case, gd_tune):
    """The grouped data gradients carrying the BatchNorm(+ReLU) backward reduction of the BN that
    produced their input (rn_conv_bwd_data_bnred on the direct kernels and on the block-diagonal
    256x64 tile) + rn_bn_bwd_part == the oracle's grouped dgrad followed by the BN+ReLU backward
    (symbol/resnext.py:20-25: bn1 -> relu -> grouped conv2); dx as stored is the unfused call's, bit
    for bit."""
    n, c, h, w, st, g = case
    k, r, pd = c, 3, 1
    rng = np.random.default_rng(21)
    xb = bf16_round(rng.standard_normal((n, c, h, w)) * 1.5 + 0.3)   # BN input
    gamma, beta = rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.2
    a_ref, cache = ops.bn_train_fwd(xb, gamma, beta, 1e-5, False)
    act = ops.relu_fwd(a_ref)
    wt = bf16_round(rng.standard_normal((k, c // g, r, r)) / np.sqrt(c // g * r * r))
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = bf16_round(rng.standard_normal((n, k, P, Q)))
    prev = bf16_round(rng.standard_normal((n, c, h, w)) * 0.5)
    dact_ref = ops.conv2d_bwd(act, wt, dy, (st, st), (pd, pd), g)[0] + prev
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd, groups=g)
    lib = L.load()
    direct = d.grouped_direct == 1
    assert direct == (c // g == 4 or (c // g == 8 and st == 2))
    # (the stride-2 block-diagonal data gradient: 4-tap parity classes, the 128-row kernel by default)
    assert direct or lib.rn_conv_tile(C.byref(d), 1) == (0 if st == 2 and gd_tune != 2 else 64)
    wc = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 1), dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), None, p(wc), stream())
    bd = L.BNDesc(dtype=BF16, m=n * h * w, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
    sm, si, sc, sh = [torch.zeros(c, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    xbd = to_nhwc(xb, BF16, gpu)
    L.call("rn_bn_fwd_train", C.byref(bd), p(xbd), None, p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc), p(sh),
           p(ws), stream())
    dyd = to_nhwc(dy, BF16, gpu)
    dact = to_nhwc(prev, BF16, gpu)                      # accumulated in place (add_src = out)
    plain = to_nhwc(prev, BF16, gpu)
    nrb = lib.rn_conv_bnred_blocks(C.byref(d))
    part = torch.full((nrb * c * 2,), float("nan"), dtype=torch.float32, device=gpu)  # every slot written
    L.call("rn_conv_bwd_data_bnred", C.byref(d), p(dyd), p(wc), p(dact), p(dact), p(xbd), p(sm), p(sc), p(sh), 1,
           p(part), stream())
    L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(plain), p(plain), stream())
    dx = torch.zeros_like(xbd)
    dg, db = torch.zeros(c, dtype=torch.float32, device=gpu), torch.zeros(c, dtype=torch.float32, device=gpu)
    L.call("rn_bn_bwd_part", C.byref(bd), p(part), nrb, p(xbd), p(dact), p(dx), None, p(g_d), p(sm), p(si), p(sc),
           p(sh), p(dg), p(db), p(ws), stream())
    torch.cuda.synchronize()
    assert torch.equal(dact, plain)
    assert not torch.isnan(part).any()
    assert rel_err(from_nhwc(dact, c), dact_ref) < TOL[BF16]
    dz = ops.relu_bwd(from_nhwc(dact, c), act)           # from the stored gradient, as the kernel reads it
    dx_ref, dg_ref, db_ref = ops.bn_train_bwd(dz, cache, False)
    assert rel_err(db.cpu().numpy(), db_ref) < 1e-4
    assert rel_err(dg.cpu().numpy(), dg_ref) < 1e-4
    assert rel_err(from_nhwc(dx, c), dx_ref) < 3e-2


@pytest.mark.parametrize("case", [c for c in GBN_CASES if c[1] // c[5] >= 8 and not (c[1] // c[5] == 8 and c[4] == 2)])
def test_grouped_conv_bnstats_epilogue(gpu, case):
    """BatchNorm statistics from the block-diagonal 256x64 tile's epilogue (rn_conv_fwd_bnstats on a
    grouped conv, the ResNeXt bn2 input) merged by rn_bn_fwd_train_part == a BatchNorm over the stored
    grouped conv output."""
    n, c, h, w, st, g = case
    k, r, pd = c, 3, 1
    rng = np.random.default_rng(22)
    x = bf16_round(rng.standard_normal((n, c, h, w)))
    wt = bf16_round(rng.standard_normal((k, c // g, r, r)) / np.sqrt(c // g * r * r))
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    res = bf16_round(rng.standard_normal((n, k, P, Q)) + 3.0)  # offset mean: exercises the pivots
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd, groups=g)
    lib = L.load()
    assert d.grouped_direct == 0 and lib.rn_conv_tile(C.byref(d), 0) == 64
    wk = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 0), dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), None, stream())
    y = torch.zeros((n, P, Q, k), dtype=torch.bfloat16, device=gpu)
    plain = torch.zeros_like(y)
    nblk = lib.rn_conv_bnstats_blocks(C.byref(d))
    part = torch.zeros(nblk * 3 * k, dtype=torch.float32, device=gpu)
    xd, rd = to_nhwc(x, BF16, gpu), to_nhwc(res, BF16, gpu)
    L.call("rn_conv_fwd_bnstats", C.byref(d), p(xd), p(wk), p(y), BF16, p(rd), None, p(part), stream())
    L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(plain), BF16, p(rd), None, stream())
    torch.cuda.synchronize()
    assert torch.equal(y, plain)
    conv_out = from_nhwc(y, k)
    assert rel_err(conv_out, ops.conv2d_fwd(x, wt, (st, st), (pd, pd), g) + res) < TOL[BF16]
    gamma, beta = rng.uniform(0.5, 1.5, k), rng.standard_normal(k) * 0.1
    _, cache = ops.bn_train_fwd(conv_out, gamma, beta, 1e-5, False)
    mm_ref, mv_ref = ops.bn_moving_update(np.zeros(k), np.ones(k), cache[3], cache[4], 0.9)
    bd = L.BNDesc(dtype=BF16, m=n * P * Q, c=k, c_real=k, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(k)), f(np.ones(k))
    sm, si, sc, sh = [torch.zeros(k, dtype=torch.float32, device=gpu) for _ in range(4)]
    yb = torch.zeros_like(y)
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    L.call("rn_bn_fwd_train_part", C.byref(bd), p(part), nblk, lib.rn_conv_bn_part_rows(C.byref(d), 0), k, p(y),
           p(yb), p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc), p(sh), p(ws), stream())
    torch.cuda.synchronize()
    assert rel_err(sm.cpu().numpy(), cache[3]) < 1e-6
    assert rel_err(mv.cpu().numpy(), mv_ref) < 1e-5
    assert rel_err(mm.cpu().numpy(), mm_ref) < 1e-5


@pytest.mark.parametrize("nblk,rows,c", [(56, 224, 512), (224, 224, 256), (224, 224, 1024), (1, 224, 64),
                                          (65, 128, 72), (256, 64, 136), (257, 64, 64), (3584, 224, 64)])
def test_bn_fwd_merge_finalize_one_launch(gpu, nblk, rows, c):
    """rn_bn_fwd_train_part merges the conv epilogue's BatchNorm partials and finalizes in ONE launch where
    they form at most 4 merge groups (nblk <= 256): every output (scale, shift, saved mean / invstd,
    moving statistics) bit for bit that of the two-launch merge + finalize (rn_set_tuning 24 = 1), on
    partials with an offset mean and ragged last blocks; beyond 4 groups the call takes the two launches."""
    lib = L.load()
    rng = np.random.default_rng(31 + nblk)
    m = nblk * rows - rows // 3  # (a ragged last block)
    ld = c + 8
    part = np.zeros((nblk, 3, ld), np.float32)
    nb = np.minimum(rows, m - np.arange(nblk) * rows).astype(np.float64)
    piv = rng.standard_normal((nblk, c)) * 0.5 + 3.0
    part[:, 2, :c] = piv
    part[:, 0, :c] = rng.standard_normal((nblk, c)) * np.sqrt(nb)[:, None]
    part[:, 1, :c] = (rng.uniform(0.5, 1.5, (nblk, c)) * nb[:, None]).astype(np.float32)
    bd = L.BNDesc(dtype=BF16, m=m, c=c, c_real=c - (8 if c % 64 else 0), eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    pd = f(part.reshape(-1))
    gamma, beta = f(rng.uniform(0.5, 1.5, c)), f(rng.standard_normal(c) * 0.1)
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16 + nblk * 8 * c, dtype=torch.float32, device=gpu)
    outs = []
    for mode in (0, 1):
        L.call("rn_set_tuning", 24, mode)
        mm, mv = f(rng.standard_normal(c) * 0 + 0.25), f(np.ones(c))
        sm, si, sc, sh = [torch.full((c,), 7.0, dtype=torch.float32, device=gpu) for _ in range(4)]
        L.call("rn_bn_fwd_train_part", C.byref(bd), p(pd), nblk, rows, ld, None, None, p(gamma), p(beta), p(mm),
               p(mv), p(sm), p(si), p(sc), p(sh), p(ws), stream())
        torch.cuda.synchronize()
        outs.append([t.clone() for t in (sm, si, sc, sh, mm, mv)])
    L.call("rn_set_tuning", 24, 0)
    for a, b in zip(*outs):
        assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    # and the merged mean is the batch mean of the partials' rows
    mean = (piv + part[:, 0, :c] / nb[:, None]) * nb[:, None]
    ref = mean.sum(0) / nb.sum()
    nreal = bd.c_real
    assert np.abs(outs[0][0].cpu().numpy()[:nreal] - ref[:nreal]).max() < 1e-4


@pytest.mark.parametrize("dtype", [F32, BF16])
def test_weight_pack_multi(gpu, dtype):
    """rn_conv_weight_pack_multi writes exactly the bytes of one rn_conv_weight_pack per layer: the
    direct (compact) and block-diagonal grouped copies batched 32 to a launch, dense layers and a NULL
    copy passed through. 40 grouped layers -> two launches."""
    geoms = [(128, 3, 1, 32), (256, 3, 2, 32), (256, 3, 1, 32), (512, 3, 1, 32), (1024, 3, 2, 32),
             (128, 1, 1, 2), (64, 3, 1, 8)] * 6
    geoms += [(64, 1, 1, 1), (96, 3, 1, 1)]  # dense
    lib = L.load()
    rng = np.random.default_rng(17)
    ds, ms, refs, outs = [], [], [], []
    for i, (c, r, st, g) in enumerate(geoms):
        d = L.ConvDesc(dtype=dtype, n=2, h=8, w=8, c=c, c_real=c, k=c, k_pad=c, r=r, s=r, stride_h=st,
                       stride_w=st, pad_h=r // 2, pad_w=r // 2, groups=g)
        L.call("rn_conv_desc_init", C.byref(d))
        wt = rng.standard_normal((c, c // g, r, r)).astype(np.float32)
        ms.append(_master_krsc(wt, gpu))
        ds.append(d)
        pair = []
        for which in (0, 1):
            nel = lib.rn_conv_pack_numel(C.byref(d), which)
            pair.append([torch.full((nel,), 7.0, dtype=tdt(dtype), device=gpu) for _ in range(2)])
        if i == 3:  # a layer without its data-gradient copy
            pair[1] = [None, None]
        L.call("rn_conv_weight_pack", C.byref(d), p(ms[-1]), p(pair[0][0]), p(pair[1][0]), stream())
        refs.append((pair[0][0], pair[1][0]))
        outs.append((pair[0][1], pair[1][1]))
    n = len(ds)
    vp = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    L.call("rn_conv_weight_pack_multi", (L.ConvDesc * n)(*ds), (C.c_void_p * n)(*[m.data_ptr() for m in ms]),
           (C.c_void_p * n)(*[vp(o[0]) for o in outs]), (C.c_void_p * n)(*[vp(o[1]) for o in outs]), n, stream())
    torch.cuda.synchronize()
    for i in range(n):
        for a, b in zip(refs[i], outs[i]):
            if a is None:
                assert b is None
                continue
            assert torch.equal(a.view(torch.int16) if dtype == BF16 else a.view(torch.int32),
                               b.view(torch.int16) if dtype == BF16 else b.view(torch.int32)), (i, geoms[i])


def _im2col_ref(xq, r, st, pd, kc):
    n, c, h, w = xq.shape
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    xp = np.pad(xq, ((0, 0), (0, 0), (pd, pd), (pd, pd)))
    cols = np.zeros((n, P, Q, kc))
    for rr in range(r):
        for ss in range(r):
            patch = xp[:, :, rr:rr + st * P:st, ss:ss + st * Q:st]  # n, c, P, Q
            base = (rr * r + ss) * c
            cols[..., base:base + c] = patch.transpose(0, 2, 3, 1)
    return cols.reshape(n * P * Q, kc)


@pytest.mark.parametrize("h,w", [(20, 18), (19, 17)])  # (19 x 17: a ragged tail after the 16-byte chunks)
def test_stem_quant(gpu, h, w):
    """conv0 of resnet_int8 (symbol/resnet_int8.py:96-98): Quantization_int8(bn_data(x)) folded into
    the stem im2col, and the STE-masked bn_data beta gradient (clip_grad_quantization_int8.py)."""
    n, c, k, r, st, pd, kc = 2, 3, 16, 7, 2, 3, 160
    rng = np.random.default_rng(12)
    x1 = rng.uniform(-1, 1, (n, c, h, w)).astype(np.float32)
    x2 = (x1 * 1.5).astype(np.float32)
    scale = np.array([1.5, 0.5, 2.0], dtype=np.float32)
    shift = np.array([0.1, -0.2, 0.3], dtype=np.float32)
    aff = lambda x: x * scale[None, :, None, None] + shift[None, :, None, None]
    t1 = np.abs(aff(x1)).max()
    t2 = np.float32(t1 * np.float32(0.99) + np.abs(aff(x2)).max() * np.float32(0.01))
    xq_ref, _ = ops.quant_int8_act(aff(x2).astype(np.float64), float(t2), False, False)
    mask = (aff(x2) > -t2) & (aff(x2) < t2)
    assert (~mask).sum() > 10  # the EMA threshold clips part of the second batch
    wq = ops.quant_int8_weight(rng.standard_normal((k, c, r, r)) * 0.1)[0]
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = rng.standard_normal((n, k, P, Q))
    dx_ref, _ = ops.conv2d_bwd(xq_ref, wq, dy, (st, st), (pd, pd))
    dbeta_ref = (dx_ref * mask).sum(axis=(0, 2, 3))

    dfull = conv_desc(F32, n, 8, h, w, k, r, r, st, pd, c_real=c)
    sc = torch.tensor(scale, device=gpu)
    sh = torch.tensor(shift, device=gpu)
    minmax = torch.zeros(1, dtype=torch.float32, device=gpu)
    ws = torch.zeros(16, dtype=torch.float32, device=gpu)
    cols = torch.zeros(n * P * Q * kc, dtype=torch.float32, device=gpu)
    for x, first in ((x1, 1), (x2, 0)):
        xd = torch.from_numpy(x).to(gpu)
        L.call("rn_im2col_nchw_quant", C.byref(dfull), p(xd), p(sc), p(sh), p(minmax), 1, C.c_float(0.99), first, 8,
               p(ws), p(cols), kc, stream())
    torch.cuda.synchronize()
    assert abs(minmax.item() - float(t2)) <= 1e-6 * float(t2)
    got = cols.cpu().numpy().reshape(n * P * Q, kc)
    assert rel_err(got, _im2col_ref(xq_ref, r, st, pd, kc)) < 1e-6
    master = _master_krsc(wq, gpu)
    dyd = to_nhwc(dy, F32, gpu)
    dbeta = torch.zeros(c, dtype=torch.float32, device=gpu)
    sws = torch.zeros(P * Q * pad8(k) + P * r * k + k * r * r, dtype=torch.float32, device=gpu)
    L.call("rn_stem_shift_grad", C.byref(dfull), p(dyd), p(master), p(dbeta), p(sws), stream())
    L.call("rn_stem_quant_clip_grad", C.byref(dfull), p(xd), p(sc), p(sh), p(minmax), p(dyd), p(master), p(dbeta),
           stream())
    torch.cuda.synchronize()
    assert rel_err(dbeta.cpu().numpy(), dbeta_ref) < 1e-4


@pytest.mark.parametrize("n,h,w,k", [(2, 20, 18, 64), (3, 32, 30, 64), (2, 19, 17, 32)])
def test_stem_clip_as_weight_gradient(gpu, n, h, w, k):
    """The int8 stem's clip gradient through its weight gradient (rn_stem_clip_mask / _wgrad / _dbeta:
    the clip masks in the NHWC-8 image's free channels, their weight gradient dotted with the weights)
    == rn_stem_quant_clip_grad's gather, and the real channels' dW == rn_conv_bwd_filter_ws on the
    unmasked image; the masks themselves vs numpy."""
    c, r, st, pd = 3, 7, 2, 3
    rng = np.random.default_rng(46)
    x = rng.uniform(-1, 1, (n, c, h, w)).astype(np.float32)
    scale = np.array([1.5, 0.5, 2.0], dtype=np.float32)
    shift = np.array([0.1, -0.2, 0.3], dtype=np.float32)
    t = np.float32(1.1)                                  # clips part of the affine image
    aff = x * scale[None, :, None, None] + shift[None, :, None, None]
    mask_ref = ~((aff > -t) & (aff < t))
    assert mask_ref.sum() > 20
    dfull = conv_desc(BF16, n, 8, h, w, k, r, r, st, pd, c_real=c)
    lib = L.load()
    assert lib.rn_stem_clip_supported(C.byref(dfull)) == 1
    x8h = np.zeros((n, h, w, 8), dtype=np.float32)
    x8h[..., :c] = bf16_round(np.clip(aff, -t, t)).transpose(0, 2, 3, 1)   # (a stand-in for the quantized input)
    x8 = torch.tensor(x8h, dtype=torch.bfloat16, device=gpu).contiguous()
    x8_plain = x8.clone()
    P, Q = dfull.p, dfull.q
    dyd = to_nhwc(bf16_round(rng.standard_normal((n, k, P, Q))), BF16, gpu)
    wq = ops.quant_int8_weight(rng.standard_normal((k, c, r, r)) * 0.1)[0]
    master = _master_krsc(wq, gpu)
    xd = torch.from_numpy(x).to(gpu)
    sc, sh = torch.tensor(scale, device=gpu), torch.tensor(shift, device=gpu)
    minmax = torch.tensor([float(t)], dtype=torch.float32, device=gpu)
    sws = torch.zeros(P * Q * pad8(k) + P * r * k + k * r * r, dtype=torch.float32, device=gpu)
    # the gather route
    wsb = max(lib.rn_conv_wgrad_ws_bytes(C.byref(dfull)), lib.rn_stem_clip_wgrad_ws_bytes(C.byref(dfull)), 16)
    ws = torch.zeros(wsb // 4 + 4, dtype=torch.float32, device=gpu)
    dw_ref = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter_ws", C.byref(dfull), p(x8_plain), p(dyd), p(dw_ref), p(ws), wsb, stream())
    dbeta_ref = torch.zeros(c, dtype=torch.float32, device=gpu)
    L.call("rn_stem_shift_grad", C.byref(dfull), p(dyd), p(master), p(dbeta_ref), p(sws), stream())
    L.call("rn_stem_quant_clip_grad", C.byref(dfull), p(xd), p(sc), p(sh), p(minmax), p(dyd), p(master),
           p(dbeta_ref), stream())
    # the weight-gradient route
    L.call("rn_stem_clip_mask", C.byref(dfull), p(xd), p(sc), p(sh), p(minmax), p(x8), stream())
    dw = torch.full((k * r * r * c,), 0.25, dtype=torch.float32, device=gpu)  # (accumulated into)
    ext = torch.full((k * r * r * 2 * c,), float("nan"), dtype=torch.float32, device=gpu)
    L.call("rn_stem_clip_wgrad", C.byref(dfull), p(x8), p(dyd), p(dw), p(ext), p(ws), wsb, stream())
    dbeta = torch.zeros(c, dtype=torch.float32, device=gpu)
    L.call("rn_stem_shift_grad", C.byref(dfull), p(dyd), p(master), p(dbeta), p(sws), stream())
    L.call("rn_stem_clip_dbeta", C.byref(dfull), p(ext), p(master), p(dbeta), stream())
    torch.cuda.synchronize()
    x8f = x8.float().cpu().numpy()
    assert np.array_equal(x8f[..., :c], x8h[..., :c]) and not x8f[..., 2 * c:].any()
    assert np.array_equal(x8f[..., c:2 * c] == 1.0, mask_ref.transpose(0, 2, 3, 1))
    assert rel_err(dw.cpu().numpy() - 0.25, dw_ref.cpu().numpy()) < 1e-5
    assert rel_err(dbeta.cpu().numpy(), dbeta_ref.cpu().numpy()) < 1e-4


@pytest.fixture(params=[(0, 0, 512), (0, 0, 8), (1, 0, 0), (1, 1, 512)],
                ids=["rows224", "rows224_persist8", "rows256_mfma32", "rows256_mfma16"])
def tile_variant(request):
    """igemm 256-row-family variants: rn_set_tuning 9 (224-row tiles on/off) x 8 (MFMA shape) x 10
    (persistent grid: 8 workgroups walk every tile of these small grids; 0 = one tile each)."""
    rows, mfma, persist = request.param
    L.call("rn_set_tuning", 9, rows)
    L.call("rn_set_tuning", 8, mfma)
    L.call("rn_set_tuning", 10, persist)
    yield request.param
    L.call("rn_set_tuning", 9, 0)
    L.call("rn_set_tuning", 8, 0)
    L.call("rn_set_tuning", 10, 512)


@pytest.fixture(params=[0, 2, "w4"], ids=["auto", "big256", "w4"])
def big_tiles(request):
    """rn_set_tuning 4 (igemm 256-row tiles): automatic choice, or 256x256 forced where eligible;
    w4: rn_set_tuning 11 = 2, the 4-wave one-buffer 224x128 tile on every 1x1 pad-0 conv."""
    if request.param == "w4":
        L.call("rn_set_tuning", 11, 2)
    else:
        L.call("rn_set_tuning", 4, request.param)
    yield request.param
    L.call("rn_set_tuning", 4, 0)
    L.call("rn_set_tuning", 11, 0)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", [(3, 32, 13, 11, 48, 3, 2, 1), (2, 64, 14, 14, 256, 1, 1, 0), (2, 16, 9, 9, 64, 1, 1, 0),
                                  (3, 128, 20, 20, 256, 3, 1, 1)])
def test_conv_bnstats_epilogue(gpu, dtype, case, big_tiles, tile_variant):
    """BatchNorm statistics emitted by the conv epilogue (rn_conv_fwd_bnstats, with the fused
    residual add) and merged by rn_bn_fwd_train_part == a BatchNorm over the stored conv output."""
    n, c, h, w, k, r, st, pd = case
    x, wt = _conv_data(case, 13)
    if dtype == BF16:
        x, wt = bf16_round(x), bf16_round(wt)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    res = np.random.default_rng(14).standard_normal((n, k, P, Q)) + 3.0  # offset mean: exercises the pivots
    if dtype == BF16:
        res = bf16_round(res)
    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd)
    xd = to_nhwc(x, dtype, gpu)
    wk = torch.zeros(k * r * r * d.c, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), None, stream())
    y = torch.zeros((n, P, Q, d.k_pad), dtype=tdt(dtype), device=gpu)
    lib = L.load()
    nblk = lib.rn_conv_bnstats_blocks(C.byref(d))
    part = torch.zeros(nblk * 3 * d.k_pad, dtype=torch.float32, device=gpu)
    rd = to_nhwc(res, dtype, gpu)
    L.call("rn_conv_fwd_bnstats", C.byref(d), p(xd), p(wk), p(y), dtype, p(rd), None, p(part), stream())
    torch.cuda.synchronize()
    conv_out = from_nhwc(y, k)  # the stored (rounded) values the statistics must describe
    gamma = np.random.default_rng(15).uniform(0.5, 1.5, k)
    beta = np.random.default_rng(16).standard_normal(k) * 0.1
    y_ref, cache = ops.bn_train_fwd(conv_out, gamma, beta, 1e-5, False)
    mm_start = np.zeros(k)
    mm_ref, mv_ref = ops.bn_moving_update(mm_start, np.ones(k), cache[3], cache[4], 0.9)
    bd = L.BNDesc(dtype=dtype, m=n * P * Q, c=d.k_pad, c_real=k, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    f = lambda a: torch.tensor(np.pad(a, (0, d.k_pad - k)), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(mm_start), f(np.ones(k))
    sm, si, sc, sh = [torch.zeros(d.k_pad, dtype=torch.float32, device=gpu) for _ in range(4)]
    yb = torch.zeros_like(y)
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    L.call("rn_bn_fwd_train_part", C.byref(bd), p(part), nblk, lib.rn_conv_bn_part_rows(C.byref(d), 0), d.k_pad, p(y), p(yb), p(g_d), p(b_d), p(mm),
           p(mv), p(sm), p(si), p(sc), p(sh), p(ws), stream())
    torch.cuda.synchronize()
    assert rel_err(sm.cpu().numpy()[:k], cache[3]) < 1e-6
    assert rel_err(mv.cpu().numpy()[:k], mv_ref) < 1e-5
    assert rel_err(mm.cpu().numpy()[:k], mm_ref) < 1e-5
    assert rel_err(from_nhwc(yb, k), ops.relu_fwd(y_ref)) < TOL[dtype]


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_stem_prepare_and_smallc_conv(gpu, dtype, mode):
    """conv0 path: bn_data (train / moving stats / none) over the NCHW batch -> NHWC-8 copy
    (rn_stem_prepare), conv0 fwd in the implicit GEMM's small-C mode, conv0 wgrad over the padded
    channels (symbol/resnet.py:90-93)."""
    n, c, h, w, k, r, st, pd = 2, 3, 20, 16, 64, 7, 2, 3
    rng = np.random.default_rng(17)
    x = rng.uniform(-1, 1, (n, c, h, w)).astype(np.float32) * 2 + 0.5
    gamma, beta = np.ones(c), rng.standard_normal(c) * 0.1
    mm0, mv0 = rng.standard_normal(c) * 0.1, rng.uniform(0.5, 1.5, c)
    if mode == 0:
        xa, cache = ops.bn_train_fwd(x.astype(np.float64), gamma, beta, 2e-5, True)
        mm_ref, mv_ref = ops.bn_moving_update(mm0, mv0, cache[3], cache[4], 0.9)
    elif mode == 1:
        xa = ops.bn_infer_fwd(x.astype(np.float64), gamma, beta, mm0, mv0, 2e-5, True)
    else:
        xa = x.astype(np.float64)
    bd = L.BNDesc(dtype=dtype, m=n * h * w, c=8, c_real=c, eps=2e-5, momentum=0.9, fix_gamma=1, relu=0)
    f = lambda a: torch.tensor(np.asarray(a, np.float32), device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(mm0), f(mv0)
    sm, si, sc, sh = [torch.zeros(8, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(4096 + 64, dtype=torch.float32, device=gpu)
    x8 = torch.zeros(n * h * w * 8, dtype=tdt(dtype), device=gpu)
    L.call("rn_stem_prepare", C.byref(bd), p(f(x)), n, c, h, w, p(x8), mode, p(g_d), p(b_d), p(mm), p(mv), p(sm),
           p(si), p(sc), p(sh), p(ws), stream())
    torch.cuda.synchronize()
    got = x8.float().cpu().numpy().reshape(n, h, w, 8)
    assert np.all(got[..., c:] == 0)
    assert rel_err(got[..., :c].transpose(0, 3, 1, 2), xa) < (1e-5 if dtype == F32 else 8e-3)
    if mode == 0:
        assert rel_err(mm.cpu().numpy(), mm_ref) < 1e-5 and rel_err(mv.cpu().numpy(), mv_ref) < 1e-5
    # conv0 on the NHWC-8 copy (small-C implicit GEMM) + wgrad over padded channels
    xq = got[..., :c].transpose(0, 3, 1, 2).astype(np.float64)  # what the conv reads
    wt = rng.standard_normal((k, c, r, r)) * 0.1
    if dtype == BF16:
        wt = bf16_round(wt)
    d = conv_desc(dtype, n, 8, h, w, k, r, r, st, pd, c_real=c)
    wk = torch.zeros(k * r * r * 8, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), None, stream())
    y = torch.zeros((n, d.p, d.q, d.k_pad), dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_fwd", C.byref(d), p(x8), p(wk), p(y), dtype, None, None, stream())
    dy = rng.standard_normal((n, k, d.p, d.q))
    if dtype == BF16:
        dy = bf16_round(dy)
    dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter", C.byref(d), p(x8), p(to_nhwc(dy, dtype, gpu)), p(dw), stream())
    torch.cuda.synchronize()
    y_ref = ops.conv2d_fwd(xq, wt, (st, st), (pd, pd))
    _, dw_ref = ops.conv2d_bwd(xq, wt, dy, (st, st), (pd, pd))
    assert rel_err(from_nhwc(y, k), y_ref) < TOL[dtype]
    assert rel_err(dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2), dw_ref) < \
        (TOL[dtype] if dtype == F32 else 5e-3)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", [(2, 64, 14, 14, 256, 1, 1, 0), (2, 256, 7, 9, 64, 1, 2, 0), (3, 48, 5, 5, 1000, 1, 1, 0)])
def test_conv_bnrelu_on_load(gpu, dtype, case):
    """rn_conv_fwd_x / rn_conv_bwd_filter_x: the conv reads the PRE-BatchNorm tensor and stages
    max(x*sc + sh, 0) (the BN+ReLU of pre-activation units, symbol/resnet.py:17-31)."""
    n, c, h, w, k, r, st, pd = case
    x, wt = _conv_data(case, 18)
    rng = np.random.default_rng(19)
    sc = rng.uniform(0.5, 1.5, c)
    sh = rng.standard_normal(c) * 0.5
    if dtype == BF16:
        x, wt = bf16_round(x), bf16_round(wt)
    xa = np.maximum(x * sc[None, :, None, None] + sh[None, :, None, None], 0)
    if dtype == BF16:
        xa = bf16_round(xa)  # the staged operand is rounded to the compute dtype
    y_ref = ops.conv2d_fwd(xa, wt, (st, st), (pd, pd))
    P, Q = y_ref.shape[2:]
    dy = rng.standard_normal((n, k, P, Q))
    if dtype == BF16:
        dy = bf16_round(dy)
    _, dw_ref = ops.conv2d_bwd(xa, wt, dy, (st, st), (pd, pd))
    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd)
    f = lambda a: torch.tensor(np.pad(a, (0, d.c - c)), dtype=torch.float32, device=gpu)
    scd, shd = f(sc), f(sh)
    xd = to_nhwc(x, dtype, gpu)
    wk = torch.zeros(k * r * r * d.c, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), None, stream())
    y = torch.zeros((n, P, Q, d.k_pad), dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_fwd_x", C.byref(d), p(xd), p(wk), p(y), dtype, None, None, p(scd), p(shd), None, stream())
    dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter_x", C.byref(d), p(xd), p(to_nhwc(dy, dtype, gpu)), p(dw), p(scd), p(shd), None, 0, stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(y, k), y_ref) < TOL[dtype]
    assert rel_err(dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2), dw_ref) < \
        (TOL[dtype] if dtype == F32 else 5e-3)


@pytest.mark.parametrize("case", [(4, 256, 28, 28, 512, 1, 1, 0), (4, 256, 28, 28, 128, 1, 2, 0),
                                  (2, 1024, 14, 14, 256, 1, 1, 0), (2, 2048, 7, 7, 512, 1, 1, 0),
                                  (3, 64, 20, 20, 256, 3, 1, 1), (2, 200, 9, 11, 136, 1, 1, 0),
                                  # act2 -> conv2 (3x3 stride 1, C = K): the 64-column tile's register table,
                                  # the 224-row tiles, the image-band weight gradients' in-place transform
                                  (3, 64, 20, 20, 64, 3, 1, 1), (4, 128, 14, 14, 128, 3, 1, 1),
                                  (3, 256, 9, 9, 256, 3, 1, 1), (2, 512, 7, 7, 512, 3, 1, 1)])
@pytest.mark.parametrize("ws", [False, True], ids=["atomic", "slab"])
def test_conv_bnrelu_on_load_tiles(gpu, case, ws, big_tiles, tile_variant):
    """BN+ReLU applied on load by the LDS-DMA tiles (igemm_big_kernel XF: the landed A chunks rewritten
    in LDS, halo chunks kept zero; wgrad_big_kernel XF: the B fragments of 1x1 convolutions after their
    transposed read) == the unfused path (rn_bn_apply, then rn_conv_fwd / rn_conv_bwd_filter_ws on its
    output) BIT FOR BIT, and the oracle on the bf16-rounded BN+ReLU output within the bf16 bar."""
    n, c, h, w, k, r, st, pd = case
    x, wt = _conv_data(case, 28)
    rng = np.random.default_rng(29)
    sc = rng.uniform(0.5, 1.5, c)
    sh = rng.standard_normal(c) * 0.5
    x, wt = bf16_round(x), bf16_round(wt)
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    P, Q = d.p, d.q
    dy = bf16_round(rng.standard_normal((n, k, P, Q)))
    f = lambda a: torch.tensor(np.pad(a, (0, d.c - c)), dtype=torch.float32, device=gpu)
    scd, shd = f(sc), f(sh)
    xd = to_nhwc(x, BF16, gpu)
    dyd = to_nhwc(dy, BF16, gpu)
    wk = torch.zeros(k * r * r * d.c, dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), None, stream())
    wsb = int(L.load().rn_conv_wgrad_ws_bytes(C.byref(d))) if ws else 0
    wsd = torch.zeros(max(wsb // 4, 4), dtype=torch.float32, device=gpu) if wsb > 0 else None
    # fused
    y = torch.zeros((n, P, Q, d.k_pad), dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_fwd_x", C.byref(d), p(xd), p(wk), p(y), BF16, None, None, p(scd), p(shd), None, stream())
    dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter_x", C.byref(d), p(xd), p(dyd), p(dw), p(scd), p(shd), p(wsd), wsb, stream())
    # unfused: the BN+ReLU output written by rn_bn_apply, then the plain entry points
    bd = L.BNDesc(dtype=BF16, m=n * h * w, c=d.c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    act = torch.zeros_like(xd)
    L.call("rn_bn_apply", C.byref(bd), p(xd), p(act), p(scd), p(shd), stream())
    y0 = torch.zeros_like(y)
    L.call("rn_conv_fwd", C.byref(d), p(act), p(wk), p(y0), BF16, None, None, stream())
    dw0 = torch.zeros_like(dw)
    L.call("rn_conv_bwd_filter_ws", C.byref(d), p(act), p(dyd), p(dw0), p(wsd), wsb, stream())
    torch.cuda.synchronize()
    if tile_variant[0] == 0 and not (big_tiles == "w4" and c > 512):  # the same tile both ways (else the transform
        assert torch.equal(y.view(torch.int16), y0.view(torch.int16))  # falls back to another tile)
    band = r == 3 and st == 1 and c == k == 64  # (the image-band weight gradient, slab and in-place transform)
    if (r == 1 or band) and wsb > 0:  # the slab path is deterministic; atomics / the 3x3 fallback kernel are not
        assert torch.equal(dw, dw0)
    else:
        assert rel_err(dw.cpu().numpy(), dw0.cpu().numpy()) < 1e-5
    xa = bf16_round(np.maximum(x * sc[None, :, None, None] + sh[None, :, None, None], 0))
    y_ref = ops.conv2d_fwd(xa, wt, (st, st), (pd, pd))
    _, dw_ref = ops.conv2d_bwd(xa, wt, dy, (st, st), (pd, pd))
    assert rel_err(from_nhwc(y, k), y_ref) < TOL[BF16]
    assert rel_err(dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2), dw_ref) < 5e-3


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("geom", [(2, 3, 20, 16, 64, 7, 2, 3), (3, 3, 18, 14, 24, 7, 2, 3), (2, 3, 12, 12, 40, 5, 1, 2)])
def test_stem_padded_nhwc4(gpu, mode, geom):
    """The bf16 stem over the zero-bordered NHWC4 image: rn_stem_prepare_p4 (bn_data in training
    mode or none), conv0 fwd (rn_stem_conv_fwd_p4) and wgrad (rn_stem_conv_wgrad_p4, adds into dw)
    against the oracle on the values the device stores; ragged output counts and odd sizes."""
    n, c, h, w, k, r, st, pd = geom
    rng = np.random.default_rng(23)
    x = rng.uniform(-1, 1, (n, c, h, w)).astype(np.float32) * 2 + 0.5
    gamma, beta = np.ones(c), rng.standard_normal(c) * 0.1
    xa = ops.bn_train_fwd(x.astype(np.float64), gamma, beta, 2e-5, True)[0] if mode == 0 else x.astype(np.float64)
    d = conv_desc(BF16, n, 8, h, w, k, r, r, st, pd, c_real=c)
    hp = max(h + 2 * pd, (d.p - 1) * st + 8)
    wp = max(w + 2 * pd, (d.q - 1) * st + 8)
    assert L.load().rn_stem_p4_supported(C.byref(d), hp, wp) == 1
    bd = L.BNDesc(dtype=BF16, m=n * h * w, c=8, c_real=c, eps=2e-5, momentum=0.9, fix_gamma=1, relu=0)
    f = lambda a: torch.tensor(np.asarray(a, np.float32), device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
    sm, si, sc, sh = [torch.zeros(8, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(4096 + 64, dtype=torch.float32, device=gpu)
    x4 = torch.zeros(n * hp * wp * 4, dtype=torch.bfloat16, device=gpu)
    L.call("rn_stem_prepare_p4", C.byref(bd), p(f(x)), n, c, h, w, p(x4), hp, wp, pd, pd, mode, p(g_d), p(b_d),
           p(mm), p(mv), p(sm), p(si), p(sc), p(sh), p(ws), stream())
    torch.cuda.synchronize()
    img = x4.float().cpu().numpy().reshape(n, hp, wp, 4)
    inner = img[:, pd:pd + h, pd:pd + w, :c].transpose(0, 3, 1, 2).astype(np.float64)
    border = img.copy()
    border[:, pd:pd + h, pd:pd + w, :c] = 0
    assert not border.any()  # zero border and zero fourth channel
    assert rel_err(inner, xa) < 8e-3
    wt = bf16_round(rng.standard_normal((k, c, r, r)) * 0.1)
    w4 = torch.full((k * 256,), 7.0, dtype=torch.bfloat16, device=gpu)
    L.call("rn_stem_weight_pack_p4", C.byref(d), p(_master_krsc(wt, gpu)), p(w4), stream())
    y = torch.zeros((n, d.p, d.q, d.k_pad), dtype=torch.bfloat16, device=gpu)
    L.call("rn_stem_conv_fwd_p4", C.byref(d), p(x4), p(w4), p(y), hp, wp, stream())
    dy = bf16_round(rng.standard_normal((n, k, d.p, d.q)))
    dw = torch.full((k * r * r * c,), 0.25, dtype=torch.float32, device=gpu)
    L.call("rn_stem_conv_wgrad_p4", C.byref(d), p(x4), p(to_nhwc(dy, BF16, gpu)), p(dw), hp, wp, stream())
    torch.cuda.synchronize()
    y_ref = ops.conv2d_fwd(inner, wt, (st, st), (pd, pd))
    _, dw_ref = ops.conv2d_bwd(inner, wt, dy, (st, st), (pd, pd))
    assert rel_err(from_nhwc(y, k), y_ref) < TOL[BF16]
    got = dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2) - 0.25
    assert rel_err(got, dw_ref) < 5e-3


@pytest.mark.parametrize("geom", [(2, 224, 224), (3, 50, 38), (1, 31, 17)])
def test_stem_band(gpu, geom):
    """stem_band_kernel (the 7x7 / stride-2 stem over image bands in LDS: 14 input rows per 4 output rows,
    the weights resident; rn_set_tuning 26 = 2: the implicit-GEMM tile) against the oracle and the tile:
    the ResNet-50 stem at 224 (several bands per workgroup), a last band with fewer rows and 16-pixel
    blocks across output rows (50 x 38 -> 25 x 19), a single ragged band."""
    n, h, w = geom
    c, k, r, st, pd = 3, 64, 7, 2, 3
    rng = np.random.default_rng(29)
    d = conv_desc(BF16, n, 8, h, w, k, r, r, st, pd, c_real=c)
    hp = max(h + 2 * pd, (d.p - 1) * st + 8)
    wp = max(w + 2 * pd, (d.q - 1) * st + 8)
    hp, wp = hp + hp % 2, wp + wp % 2
    img = np.zeros((n, hp, wp, 4), np.float32)
    xin = bf16_round(rng.uniform(-2, 2, (n, c, h, w)))
    img[:, pd:pd + h, pd:pd + w, :c] = xin.transpose(0, 2, 3, 1)
    x4 = torch.tensor(img.reshape(-1), dtype=torch.bfloat16, device=gpu)
    wt = bf16_round(rng.standard_normal((k, c, r, r)) * 0.1)
    w4 = torch.zeros((k * 256,), dtype=torch.bfloat16, device=gpu)
    L.call("rn_stem_weight_pack_p4", C.byref(d), p(_master_krsc(wt, gpu)), p(w4), stream())
    outs = []
    try:
        for mode in (0, 2):
            L.call("rn_set_tuning", 26, mode)
            y = torch.full((n, d.p, d.q, d.k_pad), float("nan"), dtype=torch.bfloat16, device=gpu)
            L.call("rn_stem_conv_fwd_p4", C.byref(d), p(x4), p(w4), p(y), hp, wp, stream())
            torch.cuda.synchronize()
            outs.append(y)
    finally:
        L.call("rn_set_tuning", 26, 0)
    y_ref = ops.conv2d_fwd(xin.astype(np.float64), wt, (st, st), (pd, pd))
    for y in outs:
        assert not torch.isnan(y).any()
        assert rel_err(from_nhwc(y, k), y_ref) < TOL[BF16]
    assert rel_err(from_nhwc(outs[0], k), from_nhwc(outs[1], k)) < 1e-2
    # bn0's statistics from the band kernel's epilogue (rn_stem_conv_fwd_p4_bnstats; whole bands per workgroup)
    lib = L.load()
    nblk = lib.rn_stem_bnstats_blocks(C.byref(d), hp, wp)
    assert (nblk > 0) == (d.p % 4 == 0)
    if nblk <= 0:
        assert lib.rn_stem_conv_fwd_p4_bnstats(C.byref(d), p(x4), p(w4), p(outs[0]), hp, wp, p(outs[0]), stream()) != 0
        return
    m = n * d.p * d.q
    part = torch.full((nblk * 3 * 64,), float("nan"), dtype=torch.float32, device=gpu)
    ys = torch.full_like(outs[0], float("nan"))
    L.call("rn_stem_conv_fwd_p4_bnstats", C.byref(d), p(x4), p(w4), p(ys), hp, wp, p(part), stream())
    torch.cuda.synchronize()
    assert torch.equal(ys.view(torch.int16), outs[0].view(torch.int16))  # the same stored output
    gamma, beta = rng.uniform(0.5, 1.5, k), rng.standard_normal(k) * 0.1
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(k)), f(np.ones(k))
    sm, si, sc, sh = [torch.zeros(k, dtype=torch.float32, device=gpu) for _ in range(4)]
    bd = L.BNDesc(dtype=BF16, m=m, c=k, c_real=k, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    L.call("rn_bn_fwd_train_part", C.byref(bd), p(part), nblk, m // nblk, 64, p(ys), None, p(g_d), p(b_d), p(mm),
           p(mv), p(sm), p(si), p(sc), p(sh), p(ws), stream())
    torch.cuda.synchronize()
    yv = ys.double().view(-1, 64)
    mean, var = yv.mean(0), yv.var(0, unbiased=False)
    assert rel_err(sm.cpu().numpy(), mean.cpu().numpy()) < 1e-5
    assert rel_err((1.0 / si.double() ** 2 - 1e-5).cpu().numpy(), var.cpu().numpy()) < 1e-4


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", [(2, 64, 14, 14, 128, 3, 1, 1), (2, 128, 14, 14, 256, 1, 2, 0),
                                  (3, 32, 13, 11, 48, 3, 2, 1), (3, 256, 20, 20, 128, 3, 2, 1),
                                  (2, 256, 14, 14, 128, 1, 1, 0), (3, 200, 9, 11, 96, 1, 1, 0)])
def test_dgrad_bn_backward_fusion(gpu, dtype, case, big_tiles, tile_variant):
    """rn_conv_bwd_data_bnred + rn_bn_bwd_part == conv dgrad followed by the BatchNorm+ReLU backward
    of the BN that produced the conv's input (pre-activation units)."""
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(20)
    xb = rng.standard_normal((n, c, h, w)) * 1.5 + 0.3            # BN input
    gamma, beta = rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.2
    if dtype == BF16:
        xb = bf16_round(xb)
    a_ref, cache = ops.bn_train_fwd(xb, gamma, beta, 1e-5, False)
    act = ops.relu_fwd(a_ref)                                      # conv input
    wt = rng.standard_normal((k, c, r, r)) / np.sqrt(c * r * r)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = rng.standard_normal((n, k, P, Q))
    prev = rng.standard_normal((n, c, h, w)) * 0.5                # an earlier contribution (add_src)
    if dtype == BF16:
        wt, dy, prev = bf16_round(wt), bf16_round(dy), bf16_round(prev)
    dact_ref, _ = ops.conv2d_bwd(act, wt, dy, (st, st), (pd, pd))
    dact_ref = dact_ref + prev
    dact_in = bf16_round(dact_ref) if dtype == BF16 else dact_ref  # the stored gradient the BN reads
    dz = ops.relu_bwd(dact_in, act)
    dx_ref, dg_ref, db_ref = ops.bn_train_bwd(dz, cache, False)

    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd)
    wc = torch.zeros(d.c * r * r * d.k_pad, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), None, p(wc), stream())
    bd = L.BNDesc(dtype=dtype, m=n * h * w, c=d.c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    f = lambda a: torch.tensor(np.pad(np.asarray(a, np.float64), (0, d.c - c)), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
    sm, si, sc, sh = [torch.zeros(d.c, dtype=torch.float32, device=gpu) for _ in range(4)]
    lib = L.load()
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    xbd = to_nhwc(xb, dtype, gpu)
    L.call("rn_bn_fwd_train", C.byref(bd), p(xbd), None, p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc), p(sh),
           p(ws), stream())
    dact = to_nhwc(prev, dtype, gpu)                               # accumulated in place (add_src = out)
    nrb = lib.rn_conv_bnred_blocks(C.byref(d))
    part = torch.full((nrb * d.c * 2,), float("nan"), dtype=torch.float32, device=gpu)  # every slot written
    dyd = to_nhwc(dy, dtype, gpu)
    L.call("rn_conv_bwd_data_bnred", C.byref(d), p(dyd), p(wc), p(dact), p(dact), p(xbd), p(sm), p(sc), p(sh), 1,
               p(part), stream())
    dx = torch.zeros_like(xbd)
    dg, db = torch.zeros(d.c, dtype=torch.float32, device=gpu), torch.zeros(d.c, dtype=torch.float32, device=gpu)
    L.call("rn_bn_bwd_part", C.byref(bd), p(part), nrb, p(xbd), p(dact), p(dx), None, p(g_d), p(sm), p(si), p(sc),
               p(sh), p(dg), p(db), p(ws), stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(dact, c), dact_ref) < TOL[dtype]
    assert not torch.isnan(part).any()
    assert rel_err(db.cpu().numpy()[:c], db_ref) < (1e-4 if dtype == F32 else 2e-2)
    assert rel_err(dg.cpu().numpy()[:c], dg_ref) < (1e-4 if dtype == F32 else 2e-2)
    assert rel_err(from_nhwc(dx, c), dx_ref) < (TOL[dtype] * 5 if dtype == F32 else 3e-2)


@pytest.mark.parametrize("relu,fix_gamma,with_add", [(1, 0, 0), (1, 0, 1), (0, 1, 1)])
@pytest.mark.parametrize("case", [(2, 256, 14, 14, 64, 1, 1, 0), (3, 512, 9, 11, 128, 1, 1, 0),
                                  (2, 1024, 7, 7, 256, 1, 1, 0), (4, 256, 28, 28, 64, 1, 1, 0)])
def test_dgrad_bn_backward_recompute(gpu, case, relu, fix_gamma, with_add, big_tiles, tile_variant):
    """rn_conv_bwd_data_bnred (dx = NULL: reduction only) + rn_bn_bwd_finalize + rn_conv_bwd_data_bnapply
    (the dgrad recomputed with the BatchNorm backward applied in its epilogue) == rn_conv_bwd_data_bnred +
    rn_bn_bwd_part, bit for bit (dx, dgamma, dbeta), and == the oracle's conv dgrad + BN(+ReLU) backward
    within bf16 tolerance. The pre-activation units' conv1 (1x1, the BN has 4x the conv's channels)."""
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(21)
    xb = bf16_round(rng.standard_normal((n, c, h, w)) * 1.5 + 0.3)  # BN input
    gamma, beta = rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.2
    a_ref, cache = ops.bn_train_fwd(xb, gamma, beta, 1e-5, bool(fix_gamma))
    act = ops.relu_fwd(a_ref) if relu else a_ref
    wt = bf16_round(rng.standard_normal((k, c, r, r)) / np.sqrt(c * r * r))
    dy = bf16_round(rng.standard_normal((n, k, h, w)))
    res = bf16_round(rng.standard_normal((n, c, h, w)) * 0.5)      # the gradient fan-in (add_src of the apply)
    dact_ref, _ = ops.conv2d_bwd(act, wt, dy, (1, 1), (0, 0))
    dz = ops.relu_bwd(bf16_round(dact_ref), act) if relu else bf16_round(dact_ref)
    dx_ref, dg_ref, db_ref = ops.bn_train_bwd(dz, cache, bool(fix_gamma))
    if with_add:
        dx_ref = dx_ref + res

    d = conv_desc(BF16, n, c, h, w, k, 1, 1, 1, 0)
    lib = L.load()
    if lib.rn_conv_tile(C.byref(d), 1) < 128:
        pytest.skip("not a 224/256-row dgrad tile under this variant")
    wc = torch.zeros(d.c * d.k_pad, dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), None, p(wc), stream())
    bd = L.BNDesc(dtype=BF16, m=n * h * w, c=d.c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=fix_gamma, relu=relu)
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
    sm, si, sc, sh = [torch.zeros(d.c, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    xbd = to_nhwc(xb, BF16, gpu)
    L.call("rn_bn_fwd_train", C.byref(bd), p(xbd), None, p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc), p(sh),
           p(ws), stream())
    dyd, resd = to_nhwc(dy, BF16, gpu), to_nhwc(res, BF16, gpu)
    add = resd if with_add else None
    nrb = lib.rn_conv_bnred_blocks(C.byref(d))
    zf = lambda: torch.zeros(d.c, dtype=torch.float32, device=gpu)
    # reference path: the dgrad stores its gradient, rn_bn_bwd_part reads it back
    part0 = torch.full((nrb * d.c * 2,), float("nan"), dtype=torch.float32, device=gpu)
    dact = torch.zeros_like(xbd)
    L.call("rn_conv_bwd_data_bnred", C.byref(d), p(dyd), p(wc), p(dact), None, p(xbd), p(sm), p(sc), p(sh), relu,
           p(part0), stream())
    dx0, dg0, db0 = torch.zeros_like(xbd), zf(), zf()
    L.call("rn_bn_bwd_part", C.byref(bd), p(part0), nrb, p(xbd), p(dact), p(dx0), p(add), p(g_d), p(sm), p(si),
           p(sc), p(sh), p(dg0), p(db0), p(ws), stream())
    # recompute path
    part1 = torch.full((nrb * d.c * 2,), float("nan"), dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_data_bnred", C.byref(d), p(dyd), p(wc), None, None, p(xbd), p(sm), p(sc), p(sh), relu,
           p(part1), stream())
    coef = torch.zeros(4 * d.c, dtype=torch.float32, device=gpu)
    dg1, db1 = zf(), zf()
    L.call("rn_bn_bwd_finalize", C.byref(bd), p(part1), nrb, p(g_d), p(sm), p(si), p(dg1), p(db1), p(coef), stream())
    dx1 = torch.full_like(xbd, float("nan"))
    L.call("rn_conv_bwd_data_bnapply", C.byref(d), p(dyd), p(wc), p(dx1), p(add), p(xbd), p(coef), p(sc), p(sh),
           relu, stream())
    torch.cuda.synchronize()
    assert torch.equal(part0, part1)
    assert torch.equal(dg0, dg1) and torch.equal(db0, db1)
    assert torch.equal(dx0.view(torch.int16), dx1.view(torch.int16))
    assert rel_err(from_nhwc(dx1, c), dx_ref) < 3e-2
    assert rel_err(db1.cpu().numpy()[:c], db_ref) < 2e-2
    if not fix_gamma:
        assert rel_err(dg1.cpu().numpy()[:c], dg_ref) < 2e-2


def test_dgrad_bn_backward_recompute_args(gpu):
    """The reduction-only dgrad and the apply dgrad need the 224/256-row tile (bf16): the fp32 path
    and a missing output are refused with an error, not run."""
    d32 = conv_desc(F32, 2, 256, 14, 14, 64, 1, 1, 1, 0)
    lib = L.load()
    x = torch.zeros(8, device=gpu)
    assert lib.rn_conv_bwd_data_bnapply(C.byref(d32), p(x), p(x), p(x), None, p(x), p(x), p(x), p(x), 1,
                                        stream()) != 0
    assert lib.rn_conv_bwd_data_bnred(C.byref(d32), p(x), p(x), None, None, p(x), p(x), p(x), p(x), 1, p(x),
                                      stream()) != 0
    assert lib.rn_conv_bwd_data_bnred(C.byref(d32), p(x), p(x), None, None, None, None, None, None, 1, None,
                                      stream()) != 0


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", [(2, 256, 14, 14, 64, 1, 1, 0), (3, 128, 13, 11, 96, 3, 1, 1), (2, 64, 16, 16, 128, 3, 2, 1)])
def test_bn_backward_quant_clip_fold(gpu, dtype, case):
    """The int8 graph's activation quantizer (Quantization_int8 after BN+ReLU, symbol/resnet_int8.py)
    folded into the BN backward (rn_bn_desc.clip): (a) rn_bn_bwd with the clip == rn_quant_int8_bwd
    followed by rn_bn_bwd without it, bit for bit; (b, bf16) the conv dgrad reducing the clipped BN
    backward in its epilogue (rn_conv_bwd_data_bnred_clip + rn_bn_bwd_part) == the oracle's dgrad ->
    STE clip (zero where the stored BN output >= t) -> BN+ReLU backward."""
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(31)
    xb = rng.standard_normal((n, c, h, w)) * 1.5 + 0.3
    if dtype == BF16:
        xb = bf16_round(xb)
    gamma, beta = rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.2
    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd)
    lib = L.load()
    f = lambda a: torch.tensor(np.pad(np.asarray(a, np.float64), (0, d.c - c)), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
    sm, si, sc, sh = [torch.zeros(d.c, dtype=torch.float32, device=gpu) for _ in range(4)]
    bd = L.BNDesc(dtype=dtype, m=n * h * w, c=d.c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    xbd = to_nhwc(xb, dtype, gpu)
    act = torch.zeros_like(xbd)
    L.call("rn_bn_fwd_train", C.byref(bd), p(xbd), p(act), p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc), p(sh),
           p(ws), stream())
    torch.cuda.synchronize()
    a_np = from_nhwc(act, c)
    t = float(np.quantile(a_np[a_np > 0], 0.7))  # a threshold that clips ~30 % of the positive outputs
    tq = torch.tensor([t], dtype=torch.float32, device=gpu)
    # (a) the BN backward with the folded clip vs the quantizer's backward pass followed by it
    dyb = to_nhwc(rng.standard_normal((n, c, h, w)), dtype, gpu)
    zf = lambda: torch.zeros(d.c, dtype=torch.float32, device=gpu)
    dq = torch.zeros_like(xbd)
    L.call("rn_quant_int8_bwd", dtype, act.numel(), p(act), p(dyb), p(dq), p(tq), 0, None, stream())
    dx0, dg0, db0 = torch.zeros_like(xbd), zf(), zf()
    L.call("rn_bn_bwd", C.byref(bd), p(xbd), p(dq), p(dx0), None, p(g_d), p(sm), p(si), p(sc), p(sh), p(dg0), p(db0),
           p(ws), stream())
    bdc = L.BNDesc(dtype=dtype, m=n * h * w, c=d.c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1,
                   clip=tq.data_ptr())
    dx1, dg1, db1 = torch.zeros_like(xbd), zf(), zf()
    L.call("rn_bn_bwd", C.byref(bdc), p(xbd), p(dyb), p(dx1), None, p(g_d), p(sm), p(si), p(sc), p(sh), p(dg1), p(db1),
           p(ws), stream())
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1) and torch.equal(dg0, dg1) and torch.equal(db0, db1)
    assert (dq == 0).float().mean().item() > 0.05  # the clip zeroed the gradient of the outputs >= t
    if dtype != BF16:
        return  # (b) runs on the bf16 LDS-DMA tiles only
    # (b) the dgrad's epilogue reduces the clipped BN backward
    wt = rng.standard_normal((k, c, r, r)) / np.sqrt(c * r * r)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = rng.standard_normal((n, k, P, Q))
    if dtype == BF16:
        wt, dy = bf16_round(wt), bf16_round(dy)
    wc = torch.zeros(d.c * r * r * d.k_pad, dtype=tdt(dtype), device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), None, p(wc), stream())
    nrb = lib.rn_conv_bnred_blocks(C.byref(d))
    part = torch.full((nrb * d.c * 2,), float("nan"), dtype=torch.float32, device=gpu)
    dact = torch.zeros_like(xbd)
    dyd = to_nhwc(dy, dtype, gpu)
    L.call("rn_conv_bwd_data_bnred_clip", C.byref(d), p(dyd), p(wc), p(dact), None, p(xbd), p(sm), p(sc), p(sh), 1,
           p(tq), p(part), stream())
    dx2, dg2, db2 = torch.zeros_like(xbd), zf(), zf()
    L.call("rn_bn_bwd_part", C.byref(bdc), p(part), nrb, p(xbd), p(dact), p(dx2), None, p(g_d), p(sm), p(si),
           p(sc), p(sh), p(dg2), p(db2), p(ws), stream())
    torch.cuda.synchronize()
    a_ref, cache = ops.bn_train_fwd(xb, gamma, beta, 1e-5, False)
    act_ref = ops.relu_fwd(a_ref)
    dact_ref, _ = ops.conv2d_bwd(act_ref, wt, dy, (st, st), (pd, pd))
    g_st = from_nhwc(dact, c)                                 # the stored gradient (what the STE reads)
    keep = (a_np > 0) & (a_np < t)                            # relu' x clip on the stored BN output
    dx_ref, dg_ref, db_ref = ops.bn_train_bwd(g_st * keep, cache, False)
    assert rel_err(g_st, dact_ref) < TOL[dtype]
    assert rel_err(from_nhwc(dx2, c), dx_ref) < (TOL[dtype] * 5 if dtype == F32 else 3e-2)
    assert rel_err(db2.cpu().numpy()[:c], db_ref) < (1e-4 if dtype == F32 else 2e-2)
    assert rel_err(dg2.cpu().numpy()[:c], dg_ref) < (1e-4 if dtype == F32 else 2e-2)


BIG_CASES = [
    # n, c, h, w, k, r, stride, pad: 256-row tiles (fwd when k >= 128, dgrad when c >= 128)
    (2, 128, 14, 14, 256, 3, 1, 1),
    (3, 256, 9, 11, 136, 3, 2, 1),     # ragged column tile, stride-2 dgrad classes
    (2, 160, 13, 13, 384, 1, 2, 0),    # reduction 160: last 64-deep K-tile partly out of range
    (1, 512, 7, 7, 512, 3, 1, 1),      # fewer rows than one tile
    (4, 128, 28, 28, 128, 3, 1, 1),    # several row tiles
    (8, 256, 16, 16, 512, 1, 2, 0),    # wgrad: M split over several workgroups
    (3, 64, 20, 20, 64, 3, 1, 1),      # 64 columns both ways: the 4-wave 256x64 tile
    (2, 40, 13, 11, 56, 5, 2, 2),      # 256x64 tile: ragged columns, 25 taps, stride-2 classes
]


@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("case", BIG_CASES)
def test_conv_big_tiles(gpu, mode, case, tile_variant):
    """igemm_big_kernel (rn_set_tuning 4: 2 = 256x256, 3 = 256x128) for fwd + residual and dgrad;
    wgrad_big_kernel (rn_set_tuning 5 = 1; >= 128 output channels, >= 256 columns) for the weight gradient."""
    n, c, h, w, k, r, st, pd = case
    x, wt = _conv_data(case, 5)
    x, wt = bf16_round(x), bf16_round(wt)
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    rng = np.random.default_rng(6)
    res = bf16_round(rng.standard_normal((n, k, P, Q)))
    dy = bf16_round(rng.standard_normal((n, k, P, Q)))
    ref = ops.conv2d_fwd(x, wt, (st, st), (pd, pd)) + res
    dx_ref, dw_ref = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd))
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    wk = torch.zeros(k * r * r * d.c, dtype=torch.bfloat16, device=gpu)
    wc = torch.zeros(d.c * r * r * d.k_pad, dtype=torch.bfloat16, device=gpu)
    wm = _master_krsc(wt, gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(wm), p(wk), p(wc), stream())
    y = torch.zeros((n, P, Q, d.k_pad), dtype=torch.bfloat16, device=gpu)
    dx = torch.zeros((n, h, w, d.c), dtype=torch.bfloat16, device=gpu)
    dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
    dw2 = torch.zeros_like(dw)
    xd, rd, dyd = to_nhwc(x, BF16, gpu), to_nhwc(res, BF16, gpu), to_nhwc(dy, BF16, gpu)  # alive across the calls
    L.call("rn_set_tuning", 4, mode)
    L.call("rn_set_tuning", 5, 1)
    try:
        L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(y), BF16, p(rd), None, stream())
        L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(dx), None, stream())
        L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dyd), p(dw), stream())  # wgrad_big_kernel when eligible
        L.call("rn_set_tuning", 5, 4)  # the LDS-DMA variants incl. the 64x128 one for K <= 64
        L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dyd), p(dw2), stream())
        L.call("rn_set_tuning", 5, 0)
        # split-M partial slabs + reduction (default tiles with a workspace), and a too-small
        # workspace (falls back to the atomic epilogue); dw is accumulated into (+=)
        need = L.load().rn_conv_wgrad_ws_bytes(C.byref(d))
        ws = torch.full((max(need, 16) // 4 + 4,), float("nan"), dtype=torch.float32, device=gpu)
        dw3 = torch.full_like(dw, 0.5)
        dw4 = torch.zeros_like(dw)
        L.call("rn_conv_bwd_filter_ws", C.byref(d), p(xd), p(dyd), p(dw3), p(ws), need, stream())
        L.call("rn_conv_bwd_filter_ws", C.byref(d), p(xd), p(dyd), p(dw4), p(ws), max(need - 4, 0), stream())
        torch.cuda.synchronize()
    finally:
        L.call("rn_set_tuning", 4, 0)
        L.call("rn_set_tuning", 5, 0)
    assert rel_err(from_nhwc(y, k), ref) < TOL[BF16]
    assert rel_err(from_nhwc(dx, c), dx_ref) < TOL[BF16]
    dw3 -= 0.5
    for g in (dw, dw2, dw3, dw4):
        assert rel_err(g.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2), dw_ref) < 5e-3


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("bnb", [False, True], ids=["identity_shortcut", "bn_shortcut"])
@pytest.mark.parametrize("relu", [1, 0])
def test_bn_apply_add(gpu, dtype, bnb, relu):
    """rn_bn_apply_add (the post-activation unit tail, symbol/resnext.py:40-47: bn3 [+ shortcut BN] ->
    add -> relu) == rn_bn_apply of each BatchNorm, then rn_eltwise_add, bit for bit."""
    n, c, h, w = 3, 72, 9, 7
    rng = np.random.default_rng(31)
    m = n * h * w
    xa = torch.tensor(rng.standard_normal((m, c)) * 2, dtype=tdt(dtype), device=gpu)
    xb = torch.tensor(rng.standard_normal((m, c)) * 2, dtype=tdt(dtype), device=gpu)
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=gpu)
    sca, sha, scb, shb = f(rng.uniform(0.3, 1.7, c)), f(rng.standard_normal(c)), f(rng.uniform(0.3, 1.7, c)), \
        f(rng.standard_normal(c))
    bd = L.BNDesc(dtype=dtype, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=0)
    y = torch.zeros_like(xa)
    L.call("rn_bn_apply_add", C.byref(bd), p(xa), p(sca), p(sha), p(xb), p(scb) if bnb else None,
           p(shb) if bnb else None, p(y), relu, stream())
    ya, yb, y0 = torch.zeros_like(xa), torch.zeros_like(xa), torch.zeros_like(xa)
    L.call("rn_bn_apply", C.byref(bd), p(xa), p(ya), p(sca), p(sha), stream())
    if bnb:
        L.call("rn_bn_apply", C.byref(bd), p(xb), p(yb), p(scb), p(shb), stream())
    L.call("rn_eltwise_add", m * c, dtype, p(ya), p(yb if bnb else xb), p(y0), relu, stream())
    torch.cuda.synchronize()
    iv = torch.int16 if dtype == BF16 else torch.int32
    assert torch.equal(y.view(iv), y0.view(iv))
    ref = xa.double().cpu().numpy() * sca.cpu().numpy() + sha.cpu().numpy()
    ref = ref + ((xb.double().cpu().numpy() * scb.cpu().numpy() + shb.cpu().numpy()) if bnb else xb.double().cpu().numpy())
    if relu:
        ref = np.maximum(ref, 0)
    assert rel_err(y.double().cpu().numpy(), ref) < TOL[dtype]


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("bnb", [False, True], ids=["identity_shortcut", "bn_shortcut"])
def test_relu_bwd_bnred(gpu, dtype, bnb):
    """rn_relu_bwd_bnred + rn_bn_bwd_part (the backward of the post-activation unit tail) == rn_relu_bwd
    then rn_bn_bwd on each BatchNorm feeding the add: the ReLU gradient bit for bit, the BN gradients
    (dx, dgamma, dbeta) within fp32 reduction-order error, and the oracle's BN backward."""
    n, c, h, w = 4, 80, 11, 9
    m = n * h * w
    rng = np.random.default_rng(37)
    t = lambda a: torch.tensor(a, dtype=tdt(dtype), device=gpu)
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=gpu)
    y = t(np.maximum(rng.standard_normal((m, c)), 0) * (rng.random((m, c)) < 0.7))
    dy = t(rng.standard_normal((m, c)))
    xs = [t(rng.standard_normal((m, c)) * 1.5 + 0.4) for _ in range(2)]
    bd = L.BNDesc(dtype=dtype, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=0)
    lib = L.load()
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    stats = []
    for x in xs:  # save_mean / save_invstd / scale / shift of each BN from its forward
        g_, b_ = f(rng.uniform(0.5, 1.5, c)), f(rng.standard_normal(c) * 0.1)
        sm, si, sc, sh = [torch.zeros(c, dtype=torch.float32, device=gpu) for _ in range(4)]
        L.call("rn_bn_fwd_train", C.byref(bd), p(x), None, p(g_), p(b_), None, None, p(sm), p(si), p(sc), p(sh), p(ws),
               stream())
        stats.append((g_, sm, si, sc, sh))
    nrb = lib.rn_bn_reduce_blocks(C.byref(bd))
    parts = [torch.full((nrb * c * 2,), float("nan"), dtype=torch.float32, device=gpu) for _ in range(2)]
    g = torch.zeros_like(dy)
    L.call("rn_relu_bwd_bnred", C.byref(bd), p(y), p(dy), p(g), p(xs[0]), p(stats[0][1]), p(parts[0]),
           p(xs[1]) if bnb else None, p(stats[1][1]) if bnb else None, p(parts[1]) if bnb else None, stream())
    g0 = torch.zeros_like(dy)
    L.call("rn_relu_bwd", m * c, dtype, p(y), p(dy), p(g0), None, stream())
    torch.cuda.synchronize()
    iv = torch.int16 if dtype == BF16 else torch.int32
    assert torch.equal(g.view(iv), g0.view(iv))
    for k in range(2 if bnb else 1):
        gam, sm, si, sc, sh = stats[k]
        dx, dx0 = torch.zeros_like(dy), torch.zeros_like(dy)
        dg, db, dg0, db0 = [torch.zeros(c, dtype=torch.float32, device=gpu) for _ in range(4)]
        L.call("rn_bn_bwd_part", C.byref(bd), p(parts[k]), nrb, p(xs[k]), p(g), p(dx), None, p(gam), p(sm), p(si),
               p(sc), p(sh), p(dg), p(db), p(ws), stream())
        L.call("rn_bn_bwd", C.byref(bd), p(xs[k]), p(g0), p(dx0), None, p(gam), p(sm), p(si), p(sc), p(sh), p(dg0),
               p(db0), p(ws), stream())
        torch.cuda.synchronize()
        assert rel_err(dg.cpu().numpy(), dg0.cpu().numpy()) < 1e-5
        assert rel_err(db.cpu().numpy(), db0.cpu().numpy()) < 1e-5
        assert rel_err(dx.double().cpu().numpy(), dx0.double().cpu().numpy()) < (1e-5 if dtype == F32 else 1e-2)
        xd = xs[k].double().cpu().numpy().reshape(n, h, w, c).transpose(0, 3, 1, 2)
        gd = g.double().cpu().numpy().reshape(n, h, w, c).transpose(0, 3, 1, 2)
        _, cache = ops.bn_train_fwd(xd, gam.double().cpu().numpy(), np.zeros(c), 1e-5, False)
        dx_ref, dg_ref, db_ref = ops.bn_train_bwd(gd, cache, False)
        assert rel_err(db.cpu().numpy(), db_ref) < 1e-4 and rel_err(dg.cpu().numpy(), dg_ref) < 1e-4
        assert rel_err(dx.double().cpu().numpy().reshape(n, h, w, c).transpose(0, 3, 1, 2), dx_ref) < TOL[dtype]



@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("with_add", [False, True])
def test_maxpool_block_bwd(gpu, dtype, with_add):
    """3x3 / stride-2 max-pool backward over 2x2 input blocks (H = 2P, W = 2Q: the stem pool,
    symbol/resnet.py:97) == the per-pixel gather (rn_set_tuning 12 = 1) bit for bit, and the oracle's
    first-max rule; ties from post-ReLU zeros, an accumulated add_src."""
    rng = np.random.default_rng(43)
    n, c, h, w = 3, 24, 14, 12
    x = np.round(np.maximum(rng.standard_normal((n, c, h, w)), 0) * 4) / 4
    y_ref, arg = ops.maxpool_fwd(x, (3, 3), (2, 2), (1, 1))
    dy = rng.standard_normal(y_ref.shape)
    prev = rng.standard_normal(x.shape)
    if dtype == BF16:
        dy, prev = bf16_round(dy), bf16_round(prev)
    dx_ref = ops.maxpool_bwd(dy, arg, x.shape, (3, 3), (2, 2), (1, 1)) + (prev if with_add else 0)
    d = L.PoolDesc(dtype=dtype, n=n, h=h, w=w, c=pad8(c), r=3, s=3, stride_h=2, stride_w=2, pad_h=1, pad_w=1,
                   type=L.RN_POOL_MAX, global_pool=0)
    L.call("rn_pool_desc_init", C.byref(d))
    assert (d.p, d.q) == (h // 2, w // 2)
    xd = to_nhwc(x, dtype, gpu)
    yd = torch.zeros((n, d.p, d.q, pad8(c)), dtype=tdt(dtype), device=gpu)
    am = torch.zeros(yd.numel(), dtype=torch.uint8, device=gpu)
    L.call("rn_pool_fwd", C.byref(d), p(xd), p(yd), p(am), stream())
    dyd, addd = to_nhwc(dy, dtype, gpu), to_nhwc(prev, dtype, gpu)
    out = []
    for mode in (0, 1):
        L.call("rn_set_tuning", 12, mode)
        dxd = torch.zeros_like(xd)
        L.call("rn_pool_bwd", C.byref(d), p(dyd), p(am), p(dxd), p(addd) if with_add else None, stream())
        torch.cuda.synchronize()
        out.append(dxd)
    L.call("rn_set_tuning", 12, 0)
    iv = torch.int16 if dtype == BF16 else torch.int32
    assert torch.equal(out[0].view(iv), out[1].view(iv))
    assert rel_err(from_nhwc(out[0], c), dx_ref) < TOL[dtype]


@pytest.mark.parametrize("case", [(3, 64, 14, 12), (2, 16, 22, 18), (1, 256, 8, 8), (5, 64, 36, 40)])
@pytest.mark.parametrize("with_add", [False, True])
def test_maxpool_bwd_bn_backward_fusion(gpu, case, with_add):
    """rn_pool_bwd_bnred + rn_bn_bwd_part (the stem's bn0 -> relu0 -> pool0 backward, symbol/resnet.py:
    94-97, the BN reduction in the pool backward) == rn_pool_bwd (dx bit for bit) followed by the
    oracle's BatchNorm+ReLU backward on the stored gradient."""
    n, c, h, w = case
    rng = np.random.default_rng(44)
    xb = bf16_round(rng.standard_normal((n, c, h, w)) * 1.5 + 0.3)  # BN input
    gamma, beta = rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.2
    a_ref, cache = ops.bn_train_fwd(xb, gamma, beta, 1e-5, False)
    d = L.PoolDesc(dtype=BF16, n=n, h=h, w=w, c=c, r=3, s=3, stride_h=2, stride_w=2, pad_h=1, pad_w=1,
                   type=L.RN_POOL_MAX, global_pool=0)
    L.call("rn_pool_desc_init", C.byref(d))
    lib = L.load()
    nrb = lib.rn_pool_bwd_bnred_blocks(C.byref(d))
    assert nrb > 0
    bd = L.BNDesc(dtype=BF16, m=n * h * w, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    g_d, b_d, mm, mv = f(gamma), f(beta), f(np.zeros(c)), f(np.ones(c))
    sm, si, sc, sh = [torch.zeros(c, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(lib.rn_bn_workspace_bytes(C.byref(bd)) // 4 + 16, dtype=torch.float32, device=gpu)
    xbd = to_nhwc(xb, BF16, gpu)
    act = torch.zeros_like(xbd)
    L.call("rn_bn_fwd_train", C.byref(bd), p(xbd), p(act), p(g_d), p(b_d), p(mm), p(mv), p(sm), p(si), p(sc), p(sh),
           p(ws), stream())
    yd = torch.zeros((n, d.p, d.q, c), dtype=torch.bfloat16, device=gpu)
    am = torch.zeros(yd.numel(), dtype=torch.uint8, device=gpu)
    L.call("rn_pool_fwd", C.byref(d), p(act), p(yd), p(am), stream())
    dyd = to_nhwc(bf16_round(rng.standard_normal((n, c, d.p, d.q))), BF16, gpu)
    prev = to_nhwc(bf16_round(rng.standard_normal((n, c, h, w)) * 0.5), BF16, gpu)
    dact = prev.clone() if with_add else torch.zeros_like(xbd)  # (accumulated in place: add_src = out)
    plain = dact.clone()
    part = torch.full((nrb * c * 2,), float("nan"), dtype=torch.float32, device=gpu)  # every slot written
    addp = (lambda t: p(t) if with_add else None)
    L.call("rn_pool_bwd_bnred", C.byref(d), p(dyd), p(am), p(dact), addp(dact), p(xbd), p(sm), p(sc), p(sh), 1,
           p(part), stream())
    L.call("rn_pool_bwd", C.byref(d), p(dyd), p(am), p(plain), addp(plain), stream())
    dx = torch.zeros_like(xbd)
    dg, db = torch.zeros(c, dtype=torch.float32, device=gpu), torch.zeros(c, dtype=torch.float32, device=gpu)
    L.call("rn_bn_bwd_part", C.byref(bd), p(part), nrb, p(xbd), p(dact), p(dx), None, p(g_d), p(sm), p(si), p(sc),
           p(sh), p(dg), p(db), p(ws), stream())
    torch.cuda.synchronize()
    assert torch.equal(dact, plain)
    assert not torch.isnan(part).any()
    dz = ops.relu_bwd(from_nhwc(dact, c), from_nhwc(act, c))  # the stored gradient, the stored ReLU output
    dx_ref, dg_ref, db_ref = ops.bn_train_bwd(dz, cache, False)
    assert rel_err(db.cpu().numpy(), db_ref) < 1e-4
    assert rel_err(dg.cpu().numpy(), dg_ref) < 1e-4
    assert rel_err(from_nhwc(dx, c), dx_ref) < 3e-2


@pytest.mark.parametrize("case", GCONV_CASES[:4])
def test_grouped_conv_zero_block_skip(gpu, case):
    """rn_set_tuning 13 / 14: the grouped 64-column tiles skip the MFMAs of their block-diagonal zero
    blocks (equal channels in and out per group, <= 32: every ResNeXt-50 3x3) -- the skipped products
    are exact zeros, so forward and data gradient equal the unskipped tile's values exactly; the weight
    gradient (fp32 atomics over the M splits: summation order varies) to fp32 rounding."""
    n, c, h, w, k, r, st, pd, g = case
    L.call("rn_set_tuning", 15, 1)  # (4 / 8 channels per group: the block-diagonal path, not the direct one)
    try:
        _zero_block_skip(gpu, n, c, h, w, k, r, st, pd, g)
    finally:
        L.call("rn_set_tuning", 15, 0)


def _zero_block_skip(gpu, n, c, h, w, k, r, st, pd, g):
    rng = np.random.default_rng(12)
    x = bf16_round(rng.standard_normal((n, c, h, w)))
    wt = bf16_round(rng.standard_normal((k, c // g, r, r)) / np.sqrt(c // g * r * r))
    P, Q = ops.conv_out_hw(h, w, r, r, (st, st), (pd, pd))
    dy = bf16_round(rng.standard_normal((n, k, P, Q)))
    d = L.ConvDesc(dtype=BF16, n=n, h=h, w=w, c=c, c_real=c, k=k, k_pad=k, r=r, s=r, stride_h=st, stride_w=st,
                   pad_h=pd, pad_w=pd, groups=g)
    L.call("rn_conv_desc_init", C.byref(d))
    lib = L.load()
    assert lib.rn_conv_tile(C.byref(d), 0) == 64
    wk = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 0), dtype=torch.bfloat16, device=gpu)
    wc = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 1), dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), p(wc), stream())
    xd, dyd = to_nhwc(x, BF16, gpu), to_nhwc(dy, BF16, gpu)
    outs = []
    for mode in (0, 1, 2):  # (14 = 2: the diagonal blocks on two of the four waves)
        L.call("rn_set_tuning", 13, min(mode, 1))
        L.call("rn_set_tuning", 14, mode)
        y = torch.zeros((n, P, Q, k), dtype=torch.bfloat16, device=gpu)
        dx = torch.zeros((n, h, w, c), dtype=torch.bfloat16, device=gpu)
        dw = torch.zeros(lib.rn_conv_weight_numel(C.byref(d)), dtype=torch.float32, device=gpu)
        L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(y), BF16, None, None, stream())
        L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(dx), None, stream())
        L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dyd), p(dw), stream())
        torch.cuda.synchronize()
        outs.append((y.float().cpu().numpy(), dx.float().cpu().numpy(), dw.cpu().numpy()))
    L.call("rn_set_tuning", 13, 0)  # (the library defaults)
    L.call("rn_set_tuning", 14, 0)
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
    assert rel_err(from_nhwc(torch.tensor(outs[0][0]), k), ops.conv2d_fwd(x, wt, (st, st), (pd, pd), g)) < TOL[BF16]
    assert rel_err(outs[0][2], outs[1][2]) < 1e-5 and rel_err(outs[2][2], outs[1][2]) < 1e-5
    _, dw_ref = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd), g)
    assert rel_err(outs[0][2].reshape(k, r, r, c // g).transpose(0, 3, 1, 2), dw_ref) < 5e-3


@pytest.mark.parametrize("case", [
    (3, 64, 56, 56, 64, 3, 1, 1),    # the stage-1 conv2 shape (one image per workgroup)
    (5, 64, 9, 13, 64, 3, 1, 1),     # odd rows: the last band has one output row
    (2, 64, 7, 62, 64, 3, 1, 1),     # the widest row the 64-pixel band image holds
    (6, 128, 28, 28, 128, 3, 1, 1),  # stage 2: 4 output-channel slices, 32-pixel rows, one-row bands
    (3, 128, 5, 30, 128, 3, 1, 1),   # the widest 32-pixel row
    (9, 256, 14, 14, 256, 3, 1, 1),  # stage 3: 2 x 8 slices, 16-pixel rows, two-row bands
    (5, 512, 7, 7, 512, 3, 1, 1),    # stage 4: 4 x 16 slices, odd rows
])
def test_wgrad_image_bands(gpu, case):
    """wgrad_dband_kernel (dense 3x3 stride-1 weight gradients with C = K; rn_set_tuning 19 = 2 runs it at
    every C, the default at C = 64 only): dW
    slices per workgroup over bands of output rows, every tap a shifted read of one staged x image.
    Against the fp64 oracle (the sums of products of bf16 values, fp32 accumulation: 2e-6 of the sum of
    the terms' magnitudes per element), bit-identical run to run (one writer per slab element, the
    reduction in split order), and equal to the tiled kernels (rn_set_tuning 19 = 1) within fp32
    summation-order rounding."""
    n, c, h, w, k, r, st, pd = case
    x, _ = _conv_data(case, 9)
    x = bf16_round(x)
    rng = np.random.default_rng(10)
    dy = bf16_round(rng.standard_normal((n, k, h, w)))
    _, dw_ref = ops.conv2d_bwd(x, np.zeros((k, c, r, r)), dy, (st, st), (pd, pd))
    dw_abs = ops.conv2d_bwd(np.abs(x), np.zeros((k, c, r, r)), np.abs(dy), (st, st), (pd, pd))[1]
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    lib = L.load()
    L.call("rn_set_tuning", 19, 2)
    need = lib.rn_conv_wgrad_ws_bytes(C.byref(d))
    L.call("rn_set_tuning", 19, 0)
    ws = torch.full((need // 4 + 4,), float("nan"), dtype=torch.float32, device=gpu)
    xd, dyd = to_nhwc(x, BF16, gpu), to_nhwc(dy, BF16, gpu)
    outs = []
    assert need >= k * 9 * c * 4
    for band in (2, 2, 1):  # (2: the band kernel at every C, 1: the tiled kernels)
        L.call("rn_set_tuning", 19, band)
        try:
            dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
            # (the buffer's own size: the tiled kernels fall back to atomics when their slab needs more)
            L.call("rn_conv_bwd_filter_ws", C.byref(d), p(xd), p(dyd), p(dw), p(ws), ws.numel() * 4, stream())
            torch.cuda.synchronize()
        finally:
            L.call("rn_set_tuning", 19, 0)
        outs.append(dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2).astype(np.float64))
    assert np.array_equal(outs[0], outs[1])
    cond = np.abs(outs[0] - dw_ref) / (dw_abs + 1e-30)
    assert cond.max() < 2e-6, cond.max()
    assert np.abs(outs[0] - outs[2]).max() <= 1e-5 * np.abs(dw_abs).max()


@pytest.mark.parametrize("kc", [(256, 64), (64, 256), (64, 64), (128, 64), (64, 128), (128, 128), (128, 256),
                                (256, 128)])
@pytest.mark.parametrize("xf", [False, True], ids=["plain", "bnrelu_on_load"])
def test_wgrad_stream_1x1(gpu, kc, xf):
    """wgrad_stream_kernel (1x1 stride-1 weight gradients whose whole dW fits one workgroup, K x C <= 32768:
    stage 1's conv1 / conv3 / shortcut; rn_set_tuning 19 = 0): one streaming pass per workgroup over its M range,
    the split partials through the slab. Plain and with the producing BatchNorm+ReLU applied to x on load
    (rn_conv_bwd_filter_x): against the fp64 oracle of the same (rounded) operands, bit-identical run to
    run, and equal to the tiled kernels (19 = 1) within fp32 summation-order rounding; a ragged M (the
    last rows of the last split past the range)."""
    k, c = kc
    n, h, w = 3, 13, 11
    rng = np.random.default_rng(11)
    x = bf16_round(rng.standard_normal((n, c, h, w)))
    dy = bf16_round(rng.standard_normal((n, k, h, w)))
    d = conv_desc(BF16, n, c, h, w, k, 1, 1, 1, 0)
    sc = torch.tensor(rng.standard_normal(c) * 0.5, dtype=torch.float32, device=gpu)
    sh = torch.tensor(rng.standard_normal(c) * 0.3, dtype=torch.float32, device=gpu)
    xin = x
    if xf:  # the kernel multiplies bf16(max(fmaf(x, sc, sh), 0)), as the BN apply pass stores it
        xt = torch.from_numpy(x).to(gpu).float()
        v = torch.relu((xt.double() * sc.double().view(1, c, 1, 1) + sh.double().view(1, c, 1, 1)).float())
        xin = v.to(torch.bfloat16).float().cpu().numpy().astype(np.float64)
    _, dw_ref = ops.conv2d_bwd(xin, np.zeros((k, c, 1, 1)), dy, (1, 1), (0, 0))
    dw_abs = ops.conv2d_bwd(np.abs(xin), np.zeros((k, c, 1, 1)), np.abs(dy), (1, 1), (0, 0))[1]
    lib = L.load()
    need = lib.rn_conv_wgrad_ws_bytes(C.byref(d))
    assert need >= k * c * 4
    ws = torch.full((need // 4 + 4,), float("nan"), dtype=torch.float32, device=gpu)
    xd, dyd = to_nhwc(x, BF16, gpu), to_nhwc(dy, BF16, gpu)
    outs = []
    for band in (0, 0, 1):
        L.call("rn_set_tuning", 19, band)
        try:
            dw = torch.zeros(k * c, dtype=torch.float32, device=gpu)
            if xf:
                L.call("rn_conv_bwd_filter_x", C.byref(d), p(xd), p(dyd), p(dw), p(sc), p(sh), p(ws), need, stream())
            else:
                L.call("rn_conv_bwd_filter_ws", C.byref(d), p(xd), p(dyd), p(dw), p(ws), need, stream())
            torch.cuda.synchronize()
        finally:
            L.call("rn_set_tuning", 19, 0)
        outs.append(dw.cpu().numpy().reshape(k, c, 1, 1).astype(np.float64))
    assert np.array_equal(outs[0], outs[1])
    cond = np.abs(outs[0] - dw_ref) / (dw_abs + 1e-30)
    assert cond.max() < 2e-6, cond.max()
    assert np.abs(outs[0] - outs[2]).max() <= 1e-5 * np.abs(dw_abs).max()


@pytest.mark.parametrize("case", [
    (3, 128, 9, 56, 128, 3, 1, 1, 32),   # ResNeXt stage 1: 4 channels per group, 56-wide rows
    (2, 256, 7, 28, 256, 3, 1, 1, 32),   # stage 2: 8 per group, 28-wide rows (32-pixel image rows)
    (4, 128, 5, 7, 128, 3, 1, 1, 32),    # short rows, several images
    (3, 512, 7, 14, 512, 3, 1, 1, 32),   # stage 3: 16 per group, two channel slices, bands of two rows
])
def test_wgrad_grouped_image_bands(gpu, case):
    """wgrad_gband_kernel (ResNeXt's grouped 3x3 stride-1 weight gradients, 4 / 8 / 16 channels per group;
    rn_set_tuning 19 = 0): the whole block-diagonal dW per workgroup, one output row per band, the
    group-diagonal parts of each 16 x 16 MFMA block kept. Against the fp64 oracle (2e-6 of the sum of
    the terms' magnitudes per element), bit-identical run to run, and equal to the tiled grouped kernel
    (19 = 1) within fp32 summation-order rounding."""
    n, c, h, w, k, r, st, pd, g = case
    rng = np.random.default_rng(12)
    x = bf16_round(rng.standard_normal((n, c, h, w)))
    dy = bf16_round(rng.standard_normal((n, k, h, w)))
    w0 = np.zeros((k, c // g, r, r))
    _, dw_ref = ops.conv2d_bwd(x, w0, dy, (st, st), (pd, pd), g)
    dw_abs = ops.conv2d_bwd(np.abs(x), w0, np.abs(dy), (st, st), (pd, pd), g)[1]
    d = L.ConvDesc(dtype=BF16, n=n, h=h, w=w, c=c, c_real=c, k=k, k_pad=k, r=r, s=r, stride_h=st, stride_w=st,
                   pad_h=pd, pad_w=pd, groups=g)
    L.call("rn_conv_desc_init", C.byref(d))
    lib = L.load()
    need = lib.rn_conv_wgrad_ws_bytes(C.byref(d))
    assert need >= k * 9 * (c // g) * 4
    ws = torch.full((need // 4 + 4,), float("nan"), dtype=torch.float32, device=gpu)
    xd, dyd = to_nhwc(x, BF16, gpu), to_nhwc(dy, BF16, gpu)
    outs = []
    for band in (0, 0, 1):
        L.call("rn_set_tuning", 19, band)
        try:
            dw = torch.zeros(k * r * r * (c // g), dtype=torch.float32, device=gpu)
            if band == 0:
                L.call("rn_conv_bwd_filter_ws", C.byref(d), p(xd), p(dyd), p(dw), p(ws), need, stream())
            else:
                L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dyd), p(dw), stream())
            torch.cuda.synchronize()
        finally:
            L.call("rn_set_tuning", 19, 0)
        outs.append(dw.cpu().numpy().reshape(k, r, r, c // g).transpose(0, 3, 1, 2).astype(np.float64))
    assert np.array_equal(outs[0], outs[1])
    cond = np.abs(outs[0] - dw_ref) / (dw_abs + 1e-30)
    assert cond.max() < 2e-6, cond.max()
    assert np.abs(outs[0] - outs[2]).max() <= 1e-5 * np.abs(dw_abs).max()


@pytest.mark.parametrize("case", [
    (3, 128, 9, 11, 128, 1, 2, 0),    # 128 columns, stride 2: the 128 x 128 tile (wgrad_big_kernel<128, 2, 128>)
    (3, 64, 13, 11, 64, 1, 1, 0),     # the streaming kernel (wgrad_stream_kernel<64, 64>), ragged M
    (2, 64, 9, 9, 256, 1, 1, 0),      # streaming, stage 1's conv3 / shortcut shape
    (2, 256, 9, 10, 64, 1, 1, 0),     # streaming, stage 1's conv1 shape
    (2, 256, 5, 7, 128, 1, 1, 0),     # streaming, stage 2's first conv1
    (2, 256, 14, 14, 512, 1, 1, 0),   # 256-column tiles, 256-row k tiles
    (2, 512, 7, 9, 128, 1, 1, 0),     # 256-column tiles, 128-row k tiles
    (2, 256, 14, 14, 1024, 1, 2, 0),  # the stride-2 shortcut
    (3, 128, 13, 10, 128, 3, 1, 1),   # a 3x3 gather with halo (9 x 128 columns)
    (2, 256, 15, 14, 256, 3, 2, 1),   # a stage's first 3x3, stride 2, odd rows
    (2, 48, 9, 9, 192, 3, 1, 1),      # 3 16-channel chunks per tap, k past the last 128-row tile
])
def test_wgrad_int8_codes(gpu, case):
    """rn_conv_bwd_filter_i8: the weight gradient of an int8 convolution from its input's int8 codes
    (symbol/resnet_int8.py: MXNet multiplies dy by the fake-quantized values unit * code): the codes
    staged as bytes, read with the transposed byte reads and widened to bf16, the unit applied once.
    Against the fp64 oracle of dy and unit * code (fp32 accumulation of exact products, one rounding of
    the unit: 2e-6 of the sum of the terms' magnitudes), bit-identical run to run (split slabs)."""
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(12)
    codes = rng.integers(-127, 128, size=(n, c, h, w)).astype(np.int8)
    codes[0, :, 0, :] = 127   # the extremes
    codes[-1, :, -1, :] = -127
    unit = np.float32(0.0137)
    x = codes.astype(np.float64) * float(unit)
    ho, wo = (h + 2 * pd - r) // st + 1, (w + 2 * pd - r) // st + 1
    dy = bf16_round(rng.standard_normal((n, k, ho, wo)))
    _, dw_ref = ops.conv2d_bwd(x, np.zeros((k, c, r, r)), dy, (st, st), (pd, pd))
    dw_abs = ops.conv2d_bwd(np.abs(x), np.zeros((k, c, r, r)), np.abs(dy), (st, st), (pd, pd))[1]
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    lib = L.load()
    assert lib.rn_conv_wgrad_i8_supported(C.byref(d)) == 1
    need = lib.rn_conv_wgrad_i8_ws_bytes(C.byref(d))
    assert need >= k * r * r * c * 4
    ws = torch.full((need // 4 + 4,), float("nan"), dtype=torch.float32, device=gpu)
    xd = torch.from_numpy(np.ascontiguousarray(codes.transpose(0, 2, 3, 1))).to(gpu)
    ud = torch.tensor([unit], dtype=torch.float32, device=gpu)
    dyd = to_nhwc(dy, BF16, gpu)
    outs = []
    for _ in range(2):
        dw = torch.zeros(k * r * r * c, dtype=torch.float32, device=gpu)
        L.call("rn_conv_bwd_filter_i8", C.byref(d), p(xd), p(ud), p(dyd), p(dw), p(ws), need, stream())
        torch.cuda.synchronize()
        outs.append(dw.cpu().numpy().reshape(k, r, r, c).transpose(0, 3, 1, 2).astype(np.float64))
    assert np.array_equal(outs[0], outs[1])
    cond = np.abs(outs[0] - dw_ref) / (dw_abs + 1e-30)
    assert cond.max() < 2e-6, cond.max()


def test_wgrad_int8_codes_unsupported(gpu):
    """Shapes the int8-codes weight gradient does not cover (<= 64 output channels off the streaming
    kernel, stage 1's 3x3 image-band kernel; channels not in 16-byte chunks) report 0 and the call fails
    with an error, never a launch."""
    lib = L.load()
    for n, c, h, w, k, r, st, pd in ((2, 256, 8, 8, 64, 1, 2, 0), (2, 64, 8, 8, 64, 3, 1, 1), (2, 24, 8, 8, 128, 3, 1, 1)):
        d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
        assert lib.rn_conv_wgrad_i8_supported(C.byref(d)) == 0
        assert lib.rn_conv_wgrad_i8_ws_bytes(C.byref(d)) == -1
        dummy = torch.zeros(16, dtype=torch.float32, device=gpu)
        assert lib.rn_conv_bwd_filter_i8(C.byref(d), p(dummy), p(dummy), p(dummy), p(dummy), None, 0, stream()) != 0


@pytest.mark.parametrize("persist", [0, 1])
@pytest.mark.parametrize("case", [
    (3, 64, 56, 56, 64, 3, 1, 1),    # stage 1's conv2 (several bands per workgroup)
    (5, 64, 9, 13, 64, 3, 1, 1),     # odd rows: the last band has one output row
    (1, 64, 7, 7, 64, 3, 1, 1),      # fewer pixels than one band's blocks
    (2, 64, 20, 56, 64, 3, 1, 1),    # the widest row
])
def test_conv3x3_band(gpu, case, persist):
    """conv3x3c64_band_kernel (image bands in LDS, all nine taps' weights resident; the default for a
    3x3 / stride-1 / pad-1 64 -> 64 convolution, rn_set_tuning 26 = 1 the implicit-GEMM tile) for the
    forward and the data gradient, against the fp32 reference and the implicit-GEMM tile. persist = 1: a
    batch large enough that every workgroup walks several bands (the double-buffered band loads)."""
    n, c, h, w, k, r, st, pd = case
    if persist:
        n = 40
    x, wt = _conv_data((n, c, h, w, k, r, st, pd), 23)
    x, wt = bf16_round(x), bf16_round(wt)
    dy = bf16_round(np.random.default_rng(24).standard_normal((n, k, h, w)))
    ref = ops.conv2d_fwd(x, wt, (st, st), (pd, pd))
    dx_ref, _ = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd))
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    wk = torch.zeros(k * r * r * d.c, dtype=torch.bfloat16, device=gpu)
    wc = torch.zeros(d.c * r * r * d.k_pad, dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), p(wc), stream())
    xd, dyd = to_nhwc(x, BF16, gpu), to_nhwc(dy, BF16, gpu)
    outs = []
    try:
        for mode in (0, 1):
            L.call("rn_set_tuning", 26, mode)
            y = torch.full((n, h, w, 64), float("nan"), dtype=torch.bfloat16, device=gpu)
            dx = torch.full((n, h, w, 64), float("nan"), dtype=torch.bfloat16, device=gpu)
            L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(y), BF16, None, None, stream())
            L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(dx), None, stream())
            torch.cuda.synchronize()
            outs.append((y, dx))
    finally:
        L.call("rn_set_tuning", 26, 0)
    for y, dx in outs:
        assert not torch.isnan(y).any() and not torch.isnan(dx).any()
        assert rel_err(from_nhwc(y, k), ref) < TOL[BF16]
        assert rel_err(from_nhwc(dx, c), dx_ref) < TOL[BF16]
    assert rel_err(from_nhwc(outs[1][0], k), from_nhwc(outs[0][0], k)) < 1e-2
    assert rel_err(from_nhwc(outs[1][1], c), from_nhwc(outs[0][1], c)) < 1e-2


@pytest.mark.parametrize("case", [
    (5, 64, 9, 13, 64, 3, 1, 1),     # ragged: odd rows, the last band has one output row
    (40, 64, 20, 20, 64, 3, 1, 1),   # every workgroup walks several bands (double-buffered band loads)
])
def test_conv3x3_band_bnrelu_on_load(gpu, case):
    """conv3x3c64_band_kernel<0, 1> (the producing BatchNorm+ReLU applied to each landed band in
    LDS, the zero halo kept) == rn_bn_apply's output through the plain band kernel, BIT FOR BIT; the same
    for the implicit-GEMM tile (rn_set_tuning 26 = 1), and the two forms within the bf16 bar of each other
    and of the oracle on the bf16-rounded BN+ReLU output."""
    n, c, h, w, k, r, st, pd = case
    x, wt = _conv_data(case, 31)
    rng = np.random.default_rng(32)
    sc = rng.uniform(0.5, 1.5, c)
    sh = rng.standard_normal(c) * 0.5
    x, wt = bf16_round(x), bf16_round(wt)
    xa = bf16_round(np.maximum(x * sc[None, :, None, None] + sh[None, :, None, None], 0))
    y_ref = ops.conv2d_fwd(xa, wt, (st, st), (pd, pd))
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    f = lambda a: torch.tensor(a, dtype=torch.float32, device=gpu)
    scd, shd = f(sc), f(sh)
    xd = to_nhwc(x, BF16, gpu)
    bd = L.BNDesc(dtype=BF16, m=n * h * w, c=d.c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    xad = torch.zeros_like(xd)  # the unfused path: rn_bn_apply's stored BN+ReLU output
    L.call("rn_bn_apply", C.byref(bd), p(xd), p(xad), p(scd), p(shd), stream())
    wk = torch.zeros(k * r * r * d.c, dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), p(wk), None, stream())
    outs = []
    try:
        for mode in (0, 1):
            L.call("rn_set_tuning", 26, mode)
            y1 = torch.full((n, h, w, k), float("nan"), dtype=torch.bfloat16, device=gpu)
            y0 = torch.full_like(y1, float("nan"))
            L.call("rn_conv_fwd_x", C.byref(d), p(xd), p(wk), p(y1), BF16, None, None, p(scd), p(shd), None, stream())
            L.call("rn_conv_fwd", C.byref(d), p(xad), p(wk), p(y0), BF16, None, None, stream())
            torch.cuda.synchronize()
            assert torch.equal(y1.view(torch.int16), y0.view(torch.int16)), mode
            outs.append(y1)
    finally:
        L.call("rn_set_tuning", 26, 0)
    for y in outs:
        assert rel_err(from_nhwc(y, k), y_ref) < TOL[BF16]
    assert rel_err(from_nhwc(outs[0], k), from_nhwc(outs[1], k)) < 1e-2



@pytest.mark.parametrize("width", [0, 2], ids=["cpw64", "cpw32"])
@pytest.mark.parametrize("mode", ["reduce", "reduce_add", "reduce_only", "norelu", "apply", "apply_add"])
@pytest.mark.parametrize("case", [
    (3, 256, 14, 14, 64, 1, 1, 0),     # stage-1 conv1's data gradient (K = 64 into 256)
    (2, 512, 9, 11, 128, 1, 1, 0),     # stage-2 conv1 (K = 128 into 512), ragged last row block
    (5, 128, 7, 9, 64, 1, 1, 0),       # one 128-channel group, fewer rows than a block
])
def test_dgrad1x1_stream(gpu, case, mode, width):
    """dgrad1x1_stream_kernel (the pre-activation units' conv1 data gradients streamed with the weights in
    registers, with the BN-backward reduction or the BN backward applied; rn_set_tuning 27 = 1: the 224-row
    tiles, 27 = 2: 32 channels per wave) against the tiles: dx BIT FOR BIT (the same MFMA
    sums), the BN-backward partials' per-channel totals within fp32 summation-order rounding, and the
    oracle's conv dgrad + BN(+ReLU) backward within the bf16 bar."""
    n, c, h, w, k, r, st, pd = case
    rng = np.random.default_rng(51)
    d = conv_desc(BF16, n, c, h, w, k, r, r, st, pd)
    xb = bf16_round(rng.standard_normal((n, c, h, w)) * 1.5 + 0.3)
    wt = bf16_round(rng.standard_normal((k, c, r, r)) / np.sqrt(c * r * r))
    dy = bf16_round(rng.standard_normal((n, k, h, w)))
    res = bf16_round(rng.standard_normal((n, c, h, w)) * 0.5)
    lib = L.load()
    wc = torch.zeros(d.c * d.k_pad, dtype=torch.bfloat16, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(_master_krsc(wt, gpu)), None, p(wc), stream())
    f = lambda a: torch.tensor(np.asarray(a, np.float64), dtype=torch.float32, device=gpu)
    mean, sc, sh = f(rng.standard_normal(c) * 0.2), f(rng.uniform(0.5, 1.5, c)), f(rng.standard_normal(c) * 0.3)
    coef = f(np.stack([rng.uniform(0.5, 1.5, c), rng.standard_normal(c) * 0.1, rng.standard_normal(c) * 0.05,
                       rng.standard_normal(c) * 0.2], 1).ravel())
    xbd, dyd, resd = to_nhwc(xb, BF16, gpu), to_nhwc(dy, BF16, gpu), to_nhwc(res, BF16, gpu)
    nrb = lib.rn_conv_bnred_blocks(C.byref(d))
    assert nrb == -(-n * h * w // 224)
    relu = 0 if mode == "norelu" else 1
    add = resd if mode.endswith("_add") else None
    outs = []
    try:
        for val in (1, width):  # the tiles, then the streaming kernel
            L.call("rn_set_tuning", 27, val)
            part = torch.full((nrb * d.c * 2,), float("nan"), dtype=torch.float32, device=gpu)
            dx = None if mode == "reduce_only" else torch.full_like(xbd, float("nan"))
            if mode.startswith("apply"):
                L.call("rn_conv_bwd_data_bnapply", C.byref(d), p(dyd), p(wc), p(dx), p(add), p(xbd), p(coef), p(sc),
                       p(sh), relu, stream())
            else:
                L.call("rn_conv_bwd_data_bnred", C.byref(d), p(dyd), p(wc), p(dx), p(add), p(xbd), p(mean), p(sc),
                       p(sh), relu, p(part), stream())
            torch.cuda.synchronize()
            outs.append((dx, part))
    finally:
        L.call("rn_set_tuning", 27, 0)
    (dx0, p0), (dx1, p1) = outs
    if dx0 is not None:
        assert not torch.isnan(dx1).any()
        assert torch.equal(dx0.view(torch.int16), dx1.view(torch.int16))
    if mode.startswith("reduce") or mode == "norelu":
        assert not torch.isnan(p1).any()
        t0 = p0.view(nrb, d.c, 2).double().sum(0)
        t1 = p1.view(nrb, d.c, 2).double().sum(0)
        assert torch.allclose(t0, t1, rtol=1e-4, atol=1e-4 * float(t0.abs().max()))
        # the oracle: dz = bf16(dgrad (+ add)) [x sc + sh > 0], sums of dz and dz (x - mean)
        dact, _ = ops.conv2d_bwd(xb, wt, dy, (1, 1), (0, 0))
        g = bf16_round(dact + (res if add is not None else 0))
        xs = xb * sc.cpu().numpy()[None, :, None, None] + sh.cpu().numpy()[None, :, None, None]
        dz = g * (xs > 0) if relu else g
        ref_s = dz.sum((0, 2, 3))
        ref_q = (dz * (xb - mean.cpu().numpy()[None, :, None, None])).sum((0, 2, 3))
        assert rel_err(t1[:, 0].cpu().numpy(), ref_s) < 1e-2 and rel_err(t1[:, 1].cpu().numpy(), ref_q) < 1e-2
