"""Deterministic weight-gradient mode (rn_set_tuning 17 / RN_DETERMINISTIC=1): every
M-split of a weight gradient stores its partial into the workspace slab and one pass sums the splits
in a fixed order, instead of fp32 atomic adds (core/solver.py:115-121's backward, reproducible).

* per kernel: the weight gradient of dense, padded-channel (stem), grouped and FullyConnected
  shapes, fp32 and bf16, is bitwise the same over repeated launches and matches the oracle;
* whole step: ResNet-50 v2 fp32 (symbol/resnet.py, full [3,4,6,3] units at 64x64) run twice gives
  bitwise identical gradients, and -- WITHOUT replaying the device's ReLU decisions into the oracle --
  its distance to the fp64 oracle (ReLU decisions flipped, gradient errors) lies within the spread
  numpy fp32 itself shows against fp64 on the same step.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import net as onet
from oracle import ops
from rn import lib as L
from gpu_util import BF16, F32, bf16_round, conv_desc, p, rel_err, stream, to_nhwc
from step_util import fro_rel, max_rel, module_step, oracle_state, oracle_step

pytestmark = pytest.mark.gpu


@pytest.fixture
def deterministic():
    L.call("rn_set_tuning", 17, 1)
    yield
    L.call("rn_set_tuning", 17, 0)


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", [
    (8, 64, 28, 28, 128, 3, 1, 1, 1),      # dense 3x3 (register-staged / LDS-DMA tiles)
    (16, 256, 14, 14, 512, 1, 2, 0, 1),    # 1x1 stride 2, large M split
    (4, 3, 32, 32, 64, 7, 2, 3, 1),        # padded channels (the stem's 3 of 8)
    (4, 128, 14, 14, 128, 3, 1, 1, 32),    # grouped (ResNeXt 32 x 4)
    (32, 2048, 1, 1, 1000, 1, 1, 0, 1),    # FullyConnected as a 1x1 conv
])
def test_wgrad_deterministic(gpu, deterministic, dtype, case):
    n, c, h, w, k, r, st, pd, g = case
    rng = np.random.default_rng(7)
    x = rng.standard_normal((n, c, h, w))
    wt = rng.standard_normal((k, c // g, r, r)) / np.sqrt(c // g * r * r)
    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd, groups=g)
    dy = rng.standard_normal((n, k, d.p, d.q))
    if dtype == BF16:
        x, dy = bf16_round(x), bf16_round(dy)
    _, dw_ref = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd), groups=g) if g > 1 else \
        ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd))
    lib = L.load()
    need = int(lib.rn_conv_wgrad_ws_bytes(C.byref(d)))
    assert need > 0, "the deterministic mode always stores slabs"
    ws = torch.empty(need // 4, dtype=torch.float32, device=gpu)
    xd, dyd = to_nhwc(x, dtype, gpu), to_nhwc(dy, dtype, gpu)
    outs = []
    for _ in range(3):
        dw = torch.zeros(k * r * r * (c // g), dtype=torch.float32, device=gpu)
        ws.fill_(float("nan"))  # every slab element of every split is written before it is read
        L.call("rn_conv_bwd_filter_ws", C.byref(d), p(xd), p(dyd), p(dw), p(ws), need, stream())
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)) and torch.equal(outs[0], outs[2])
    got = outs[0].cpu().numpy().reshape(k, r, r, c // g).transpose(0, 3, 1, 2)
    assert rel_err(got, dw_ref) < (2e-5 if dtype == F32 else 5e-3)
    # without a workspace the mode refuses instead of falling back to atomics
    assert lib.rn_conv_bwd_filter_ws(C.byref(d), p(xd), p(dyd), p(outs[0]), None, 0, stream()) != 0


def _oracle_masks(g, args, aux, data, label, dtype):
    a = {k: v.astype(dtype) for k, v in args.items()}
    x = {k: v.astype(dtype).copy() for k, v in aux.items()}
    _, st = onet.forward(g, a, x, data.astype(dtype), label, True)
    return {t["op"]["name"]: np.asarray(t["mask"], bool) for t in st["tape"] if "mask" in t}


def test_resnet50_fp32_deterministic_unreplayed(gpu, deterministic):
    """At this size a few pre-activations lie within fp32 rounding of zero (numpy fp32 flips 2 of
    3.2 M ReLU decisions of the fp64 run with init seed 7), and one flip moves every upstream gradient
    by ~1 %. So without replay the bar is the spread numpy fp32 itself shows against fp64: the device
    may flip about as many decisions, and its per-tensor gradient errors (median and worst) must lie
    within 4x numpy fp32's (plus a 1e-4 floor)."""
    from rn import graphs
    g = onet.resnet50_imagenet(num_classes=16)
    args, aux = oracle_state(g, seed=7)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    sym = lambda: graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16)
    r1 = module_step(sym(), args, aux, data, label, "float32")
    r2 = module_step(sym(), args, aux, data, label, "float32")
    for n in r1["grads"][0]:
        assert np.array_equal(r1["grads"][0][n], r2["grads"][0][n]), n  # bitwise reproducible
    assert np.array_equal(r1["prob"][0], r2["prob"][0])

    # ReLU decisions: the fp64 oracle's own vs numpy fp32's and the device's (no replay anywhere)
    m64 = _oracle_masks(g, args, aux, data, label, np.float64)
    m32 = _oracle_masks(g, args, aux, data, label, np.float32)
    flips32 = sum(int((m32[k] != m64[k]).sum()) for k in m64)
    assert set(m64) <= set(r1["relu_masks"][0])
    flips_dev = sum(int((r1["relu_masks"][0][k] != m64[k]).sum()) for k in m64)
    ref = oracle_step(g, args, aux, data, label)
    r32 = oracle_step(g, args, aux, data, label, dtype=np.float32)
    e_dev = {n: fro_rel(r1["grads"][0][n], ref["grads"][0][n]) for n in ref["grads"][0]}
    e32 = {n: fro_rel(r32["grads"][0][n], ref["grads"][0][n]) for n in ref["grads"][0]}
    med = lambda d: float(np.median(list(d.values())))
    print("ReLU decisions differing from fp64 (of %d): numpy fp32 %d, device %d" %
          (sum(v.size for v in m64.values()), flips32, flips_dev))
    print("gradient error vs fp64, unreplayed: device median %.2e max %.2e; numpy fp32 median %.2e max %.2e"
          % (med(e_dev), max(e_dev.values()), med(e32), max(e32.values())))
    print("probabilities: device %.2e, numpy fp32 %.2e" % (max_rel(r1["prob"][0], ref["prob"][0]),
                                                           max_rel(r32["prob"][0], ref["prob"][0])))
    assert flips_dev <= 4 * max(flips32, 1)
    assert med(e_dev) <= max(1e-4, 4 * med(e32))
    assert max(e_dev.values()) <= max(1e-4, 4 * max(e32.values()))
    assert max_rel(r1["prob"][0], ref["prob"][0]) <= max(1e-4, 4 * max_rel(r32["prob"][0], ref["prob"][0]))


@pytest.mark.parametrize("dtype", [F32, BF16])
@pytest.mark.parametrize("case", [
    (8, 64, 28, 28, 128, 3, 1, 1, 1),
    (16, 256, 14, 14, 512, 1, 2, 0, 1),
    (4, 3, 32, 32, 64, 7, 2, 3, 1),
    (4, 128, 14, 14, 128, 3, 1, 1, 32),
    (32, 2048, 1, 1, 1000, 1, 1, 0, 1),
    (64, 64, 56, 56, 64, 1, 1, 0, 1),      # many splits (> 16: the general kernel in both modes)
    (16, 64, 14, 14, 64, 3, 1, 1, 1),      # image bands: one split per image, exactly 16
    (16, 64, 14, 14, 64, 3, 1, 1, -1),     # the same onto a -0 start (zero signs compared too)
])
def test_slab_reduce_few_splits_bitwise(gpu, deterministic, dtype, case):
    """rn_set_tuning 25: the few-split slab reduction (one thread per 16-byte column, <= 16 splits)
    stores exactly the general kernel's sums, bit for bit including the sign of zero (dw accumulated
    into: += onto a nonzero start; g = -1: a -0 start)."""
    n, c, h, w, k, r, st, pd, g = case
    negzero = g < 0
    g = abs(g)
    rng = np.random.default_rng(11)
    x = rng.standard_normal((n, c, h, w))
    d = conv_desc(dtype, n, c, h, w, k, r, r, st, pd, groups=g)
    dy = rng.standard_normal((n, k, d.p, d.q))
    if dtype == BF16:
        x, dy = bf16_round(x), bf16_round(dy)
    lib = L.load()
    need = int(lib.rn_conv_wgrad_ws_bytes(C.byref(d)))
    ws = torch.empty(need // 4, dtype=torch.float32, device=gpu)
    xd, dyd = to_nhwc(x, dtype, gpu), to_nhwc(dy, dtype, gpu)
    start = torch.tensor(rng.standard_normal(k * r * r * (c // g)), dtype=torch.float32, device=gpu)
    if negzero:
        start = torch.full_like(start, -0.0)
    if dtype == BF16 and case[0] == 16 and case[1] == 64 and case[4] == 64:
        assert need == 16 * k * r * r * c * 4  # 16 splits, the few-split kernel's limit
    outs = []
    try:
        for mode in (1, 0):
            L.call("rn_set_tuning", 25, mode)
            dw = start.clone()
            ws.fill_(float("nan"))
            L.call("rn_conv_bwd_filter_ws", C.byref(d), p(xd), p(dyd), p(dw), p(ws), need, stream())
            outs.append(dw)
        torch.cuda.synchronize()
    finally:
        L.call("rn_set_tuning", 25, 0)
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
