"""The oracle (oracle/ops.py, oracle/net.py) against an independent torch-CPU fp64 restatement.

torch.nn.functional + autograd computes every op and the whole-network gradient in fp64; the
numpy oracle's hand-written backward must agree to ~1e-10. This is how the oracle is pinned
while MXNet itself is unavailable (parity vs MXNet is unpinned; see oracle/__init__.py).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import net as onet
from oracle import ops
from torch_ref import T, torch_net_grads as _torch_net_grads


@pytest.mark.parametrize("case", [(2, 6, 9, 7, 4, 3, 2, 1, 1), (1, 8, 8, 8, 16, 1, 1, 0, 1), (2, 8, 10, 10, 8, 3, 1, 1, 4),
                                  (1, 3, 15, 15, 5, 7, 2, 3, 1)])
def test_conv(case):
    n, c, h, w, k, r, st, pd, g = case
    rng = np.random.default_rng(0)
    x = rng.standard_normal((n, c, h, w))
    wt = rng.standard_normal((k, c // g, r, r))
    y = ops.conv2d_fwd(x, wt, (st, st), (pd, pd), g)
    xt, wtt = T(x, True), T(wt, True)
    yt = F.conv2d(xt, wtt, stride=st, padding=pd, groups=g)
    np.testing.assert_allclose(y, yt.detach().numpy(), rtol=1e-10, atol=1e-10)
    dy = rng.standard_normal(y.shape)
    yt.backward(T(dy))
    dx, dw = ops.conv2d_bwd(x, wt, dy, (st, st), (pd, pd), g)
    np.testing.assert_allclose(dx, xt.grad.numpy(), rtol=1e-10, atol=1e-10)
    np.testing.assert_allclose(dw, wtt.grad.numpy(), rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("fix_gamma", [False, True])
def test_batchnorm(fix_gamma):
    rng = np.random.default_rng(1)
    x = rng.standard_normal((3, 5, 4, 6)) * 3 + 1
    gamma, beta = rng.uniform(0.5, 2, 5), rng.standard_normal(5)
    y, cache = ops.bn_train_fwd(x, gamma, beta, 1e-5, fix_gamma)
    xt = T(x, True)
    gt = T(np.ones(5) if fix_gamma else gamma, True)
    bt = T(beta, True)
    yt = F.batch_norm(xt, None, None, gt, bt, training=True, eps=1e-5)
    np.testing.assert_allclose(y, yt.detach().numpy(), rtol=1e-10, atol=1e-10)
    dy = rng.standard_normal(x.shape)
    yt.backward(T(dy))
    dx, dg, db = ops.bn_train_bwd(dy, cache, fix_gamma)
    np.testing.assert_allclose(dx, xt.grad.numpy(), rtol=1e-9, atol=1e-10)
    np.testing.assert_allclose(db, bt.grad.numpy(), rtol=1e-10)
    if fix_gamma:
        assert np.all(dg == 0)
    else:
        np.testing.assert_allclose(dg, gt.grad.numpy(), rtol=1e-9)
    # moving stats: biased variance
    mm, mv = ops.bn_moving_update(np.zeros(5), np.ones(5), cache[3], cache[4], 0.9)
    np.testing.assert_allclose(mv, 0.9 + 0.1 * x.var(axis=(0, 2, 3)))


def test_maxpool_first_max_rule():
    rng = np.random.default_rng(2)
    x = np.round(np.maximum(rng.standard_normal((2, 3, 9, 9)), 0) * 2) / 2  # many ties
    y, arg = ops.maxpool_fwd(x, (3, 3), (2, 2), (1, 1))
    yt = F.max_pool2d(T(x), 3, 2, 1)
    np.testing.assert_array_equal(y, yt.numpy())
    dy = rng.standard_normal(y.shape)
    dx = ops.maxpool_bwd(dy, arg, x.shape, (3, 3), (2, 2), (1, 1))
    # brute force: gradient to the first maximal element of each window in (r, s) scan order
    ref = np.zeros_like(x)
    for nn in range(2):
        for cc in range(3):
            for p in range(y.shape[2]):
                for q in range(y.shape[3]):
                    best, pos = -np.inf, None
                    for r in range(3):
                        for s in range(3):
                            hh, ww = 2 * p - 1 + r, 2 * q - 1 + s
                            if 0 <= hh < 9 and 0 <= ww < 9 and x[nn, cc, hh, ww] > best:
                                best, pos = x[nn, cc, hh, ww], (hh, ww)
                    ref[nn, cc, pos[0], pos[1]] += dy[nn, cc, p, q]
    np.testing.assert_allclose(dx, ref, rtol=1e-12, atol=1e-12)


def test_softmax_fc():
    rng = np.random.default_rng(3)
    x, w, b = rng.standard_normal((5, 7)), rng.standard_normal((4, 7)), rng.standard_normal(4)
    z = ops.fc_fwd(x, w, b)
    p = ops.softmax_output_fwd(z)
    lab = np.array([0, 3, 1, 2, 3], dtype=np.float32)
    xt, wt, bt = T(x, True), T(w, True), T(b, True)
    loss = F.cross_entropy(F.linear(xt, wt, bt), torch.tensor(lab.astype(np.int64)), reduction="sum")
    loss.backward()
    g = ops.softmax_output_bwd(p, lab)  # SoftmaxOutput grad = d(sum CE)/dz ('null' normalization)
    dx, dw, db = ops.fc_bwd(x, w, g)
    np.testing.assert_allclose(dx, xt.grad.numpy(), rtol=1e-10)
    np.testing.assert_allclose(dw, wt.grad.numpy(), rtol=1e-10)
    np.testing.assert_allclose(db, bt.grad.numpy(), rtol=1e-10)
    assert abs(ops.cross_entropy(p, lab) - loss.item()) < 1e-10


def test_sgd_momentum_form():
    w, g, m = np.array([1.0, -2.0]), np.array([0.5, 0.25]), np.array([0.1, 0.0])
    ops.sgd_mom_update(w, g, m, lr=0.1, wd=0.01, momentum=0.9, rescale_grad=0.5)
    mom = 0.9 * np.array([0.1, 0.0]) - 0.1 * (0.5 * np.array([0.5, 0.25]) + 0.01 * np.array([1.0, -2.0]))
    np.testing.assert_allclose(m, mom)
    np.testing.assert_allclose(w, np.array([1.0, -2.0]) + mom)
    assert ops.wd_mult_for("conv0_weight") == 1 and ops.wd_mult_for("bn0_gamma") == 1
    assert ops.wd_mult_for("bn0_beta") == 0 and ops.wd_mult_for("fc1_bias") == 0


def test_mx_round_half_away():
    np.testing.assert_array_equal(ops.mx_round(np.array([0.5, 1.5, 2.5, -0.5, -2.5])), [1, 2, 3, -1, -3])


@pytest.mark.parametrize("which", ["resnet20", "resnet_tiny_v2", "resnext_tiny"])
def test_network_gradients_vs_torch_autograd(which):
    if which == "resnet20":
        g = onet.resnet20_cifar()
        shape, ncls = (3, 16, 16), 10
    elif which == "resnet_tiny_v2":
        g = onet.resnet([1, 1], 2, [8, 16, 32], 6, bottle_neck=True, dataset="imagenet")
        shape, ncls = (3, 32, 32), 6
    else:
        g = onet.resnext([1, 1], 2, [8, 64, 128], 6, num_group=32)
        shape, ncls = (3, 32, 32), 6
    args, aux = onet.init_params(g, seed=4)
    data, label = onet.synthetic_batch(3, shape, ncls)
    prob, st = onet.forward(g, args, aux, data, label)
    grads = onet.backward(g, args, st)
    ref = _torch_net_grads(g, args, data, label)
    for k in g.params:
        np.testing.assert_allclose(grads[k], ref[k], rtol=1e-7, atol=1e-9, err_msg=k)


def test_schedulers():
    s = ops.WarmupMultiFactorScheduler(0.8, [100, 200], 0.1, True, "gradual", 0.1, 50)
    assert abs(s(1) - (0.7 / 50 + 0.1)) < 1e-12
    assert abs(s(50) - 0.8) < 1e-12
    assert s(100) == 0.8 and abs(s(101) - 0.08) < 1e-12 and abs(s(201) - 0.008) < 1e-12
    m = ops.MultiFactorScheduler([10, 20], 0.5, base_lr=1.0)
    assert m(10) == 1.0 and m(11) == 0.5 and m(21) == 0.25


def test_data_parallel_split_semantics():
    """Even batch split: per-slice BN stats, summed grads -- differs from one big batch."""
    g = onet.resnet([1], 1, [8, 16], 4, bottle_neck=False, dataset="cifar10")
    args, aux = onet.init_params(g)
    data, label = onet.synthetic_batch(4, (3, 8, 8), 4)
    a1 = {k: v.copy() for k, v in args.items()}
    m1 = {k: np.zeros_like(v) for k, v in args.items()}
    _, g2, auxes = onet.train_step(g, a1, aux, m1, data, label, 0.1, num_devices=2)
    gsum = {}
    for d in range(2):
        _, st = onet.forward(g, args, {k: v.copy() for k, v in aux.items()}, data[2 * d:2 * d + 2],
                             label[2 * d:2 * d + 2])
        for k, v in onet.backward(g, args, st).items():
            gsum[k] = gsum.get(k, 0) + v
    for k in gsum:
        np.testing.assert_allclose(g2[k], gsum[k], rtol=1e-12, atol=1e-14)
    assert len(auxes) == 2
