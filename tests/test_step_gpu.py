"""Whole-network training-step parity: mxnet shim + librn on the GPU vs the numpy oracle.

Same initial parameters, same seeded synthetic batch (data/imagenet.py:15-18 restated), one or
two Solver steps (forward(is_train) -> backward -> SGD update, core/solver.py:115-121).
Tolerances (max |err| / max |ref| per tensor):
  ResNet-20 fp32: probs 1e-4, grads 2e-3, updated params 1e-5, moving stats 1e-4.
  ResNet-50 fp32: probs 1e-4, loss 1e-5. At this small spatial size a single ReLU decision
    that flips under fp32 rounding (e.g. in stage4_unit3_bn2: 4x2x2 = 16 elements per channel)
    moves every upstream gradient by ~1/sqrt(8192) = 1.1% -- numpy fp32 vs fp64 shows the same
    chaos, and which elements flip depends on fp32 atomic summation order. So the oracle REPLAYS
    the ReLU decisions the device made (oracle.net.forward relu_masks); then every gradient must
    match the fp64 oracle to max(1e-4, 4x the error numpy fp32 makes on that tensor under the same
    decisions) (Frobenius-relative; only cancellation-dominated BN-gamma grads use the second term).
  ResNet-20 two steps: the same replay for step 1's decisions, step 2 compared on probs (1e-4).
  bf16 runtime path: per-kernel parity lives in test_kernels_gpu.py. Whole-network, bf16 storage
    makes tiny-config gradients noise-dominated (also in the oracle's bf16-storage emulation),
    so the checks are: first-step loss within 2% of the fp64 oracle, and 4 SGD steps on a fixed
    batch decrease the loss monotonically (ResNet-20 below 80% / ResNet-50 below 50% of the start).
"""
import numpy as np
import pytest

from oracle import net as onet
from step_util import ce_loss, fro_rel, max_rel, module_step, oracle_state, oracle_step, replayed_parity

pytestmark = pytest.mark.gpu


def _check(res, ref, tol_p=1e-4, tol_g=2e-3, tol_w=1e-5, tol_a=1e-4, step=0):
    assert max_rel(res["prob"][step], ref["prob"][step]) < tol_p
    worst = max((max_rel(res["grads"][step][n], ref["grads"][step][n]), n) for n in ref["grads"][step])
    assert worst[0] < tol_g, worst
    worst = max((max_rel(res["args"][n], ref["args"][n]), n) for n in ref["args"])
    assert worst[0] < tol_w, worst
    worst = max((max_rel(res["aux"][n], ref["aux"][n]), n) for n in ref["aux"])
    assert worst[0] < tol_a, worst


def _assert_replayed(errs):
    bad = {n: v for n, v in errs.items() if v[0] > v[2]}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:5]


def test_resnet20_cifar_fp32_two_steps(gpu):
    from rn import graphs
    g = onet.resnet20_cifar()
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(8, (3, 32, 32), 10)
    res = module_step(graphs.resnet20_cifar(), args, aux, data, label, "float32", steps=2)
    assert len(res["relu_masks"][0]) == 19
    errs, ref = replayed_parity(res, g, args, aux, data, label)
    _assert_replayed(errs)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    ref2 = oracle_step(g, args, aux, data, label, steps=2)
    assert max_rel(res["prob"][1], ref2["prob"][1]) < 1e-4


def test_resnet50_fp32_small(gpu):
    from rn import graphs
    g = onet.resnet50_imagenet(num_classes=16)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    res = module_step(graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16), args, aux, data, label,
                      "float32")
    assert len(res["relu_masks"][0]) == 50
    errs, ref = replayed_parity(res, g, args, aux, data, label)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    assert abs(ce_loss(res["prob"][0], label) - ce_loss(ref["prob"][0], label)) < 1e-5 * ce_loss(ref["prob"][0], label)
    _assert_replayed(errs)
    assert sum(1 for v in errs.values() if v[0] <= 1e-4) >= 150  # all but a few cancellation-dominated tensors
    # updated params inherit the gradient bar (beta_1 = -lr*g/B for zero-initialised betas)
    worst = max((fro_rel(res["args"][n], ref["args"][n]), n) for n in ref["args"])
    assert worst[0] < 1e-4, worst
    # moving means of deep-stage BN inputs are means of 16 mixed-sign values: Frobenius bar
    worst = max((fro_rel(res["aux"][n], ref["aux"][n]), n) for n in ref["aux"])
    assert worst[0] < 1e-4, worst


def _loss_traj(g, symf, n, hw, ncls, steps, lr):
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(n, (3, hw, hw), ncls)
    ref = oracle_step(g, args, aux, data, label, lr=lr, steps=steps)
    res = module_step(symf(), args, aux, data, label, "bfloat16", lr=lr, steps=steps)
    return [ce_loss(p, label) for p in res["prob"]], [ce_loss(p, label) for p in ref["prob"]]


def _check_traj(gpu_l, ref_l, final_frac):
    assert abs(gpu_l[0] - ref_l[0]) < 0.02 * ref_l[0], (gpu_l, ref_l)
    # monotone until the fixed batch is memorised (below 1e-2 bf16 rounding moves it either way)
    assert all(b < a or b < 1e-2 for a, b in zip(gpu_l, gpu_l[1:])), gpu_l
    assert gpu_l[-1] < final_frac * gpu_l[0], gpu_l


def test_resnet20_bf16_loss_trajectory(gpu):
    from rn import graphs
    gpu_l, ref_l = _loss_traj(onet.resnet20_cifar(), graphs.resnet20_cifar, 8, 32, 10, 4, 0.1)
    _check_traj(gpu_l, ref_l, 0.8)


def test_resnet50_bf16_loss_trajectory(gpu):
    from rn import graphs
    gpu_l, ref_l = _loss_traj(onet.resnet50_imagenet(16),
                              lambda: graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16), 4, 64, 16, 4, 0.05)
    _check_traj(gpu_l, ref_l, 0.5)


def _resnext_small():
    return ([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16)


def test_resnext_fp32_small(gpu):
    """ResNeXt 32x4d units (symbol/resnext.py) with one unit per stage: every grouped width
    (4/8/16/32 channels per group) through the whole step, ReLU decisions replayed."""
    from rn import graphs
    cfg = _resnext_small()
    g = onet.resnext(*cfg, num_group=32)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    res = module_step(graphs.resnext(*cfg, "float32", 32), args, aux, data, label, "float32")
    errs, ref = replayed_parity(res, g, args, aux, data, label)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    _assert_replayed(errs)
    worst = max((fro_rel(res["args"][n], ref["args"][n]), n) for n in ref["args"])
    assert worst[0] < 1e-4, worst


def test_resnext_bf16_loss_trajectory(gpu):
    from rn import graphs
    cfg = _resnext_small()
    gpu_l, ref_l = _loss_traj(onet.resnext(*cfg, num_group=32), lambda: graphs.resnext(*cfg, "float32", 32), 4, 64,
                              16, 4, 0.05)
    _check_traj(gpu_l, ref_l, 0.5)


def test_resnet_int8_fp32_small(gpu):
    """resnet_int8 (symbol/resnet_int8.py, C5) one QAT step. Rounding to the int8 grid is as
    chaotic as ReLU under fp32 vs fp64 (numpy fp32 alone moves the probabilities by 3% here), so
    the oracle replays the device's ReLU decisions AND its fake-quantized tensors (weights and
    data, oracle.net.forward quant_values); the quantizer EMA states and the STE masks are still
    computed by the oracle. Then the float-graph bar applies: probs 1e-4, gradients
    max(1e-4, 4x numpy-fp32 error) (Frobenius-relative), quantizer states 1e-6."""
    from rn import graphs
    cfg = ([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16)
    g = onet.resnet_int8(*cfg)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    res = module_step(graphs.resnet_int8(*cfg), args, aux, data, label, "float32")
    qv = res["quant_values"][0]
    assert len(qv) == 2 * 18
    errs, ref = replayed_parity(res, g, args, aux, data, label, quant_values=qv)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    _assert_replayed(errs)
    st = res["mod"].get_params()[1]
    q = {k: v.asnumpy() for k, v in st.items() if k.endswith("_data_minmax")}
    assert len(q) == 18
    for k, v in q.items():
        assert abs(v.item() - ref["quant_state"][k]) <= 1e-6 * ref["quant_state"][k], k


def test_resnet_int8_fp32_full_units(gpu):
    """resnet_int8 with the full ResNet-50 [3,4,6,3] units (the C5 graph at 64x64, batch 4): the
    same replayed parity as the one-unit case above, 53 quantized convs + fc1."""
    from rn import graphs
    cfg = ([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16)
    g = onet.resnet_int8(*cfg)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    res = module_step(graphs.resnet_int8(*cfg), args, aux, data, label, "float32")
    qv = res["quant_values"][0]
    assert len(qv) == 2 * 54
    errs, ref = replayed_parity(res, g, args, aux, data, label, quant_values=qv)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    _assert_replayed(errs)


def test_resnext50_fp32_full_units(gpu):
    """ResNeXt-50 32x4d with its full [3,4,6,3] units (the C4 graph at 64x64, batch 4), ReLU
    decisions replayed: probabilities 1e-4, every gradient max(1e-4, 4x numpy-fp32 error)."""
    from rn import graphs
    cfg = ([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16)
    g = onet.resnext(*cfg, num_group=32)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    res = module_step(graphs.resnext(*cfg, "float32", 32), args, aux, data, label, "float32")
    errs, ref = replayed_parity(res, g, args, aux, data, label)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    _assert_replayed(errs)


def test_resnet_int8_bf16_loss_trajectory(gpu):
    from rn import graphs
    cfg = ([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16)
    gpu_l, ref_l = _loss_traj(onet.resnet_int8(*cfg), lambda: graphs.resnet_int8(*cfg), 4, 64, 16, 4, 0.05)
    _check_traj(gpu_l, ref_l, 0.5)
