"""Whole-network training-step parity: mxnet shim + librn on the GPU vs the numpy oracle.

Same initial parameters, same seeded synthetic batch (data/imagenet.py:15-18 restated), one or
two Solver steps (forward(is_train) -> backward -> SGD update, core/solver.py:115-121).
Tolerances (max |err| / max |ref| per tensor), fp32 runtime path: probs 1e-4, grads 2e-3,
updated params 1e-5, moving stats 1e-4. bf16 path: probs 5e-2 and gradient direction cosine > 0.98.
"""
import numpy as np
import pytest

from oracle import net as onet
from step_util import max_rel, module_step, oracle_state, oracle_step

pytestmark = pytest.mark.gpu


def _check(res, ref, tol_p=1e-4, tol_g=2e-3, tol_w=1e-5, tol_a=1e-4, step=0):
    assert max_rel(res["prob"][step], ref["prob"][step]) < tol_p
    worst = max((max_rel(res["grads"][step][n], ref["grads"][step][n]), n) for n in ref["grads"][step])
    assert worst[0] < tol_g, worst
    worst = max((max_rel(res["args"][n], ref["args"][n]), n) for n in ref["args"])
    assert worst[0] < tol_w, worst
    worst = max((max_rel(res["aux"][n], ref["aux"][n]), n) for n in ref["aux"])
    assert worst[0] < tol_a, worst


def test_resnet20_cifar_fp32_two_steps(gpu):
    from rn import graphs
    g = onet.resnet20_cifar()
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(8, (3, 32, 32), 10)
    ref = oracle_step(g, args, aux, data, label, steps=2)
    res = module_step(graphs.resnet20_cifar(), args, aux, data, label, "float32", steps=2)
    _check(res, ref, step=0)
    assert max_rel(res["prob"][1], ref["prob"][1]) < 1e-4


def test_resnet50_fp32_small(gpu):
    from rn import graphs
    g = onet.resnet50_imagenet(num_classes=16)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(2, (3, 64, 64), 16)
    ref = oracle_step(g, args, aux, data, label)
    res = module_step(graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16), args, aux, data, label,
                      "float32")
    _check(res, ref)


def test_resnet50_bf16_small(gpu):
    from rn import graphs
    g = onet.resnet50_imagenet(num_classes=16)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    ref = oracle_step(g, args, aux, data, label)
    res = module_step(graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16), args, aux, data, label,
                      "bfloat16")
    assert max_rel(res["prob"][0], ref["prob"][0]) < 5e-2
    for n, gref in ref["grads"][0].items():
        a, b = res["grads"][0][n].ravel(), gref.ravel()
        if np.abs(b).max() == 0:
            continue
        cos = float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))
        assert cos > 0.98, (n, cos)
