"""BASELINE config C1 -- ResNet-20 on CIFAR-10 through the mxnet drop-in on an mx.cpu() context (the
reference's MXNet CPU executor, train.py:34 with no GPU), against the numpy fp64 oracle.

The host executor (rn/cpu_executor.py) runs the same Plan as the GPU in torch-CPU fp32. Bars: the
same as the GPU's fp32 whole-step tests (tests/test_step_gpu.py): probabilities 1e-4; gradients
Frobenius-relative max(1e-4, 4x the error a numpy-fp32 run of the oracle makes on the same tensor,
under the same ReLU decisions) on the first step; probabilities of the second; parameters after the
first update 1e-5; BN moving statistics 1e-4.
"""
import numpy as np
import pytest

import mxnet as mx
from oracle import net as onet
from rn import graphs
from step_util import fro_rel, max_rel, oracle_step


def _module_step(sym, args, aux, data, label, steps=1, lr=0.1, ctx=None):
    mod = mx.mod.Module(sym, context=ctx if ctx is not None else mx.cpu())
    mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", label.shape)], for_training=True)
    mod.init_params(arg_params={k: v.astype(np.float32) for k, v in args.items()},
                    aux_params={k: v.astype(np.float32) for k, v in aux.items()}, allow_missing=True)
    mod.init_optimizer(kvstore="local", optimizer="sgd", optimizer_params={"learning_rate": lr, "wd": 1e-4,
                                                                            "momentum": 0.9})
    ex = mod.executor
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    out = {"prob": [], "grads": []}
    for _ in range(steps):
        mod.forward(batch, is_train=True)
        out["prob"].append(mod.get_outputs()[0].asnumpy().copy())
        mod.backward()
        out["grads"].append({n: ex.get_param(n, grad=True) for n in ex.plan.param_names})
        mod.update()
    arg, aux_o = mod.get_params()
    out["args"] = {k: v.asnumpy() for k, v in arg.items()}
    out["aux"] = {k: v.asnumpy() for k, v in aux_o.items()}
    out["mod"] = mod
    return out


def _check_grads(res, ref, ref32, step=0):
    bad = []
    for n, g in ref["grads"][step].items():
        e = fro_rel(res["grads"][step][n], g)
        tol = max(1e-4, 4 * fro_rel(ref32["grads"][step][n], g))
        if e > tol:
            bad.append((n, e, tol))
    assert not bad, bad[:5]


def test_c1_resnet20_cifar_two_steps():
    """C1: ResNet-20 (symbol/resnet.py:123-148), CIFAR 32x32, batch 16, two SGD steps on mx.cpu()."""
    g = onet.resnet20_cifar()
    args, aux = onet.init_params(g)
    data, label = onet.synthetic_batch(16, (3, 32, 32), 10)
    res = _module_step(graphs.resnet20_cifar(), args, aux, data, label, steps=2)
    assert type(res["mod"].executor).__name__ == "CPUExecutor"
    ref = oracle_step(g, args, aux, data, label, steps=2)
    ref32 = oracle_step(g, args, aux, data, label, steps=2, dtype=np.float32)
    # step 1 on every gradient; step 2 (whose inputs carry step 1's fp32 rounding through ReLU
    # decisions, test_step_gpu.py) on the probabilities, as the GPU's ResNet-20 test does
    _check_grads(res, ref, ref32, 0)
    for s in (0, 1):
        assert max_rel(res["prob"][s], ref["prob"][s]) < 1e-4
    # parameters and moving statistics after the first update
    res1 = _module_step(graphs.resnet20_cifar(), args, aux, data, label, steps=1)
    ref1 = oracle_step(g, args, aux, data, label, steps=1)
    for k, v in ref1["args"].items():
        assert max_rel(res1["args"][k], v) < 1e-5, k
    for k, v in ref1["aux"].items():
        assert max_rel(res1["aux"][k], v) < 1e-4, k


def test_cpu_resnet_v2_and_resnext_one_step():
    """The ImageNet graphs on the host: ResNet-50-style v2 (bn_data stem, 7x7 conv0, max pool) and a
    grouped ResNeXt, one step each at small sizes."""
    cases = [(onet.resnet([1, 1, 1, 1], 4, [16, 32, 64, 64, 128], 8),
              graphs.resnet([1, 1, 1, 1], 4, [16, 32, 64, 64, 128], 8)),
             (onet.resnext([1, 1, 1, 1], 4, [64, 128, 128, 256, 256], 8, num_group=32),
              graphs.resnext([1, 1, 1, 1], 4, [64, 128, 128, 256, 256], 8, "float32", 32))]
    for g, sym in cases:
        args, aux = onet.init_params(g)
        data, label = onet.synthetic_batch(4, (3, 48, 48), 8)
        res = _module_step(sym, args, aux, data, label)
        ref = oracle_step(g, args, aux, data, label)
        ref32 = oracle_step(g, args, aux, data, label, dtype=np.float32)
        assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
        _check_grads(res, ref, ref32)


def test_cpu_int8_graph_one_step():
    """resnet_int8 (C5's graph) on the host: the fake-quant ops with EMA thresholds and clipped STE."""
    g = onet.resnet_int8([1, 1, 1, 1], 4, [16, 32, 64, 64, 128], 8)
    args, aux = onet.init_params(g)
    data, label = onet.synthetic_batch(4, (3, 48, 48), 8)
    res = _module_step(graphs.resnet_int8([1, 1, 1, 1], 4, [16, 32, 64, 64, 128], 8), args, aux, data, label)
    ref = oracle_step(g, args, aux, data, label)
    # rounding to the int8 grid is chaotic under fp32 vs fp64 (test_resnet_int8_fp32_small): the
    # loss and the probabilities to the quantization step, the thresholds exactly-ish
    assert max_rel(res["prob"][0], ref["prob"][0]) < 5e-2
    st = res["mod"].get_params()[1]
    for k, v in st.items():
        if k.endswith("_minmax") and k in ref["quant_state"]:
            assert abs(v.asnumpy().item() - ref["quant_state"][k]) <= 1e-5 * max(ref["quant_state"][k], 1e-6), k


def test_cpu_context_rules():
    sym = graphs.resnet20_cifar()
    with pytest.raises(mx.MXNetError):
        mx.mod.Module(sym, context=[mx.cpu(), mx.gpu(0)]).bind([("data", (2, 3, 32, 32))], [("softmax_label", (2,))])
    mod = mx.mod.Module(sym, context=[])  # MXNet's default context: the host
    mod.bind([("data", (2, 3, 32, 32))], [("softmax_label", (2,))])
    assert type(mod.executor).__name__ == "CPUExecutor"


def test_c1_solver_fit_on_cpu(tmp_path):
    """C1 end to end: the reference's Solver.fit sequence (restated in test_solver_loop_cpu.solver_fit,
    core/solver.py:65-212) over SyntheticDataIter batches on mx.cpu(), with the warm-up scheduler,
    Speedometer and do_checkpoint of train.py: the training loss falls on the fixed batch, and the
    checkpoint reloads into a fresh CPU Module that predicts the same probabilities."""
    import logging
    from test_solver_loop_cpu import SyntheticDataIter, WarmupMultiFactorScheduler, solver_fit
    batch, epoch_size, num_epoch = 32, 4, 3
    sched = WarmupMultiFactorScheduler(base_lr=0.1, step=[8], factor=0.1, warmup=True, warmup_type="gradual",
                                       warmup_lr=0.02, warmup_step=4)
    mod = mx.mod.Module(graphs.resnet20_cifar(), logger=logging, context=mx.cpu())
    train = SyntheticDataIter(10, (batch, 3, 32, 32), epoch_size, np.float32)
    prefix = str(tmp_path / "c1")
    losses = []

    def track(param):
        ex = mod.executor
        losses.append(float(ex.stats[0]) / batch)

    solver_fit(mod, [("data", (batch, 3, 32, 32))], [("softmax_label", (batch,))], train, ["acc"],
               mx.callback.do_checkpoint(prefix), [mx.callback.Speedometer(batch, 2), track],
               mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2), "sgd",
               {"learning_rate": 0.1, "wd": 1e-4, "lr_scheduler": sched, "momentum": 0.9}, 0, num_epoch,
               mx.kvstore.create("local"))
    assert len(losses) == num_epoch * epoch_size
    assert losses[-1] < 0.8 * losses[0], losses
    sym, arg, aux = mx.model.load_checkpoint(prefix, num_epoch)
    m2 = mx.mod.Module(sym, context=mx.cpu())
    it = mx.io.NDArrayIter(train.data.asnumpy(), train.label.asnumpy(), batch_size=batch,
                           label_name="softmax_label")
    m2.bind(it.provide_data, it.provide_label, for_training=False)
    m2.init_params(arg_params=arg, aux_params=aux)
    mod2_prob = m2.predict(it).asnumpy()
    mod.forward(mx.io.DataBatch(data=[train.data], label=[train.label]), is_train=False)
    np.testing.assert_allclose(mod2_prob, mod.get_outputs()[0].asnumpy(), rtol=1e-5, atol=1e-7)
