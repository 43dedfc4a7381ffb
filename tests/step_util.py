"""Run one training step through the mxnet shim on the GPU and through the oracle on the CPU."""
import numpy as np

import mxnet as mx
from oracle import net as onet


def oracle_state(graph, seed=2):
    args, aux = onet.init_params(graph, seed=seed)
    return args, aux


def module_step(sym, args, aux, data, label, precision, lr=0.1, wd=1e-4, momentum=0.9, ctx=None, steps=1):
    """bind/init/forward/backward/update like core/solver.py:75-121; returns dict of results."""
    mod = mx.mod.Module(sym, context=ctx or [mx.gpu(0)], precision=precision)
    mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", label.shape)], for_training=True)
    mod.init_params(arg_params={k: v.astype(np.float32) for k, v in args.items()},
                    aux_params={k: v.astype(np.float32) for k, v in aux.items()})
    mod.init_optimizer(kvstore="device", optimizer="sgd",
                       optimizer_params={"learning_rate": lr, "wd": wd, "momentum": momentum})
    out = {"prob": [], "grads": []}
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    ex = mod.executor
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


def oracle_step(graph, args, aux, data, label, lr=0.1, wd=1e-4, momentum=0.9, steps=1, dtype=np.float64,
                storage=None):
    args = {k: v.astype(dtype) for k, v in args.items()}
    aux = {k: v.astype(dtype) for k, v in aux.items()}
    data = data.astype(dtype)
    moms = {k: np.zeros_like(v) for k, v in args.items()}
    probs, grads = [], []
    cur_aux = {k: v.copy() for k, v in aux.items()}
    for _ in range(steps):
        prob, g, auxes = onet.train_step(graph, args, cur_aux, moms, data, label, lr, momentum, wd, storage=storage)
        cur_aux = auxes[0]
        probs.append(prob)
        grads.append(g)
    return {"prob": probs, "grads": grads, "args": args, "aux": cur_aux}


def fro_rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-12))


def ce_loss(prob, label):
    return float(-np.log(np.maximum(prob[np.arange(prob.shape[0]), label.astype(np.int64)], 1e-30)).mean())


def max_rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))


def conditioned_errors(res, ref64, ref32, step=0):
    """Per-tensor (gpu_err, oracle_fp32_err) against the fp64 oracle.

    A deep randomly-initialised ResNet at small spatial size is ill-conditioned (train-mode BN
    backward over few elements is a projection with heavy cancellation; ReLU decisions flip
    under rounding), so an fp32 implementation is judged against the error the numpy oracle
    itself makes when run in fp32 on the same inputs."""
    out = {}
    for n in ref64["grads"][step]:
        out["grad:" + n] = (fro_rel(res["grads"][step][n], ref64["grads"][step][n]),
                            fro_rel(ref32["grads"][step][n], ref64["grads"][step][n]))
    for n in ref64["args"]:
        out["arg:" + n] = (max_rel(res["args"][n], ref64["args"][n]), max_rel(ref32["args"][n], ref64["args"][n]))
    for n in ref64["aux"]:
        out["aux:" + n] = (max_rel(res["aux"][n], ref64["aux"][n]), max_rel(ref32["aux"][n], ref64["aux"][n]))
    return out


def assert_conditioned(errs, factor=4.0, floor=2e-3):
    bad = [(k, e, r) for k, (e, r) in errs.items() if e > factor * r + floor]
    assert not bad, sorted(bad, key=lambda x: -x[1])[:5]
