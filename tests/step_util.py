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
                    aux_params={k: v.astype(np.float32) for k, v in aux.items()},
                    allow_missing=True)  # Quantization_int8 minmax states start at 0 (initializer)
    mod.init_optimizer(kvstore="device", optimizer="sgd",
                       optimizer_params={"learning_rate": lr, "wd": wd, "momentum": momentum})
    out = {"prob": [], "grads": [], "relu_masks": [], "quant_values": []}
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    ex = mod.executor
    for _ in range(steps):
        mod.forward(batch, is_train=True)
        out["prob"].append(mod.get_outputs()[0].asnumpy().copy())
        out["relu_masks"].append(gpu_relu_masks(ex))
        out["quant_values"].append(gpu_quant_values(ex))
        mod.backward()
        out["grads"].append({n: ex.get_param(n, grad=True) for n in ex.plan.param_names})
        mod.update()
    arg, aux_o = mod.get_params()
    out["args"] = {k: v.asnumpy() for k, v in arg.items()}
    out["aux"] = {k: v.asnumpy() for k, v in aux_o.items()}
    out["mod"] = mod
    return out


def gpu_relu_masks(ex):
    """ReLU decisions the device made: {Activation node name: bool NCHW mask} for every ReLU the
    executor ran (fused BatchNorm+ReLU, fused add+ReLU, or standalone). The oracle names its relu
    ops after the same Activation nodes, so the masks replay 1:1."""
    masks = {}
    for op in ex.plan.ops:
        name = getattr(op, "relu_name", None)
        if not name:
            continue
        t = op.y
        if op.kind == "bn" and (getattr(op, "apply_fused", False) or getattr(op, "apply_in_quant", False)):
            # BN+ReLU applied on load by its 1x1 consumers or its quantizer: the decision is fmaf(x, sc, sh) > 0 (exact
            # in fp64 for fp32 operands, same sign as the device's fused multiply-add)
            x = op.x
            xv = ex.act(x).float().cpu().numpy().reshape(x.n, x.h, x.w, x.cp).astype(np.float64)
            buf = op.buf.cpu().numpy().astype(np.float64)
            sc, sh = buf[2 * x.cp:3 * x.cp], buf[3 * x.cp:4 * x.cp]
            a = (xv * sc + sh)[..., :t.c].transpose(0, 3, 1, 2)
        else:
            a = ex.act(t).float().cpu().numpy().reshape(t.n, t.h, t.w, t.cp)[..., :t.c].transpose(0, 3, 1, 2)
        masks[name] = a > 0
    return masks


def gpu_quant_values(ex):
    """The fake-quantized tensors the device computed (Quantization_int8 outputs), keyed like
    oracle.net.forward's quant_values: '<conv>_data' (NCHW) and '<conv>_weight' (OIHW)."""
    vals = {}
    for op in ex.plan.ops:
        q = getattr(op, "qweight", None)
        if q is not None:
            k, c, r, s_ = ex.param_shape[op.weight] if len(ex.param_shape[op.weight]) == 4 else \
                ex.param_shape[op.weight] + (1, 1)
            vals[q["name"]] = op.qw.cpu().numpy().reshape(k, r, s_, c).transpose(0, 3, 1, 2)
        if op.kind == "quant":
            t = op.y
            src = ex.act(t)
            if getattr(op, "defer_values", False) or getattr(op, "codes_wgrad", False):
                # (after the forward only the codes exist: the values as rn_quant_int8_expand gives them)
                import ctypes as C
                import torch
                from rn import lib as L
                src = torch.empty_like(src)
                L.call("rn_quant_int8_expand", ex.dtype, src.numel(), C.c_void_p(op.codes.data_ptr()),
                       C.c_void_p(op.unit.data_ptr()), C.c_void_p(src.data_ptr()),
                       C.c_void_p(torch.cuda.current_stream().cuda_stream))
            a = src.float().cpu().numpy().reshape(t.n, t.h, t.w, t.cp)[..., :t.c].transpose(0, 3, 1, 2)
            vals[op.q["name"]] = a
        elif op.kind == "stem" and op.quant:
            # the quantized stem input is the NHWC-8 compute copy conv0 reads
            x = op.x
            xq = op.x8.float().cpu().numpy().reshape(x.n, x.h, x.w, 8)[..., :x.c].transpose(0, 3, 1, 2)
            vals[op.quant["name"]] = xq
    return vals


def replayed_parity(res, g, args, aux, data, label, steps=1, base_tol=1e-4, factor=4.0, quant_values=None):
    """Oracle fp64 and fp32 runs replaying the device's ReLU decisions; returns per-grad-tensor
    (gpu_err, numpy_fp32_err, tol) Frobenius-relative errors and the fp64 reference. Tensors whose
    reference cancels heavily (e.g. BN gamma grads: sum dz*xhat) get factor x the error numpy fp32
    itself makes on them."""
    masks = res["relu_masks"][0]
    ref = oracle_step(g, args, aux, data, label, relu_masks=masks, steps=steps, quant_values=quant_values)
    r32 = oracle_step(g, args, aux, data, label, relu_masks=masks, steps=steps, dtype=np.float32,
                      quant_values=quant_values)
    out = {}
    for n in ref["grads"][0]:
        e = fro_rel(res["grads"][0][n], ref["grads"][0][n])
        e32 = fro_rel(r32["grads"][0][n], ref["grads"][0][n])
        out[n] = (e, e32, max(base_tol, factor * e32))
    return out, ref


def oracle_step(graph, args, aux, data, label, lr=0.1, wd=1e-4, momentum=0.9, steps=1, dtype=np.float64,
                storage=None, relu_masks=None, quant_values=None):
    args = {k: v.astype(dtype) for k, v in args.items()}
    aux = {k: v.astype(dtype) for k, v in aux.items()}
    data = data.astype(dtype)
    moms = {k: np.zeros_like(v) for k, v in args.items()}
    probs, grads = [], []
    cur_aux = {k: v.copy() for k, v in aux.items()}
    qstate = {}
    for i in range(steps):
        prob, g, auxes = onet.train_step(graph, args, cur_aux, moms, data, label, lr, momentum, wd, storage=storage,
                                         relu_masks=relu_masks, quant_values=quant_values, quant_state=qstate,
                                         first_batch=i == 0)
        cur_aux = auxes[0]
        probs.append(prob)
        grads.append(g)
    return {"prob": probs, "grads": grads, "args": args, "aux": cur_aux, "quant_state": qstate}


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


def grad_summary(grads, ref):
    """Aggregate gradient agreement (fp64 arithmetic): global cosine, global Frobenius-relative
    error, and the median / 95th percentile of the per-tensor Frobenius-relative errors."""
    ks = sorted(ref)
    a = np.concatenate([np.asarray(grads[k], np.float64).ravel() for k in ks])
    b = np.concatenate([np.asarray(ref[k], np.float64).ravel() for k in ks])
    per = np.array([fro_rel(grads[k], ref[k]) for k in ks])
    return {"cos": float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b))),
            "fro": float(np.linalg.norm(a - b) / np.linalg.norm(b)),
            "median": float(np.median(per)), "p95": float(np.percentile(per, 95)), "max": float(per.max())}


# Whole-network R50 criteria; tests assert the oracle's own fp32 run meets them too.
R50_FP32 = {"cos": 0.9999, "fro": 1e-2, "median": 1e-2, "p95": 3e-2}


def assert_grad_summary(s, crit=R50_FP32):
    assert s["cos"] > crit["cos"] and s["fro"] < crit["fro"] and s["median"] < crit["median"] and \
        s["p95"] < crit["p95"], s
