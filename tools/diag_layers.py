"""GPU diagnostic: per-tensor forward activations and backward activation-gradients of the shim
executor (fp32 path) vs the fp64 oracle, in execution order; prints the first divergences."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch

import mxnet as mx
from oracle import net as onet
from rn import graphs


def nchw(buf, t):
    a = buf.float().cpu().numpy()
    if t.kind in ("logits",):
        return a.reshape(t.n, t.cp)[:, :t.c]
    return a.reshape(t.n, t.h, t.w, t.cp)[..., :t.c].transpose(0, 3, 1, 2)


def run(name, g, sym, n, hw, ncls, steps=2):
    from oracle import ops
    args, aux = onet.init_params(g)
    data, label = onet.synthetic_batch(n, (3, hw, hw), ncls)
    mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision="float32")
    mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", label.shape)])
    mod.init_params(arg_params={k: v.astype(np.float32) for k, v in args.items()},
                    aux_params={k: v.astype(np.float32) for k, v in aux.items()})
    mod.init_optimizer(optimizer_params={"learning_rate": 0.1, "momentum": 0.9, "wd": 1e-4})
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    ex = mod.executor
    moms = {k: np.zeros_like(v) for k, v in args.items()}
    for step in range(steps):
        aux64 = {k: v.copy() for k, v in aux.items()}
        prob, st = onet.forward(g, args, aux64, data, label)
        keep = {}
        grads = onet.backward(g, args, st, keep=keep)
        mod.forward(batch, is_train=True)
        mod.backward()
        torch.cuda.synchronize()
        print("== %s step %d" % (name, step), flush=True)
        worst = sorted(((float(np.linalg.norm(ex.get_param(k, grad=True) - v) / max(np.linalg.norm(v), 1e-30)), k)
                        for k, v in grads.items()), reverse=True)[:12]
        print("  worst param grads:", worst)
        _compare(ex, st, keep)
        mod.update()
        for k in g.params:
            ops.sgd_mom_update(args[k], grads[k], moms[k], 0.1, 1e-4 * ops.wd_mult_for(k), 0.9, 1.0 / n)
        torch.cuda.synchronize()
        worst = sorted(((float(np.abs(ex.get_param(k) - v).max() / max(np.abs(v).max(), 1e-30)), k)
                        for k, v in args.items()), reverse=True)[:3]
        print("  worst params after update:", worst, flush=True)


def _compare(ex, st, keep):
    for t in ex.plan.tensors.values():
        if t.kind not in ("act", "logits") or t.name not in st["env"] or "_bn" in t.name or t.name.startswith("bn"):
            continue
        ref = st["env"][t.name].reshape(nchw(ex.act(t), t).shape)
        got = nchw(ex.act(t), t)
        e = float(np.abs(got - ref).max() / max(np.abs(ref).max(), 1e-30))
        gerr = None
        gb = ex._grads.get(id(t))
        if gb is not None and t.name in keep:
            gref = keep[t.name].reshape(nchw(gb, t).shape)
            ggot = nchw(gb, t)
            gerr = float(np.linalg.norm(ggot - gref) / max(np.linalg.norm(gref), 1e-30))
        if e > 1e-4 or (gerr is not None and gerr > 1e-4) or "--all" in sys.argv:
            print("  %-32s fwd %.2e   grad(fro) %s" % (t.name, e, "-" if gerr is None else "%.2e" % gerr), flush=True)


if "--poison" in sys.argv:
    # fill the caching allocator's free pool with NaN: any read of memory no kernel wrote
    # (out-of-bounds or uninitialised) now shows up as NaN / garbage instead of zeros.
    blk = torch.empty(6 << 30, dtype=torch.uint8, device="cuda")
    blk.view(torch.float32).fill_(float("nan"))
    del blk
if "--r50" in sys.argv:
    run("r50", onet.resnet50_imagenet(16), graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16), 4, 64, 16,
        steps=1)
else:
    run("r20", onet.resnet20_cifar(), graphs.resnet20_cifar(), 8, 32, 10)
