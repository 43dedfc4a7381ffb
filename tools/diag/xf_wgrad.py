"""Diagnostic: the BN+ReLU-on-load weight gradient (rn_conv_bwd_filter_x) vs references built from
(a) the torch transform relu(addcmul(sh, x, sc)) -> bf16 and (b) the device's own rn_bn_apply output."""
import sys, os, ctypes as C
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd"), os.path.join(REPO, "tests")]
import mxnet as mx
from rn import graphs, lib as L
from layerwise import Checker, ref_wgrad, _bf16
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
sym = graphs.resnet50()
rng = np.random.default_rng(0)
data = rng.uniform(-1, 1, (n, 3, 224, 224)).astype(np.float32)
label = np.random.default_rng(1).integers(0, 1000, n).astype(np.float32)
mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision="bfloat16")
mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", (n,))])
mx.random.seed(2)
mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
mod.init_optimizer(kvstore="device", optimizer="sgd", optimizer_params={"learning_rate": 0.1})
ex = mod.executor
ex.side_enabled = False
batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
mod.forward(batch, is_train=True)
ck = Checker(ex)
lib = L.load()
res = {}
targets = {"stage4_unit2_conv1", "stage4_unit3_conv3", "stage1_unit1_conv1", "stage3_unit3_conv3", "stage4_unit1_sc"}
xf_ops = {op.name: op for op in ex.plan.ops if op.kind == "conv" and op.xf is not None and op.name in targets}
hooks = {}
for i, (name, fn, args) in enumerate(ex._bwd):
    if name != "rn_conv_bwd_filter_x":
        continue
    d = args[0]._obj
    wname = ck.grad_name(args[3])
    opn = wname[:-len("_weight")]
    if opn not in xf_ops:
        continue
    op = xf_ops[opn]
    def post(op=op, d=d, args=args, wname=wname):
        bn = op.xf
        dy = ck.nchw(ck.t(args[2]), d.n, d.p, d.q, d.k_pad, d.k)
        xa = ck.bn_relu_input(bn)
        # device's own materialised transform
        tmp = torch.empty_like(ex.act(bn.x))
        L.check(lib.rn_bn_apply(C.byref(bn.desc), L.ptr(ex.act(bn.x)), L.ptr(tmp), bn.sc, bn.sh,
                                C.c_void_p(torch.cuda.current_stream().cuda_stream)), "apply")
        xb = ck.nchw(tmp, bn.x.n, bn.x.h, bn.x.w, bn.x.cp, bn.x.c)
        mism = int((xa != xb).sum())
        dev = ex.gview(wname).view(d.k, d.r, d.s, d.c_real).permute(0, 3, 1, 2).double()
        out = {"transform mismatches": mism, "of": xa.numel()}
        for tag, x in (("torch transform", xa), ("device bn_apply", xb)):
            ref, rab = ref_wgrad(x, dy, (1, 1), (d.stride_h, d.stride_w), (0, 0), with_abs=True)
            out[tag] = (float(((dev - ref).abs() / (rab.double() + 1e-30)).max()),
                        float((dev - ref).norm() / ref.norm()))
        # the same conv weight gradient through the plain (non-XF) kernel on the materialised input
        dw2 = torch.zeros(d.k * d.c_real, device=dy.device, dtype=torch.float32)
        ws = ex.wgrad_ws
        L.check(lib.rn_conv_bwd_filter_ws(C.byref(d), L.ptr(tmp), args[2], L.ptr(dw2), L.ptr(ws), ex.wgrad_ws_bytes,
                                          C.c_void_p(torch.cuda.current_stream().cuda_stream)), "wg")
        ref, rab = ref_wgrad(xb, dy, (1, 1), (d.stride_h, d.stride_w), (0, 0), with_abs=True)
        dw2 = dw2.view(d.k, 1, 1, d.c_real).permute(0, 3, 1, 2).double()
        out["plain kernel on device bn_apply"] = (float(((dw2 - ref).abs() / (rab.double() + 1e-30)).max()),
                                                  float((dw2 - ref).norm() / ref.norm()))
        out["xf vs plain kernel"] = float((dev - dw2).norm() / dw2.norm())
        res[wname] = out
    hooks[i + 1] = post
with torch.no_grad():
    ex.backward(hooks=hooks)
torch.cuda.synchronize()
for k, v in res.items():
    print(k, v)
