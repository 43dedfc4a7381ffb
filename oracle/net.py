"""Numpy restatement of the reference graphs and of one Solver training step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py); parity against MXNet is unpinned.

Graphs (restated, not imported -- the reference cannot travel to the GPU box):
  resnet          symbol/resnet.py:77-121   (pre-activation ResNet-v2, bn_data + 7x7 stem)
  resnet_cifar10  symbol/resnet.py:123-148  (post-activation basic blocks, 3x3 stem)
  resnext         symbol/resnext.py:72-103  (post-activation, grouped 3x3, BN on shortcut)
  resnet_int8     symbol/resnet_int8.py:83-131 + symbol/int8_api.py:120-171 (fake-quant on
                  every conv / fc data and weight input)
Step order follows core/solver.py:115-121 (forward(is_train) -> backward -> update) with the
optimizer of train.py:186-194. Data-parallel semantics: the batch is
split evenly over devices, BN statistics per slice, gradients summed, one update.
"""
import numpy as np

from . import ops

EPS = 1e-5


class Graph:
    """A flat op list over named tensors; params / aux registered with MXNet names and shapes."""

    def __init__(self):
        self.ops = []
        self.params = {}  # name -> shape (in MXNet arg order)
        self.aux = {}
        self.chan = {}
        self.quant_state = {}  # activation-quant node name -> minmax (aux 'minmax')

    def add_param(self, name, shape):
        self.params[name] = tuple(shape)

    # --- op constructors (return output tensor name)
    def conv(self, name, x, k, kernel, stride=(1, 1), pad=(0, 0), groups=1, quant=False):
        c = self.chan[x]
        self.add_param(name + "_weight", (k, c // groups) + tuple(kernel))
        self.ops.append(dict(op="conv", name=name, x=x, y=name, k=k, kernel=kernel, stride=stride, pad=pad,
                             groups=groups, quant=quant, qname=None, wbits=8, abits=8))
        self.chan[name] = k
        return name

    def bn(self, name, x, eps=EPS, fix_gamma=False, momentum=0.9):
        c = self.chan[x]
        self.add_param(name + "_gamma", (c,))
        self.add_param(name + "_beta", (c,))
        self.aux[name + "_moving_mean"] = (c,)
        self.aux[name + "_moving_var"] = (c,)
        self.ops.append(dict(op="bn", name=name, x=x, y=name, eps=eps, fix_gamma=fix_gamma, momentum=momentum))
        self.chan[name] = c
        return name

    def relu(self, name, x):
        self.ops.append(dict(op="relu", name=name, x=x, y=name))
        self.chan[name] = self.chan[x]
        return name

    def maxpool(self, name, x, kernel, stride, pad):
        self.ops.append(dict(op="maxpool", name=name, x=x, y=name, kernel=kernel, stride=stride, pad=pad))
        self.chan[name] = self.chan[x]
        return name

    def gap(self, name, x):
        self.ops.append(dict(op="gap", name=name, x=x, y=name))
        self.chan[name] = self.chan[x]
        return name

    def fc(self, name, x, nh, quant=False):
        c = self.chan[x]
        self.add_param(name + "_weight", (nh, c))
        self.add_param(name + "_bias", (nh,))
        self.ops.append(dict(op="fc", name=name, x=x, y=name, nh=nh, quant=quant, qname=None, wbits=8, abits=8))
        self.chan[name] = nh
        return name

    def add(self, name, a, b):
        self.ops.append(dict(op="add", name=name, a=a, b=b, y=name))
        self.chan[name] = self.chan[a]
        return name

    def softmax(self, name, x):
        self.ops.append(dict(op="softmax", name=name, x=x, y=name))
        return name


# ----------------------------------------------------------------------------- graph builders
def resnet(units, num_stage, filter_list, num_classes, bottle_neck=True, dataset="imagenet", in_ch=3):
    """symbol/resnet.py:77-121 (+ residual_unit :9-53)."""
    g = Graph()
    g.chan["data"] = in_ch
    x = g.bn("bn_data", "data", eps=2e-5, fix_gamma=True)
    if dataset == "imagenet":
        x = g.conv("conv0", x, filter_list[0], (7, 7), (2, 2), (3, 3))
        x = g.bn("bn0", x)
        x = g.relu("relu0", x)
        x = g.maxpool("pooling0", x, (3, 3), (2, 2), (1, 1))
    else:
        x = g.conv("conv0", x, filter_list[0], (3, 3), (1, 1), (1, 1))
    for i in range(num_stage):
        for j in range(units[i]):
            st = (1, 1) if (i == 0 or j > 0) else (2, 2)
            x = _preact_unit(g, x, filter_list[i + 1], st, j > 0, "stage%d_unit%d" % (i + 1, j + 1), bottle_neck)
    x = g.bn("bn1", x)
    x = g.relu("relu1", x)
    x = g.gap("pool1", x)
    x = g.fc("fc1", x, num_classes)
    g.softmax("softmax", x)
    return g


def _preact_unit(g, data, nf, stride, dim_match, name, bottle_neck, quant=False):
    if bottle_neck:
        a1 = g.relu(name + "_relu1", g.bn(name + "_bn1", data))
        c1 = g.conv(name + "_conv1", a1, nf // 4, (1, 1), quant=quant)
        a2 = g.relu(name + "_relu2", g.bn(name + "_bn2", c1))
        c2 = g.conv(name + "_conv2", a2, nf // 4, (3, 3), stride, (1, 1), quant=quant)
        a3 = g.relu(name + "_relu3", g.bn(name + "_bn3", c2))
        c3 = g.conv(name + "_conv3", a3, nf, (1, 1), quant=quant)
        last = c3
    else:
        a1 = g.relu(name + "_relu1", g.bn(name + "_bn1", data))
        c1 = g.conv(name + "_conv1", a1, nf, (3, 3), stride, (1, 1), quant=quant)
        a2 = g.relu(name + "_relu2", g.bn(name + "_bn2", c1))
        last = g.conv(name + "_conv2", a2, nf, (3, 3), (1, 1), (1, 1), quant=quant)
    sc = data if dim_match else g.conv(name + "_sc", a1, nf, (1, 1), stride, quant=quant)
    return g.add(name + "_plus", last, sc)


def resnet_cifar10(units, num_stage, filter_list, num_classes, in_ch=3):
    """symbol/resnet.py:123-148 (+ residual_unit_cifar10 :55-74)."""
    g = Graph()
    g.chan["data"] = in_ch
    x = g.conv("conv0", "data", filter_list[0], (3, 3), (1, 1), (1, 1))
    x = g.relu("relu0", g.bn("bn0", x))
    for i in range(num_stage):
        for j in range(units[i]):
            st = (1, 1) if (i == 0 or j > 0) else (2, 2)
            dm = (filter_list[i] == filter_list[i + 1]) if j == 0 else True
            name = "stage%d_unit%d" % (i + 1, j + 1)
            c1 = g.conv(name + "_conv1", x, filter_list[i + 1], (3, 3), st, (1, 1))
            a1 = g.relu(name + "_relu1", g.bn(name + "_bn1", c1))
            c2 = g.conv(name + "_conv2", a1, filter_list[i + 1], (3, 3), (1, 1), (1, 1))
            b2 = g.bn(name + "_bn2", c2)
            if dm:
                sc = x
            else:
                sc = g.bn(name + "_sc_bn", g.conv(name + "_sc", x, filter_list[i + 1], (1, 1), st))
            x = g.relu(name + "_relu2", g.add(name + "_plus", b2, sc))
    x = g.gap("pool1", x)
    x = g.fc("fc1", x, num_classes)
    g.softmax("softmax", x)
    return g


def resnext(units, num_stage, filter_list, num_classes, num_group=32, bottle_neck=True, in_ch=3):
    """symbol/resnext.py:72-103 (+ xresidual_unit :10-69)."""
    mf = {32: 0.5, 64: 1.0}[num_group]
    g = Graph()
    g.chan["data"] = in_ch
    x = g.conv("conv0", "data", filter_list[0], (7, 7), (2, 2), (3, 3))
    x = g.relu("relu0", g.bn("bn0", x))
    x = g.maxpool("pooling0", x, (3, 3), (2, 2), (1, 1))
    for i in range(num_stage):
        for j in range(units[i]):
            st = (1, 1) if (i == 0 or j > 0) else (2, 2)
            name = "stage%d_unit%d" % (i + 1, j + 1)
            nf = filter_list[i + 1]
            if bottle_neck:
                c1 = g.conv(name + "_conv1", x, int(nf * mf), (1, 1))
                a1 = g.relu(name + "_relu1", g.bn(name + "_bn1", c1))
                c2 = g.conv(name + "_conv2", a1, int(nf * mf), (3, 3), st, (1, 1), groups=num_group)
                a2 = g.relu(name + "_relu2", g.bn(name + "_bn2", c2))
                c3 = g.conv(name + "_conv3", a2, nf, (1, 1))
                last = g.bn(name + "_bn3", c3)
            else:
                c1 = g.conv(name + "_conv1", x, nf, (3, 3), st, (1, 1))
                a1 = g.relu(name + "_relu1", g.bn(name + "_bn1", c1))
                c2 = g.conv(name + "_conv2", a1, nf, (3, 3), (1, 1), (1, 1))
                last = g.bn(name + "_bn2", c2)
            if j > 0:
                sc = x
            else:
                sc = g.bn(name + "_sc_bn", g.conv(name + "_sc", x, nf, (1, 1), st))
            x = g.relu(name + "_relu", g.add(name + "_plus", last, sc))
    x = g.gap("pool1", x)
    x = g.fc("fc1", x, num_classes)
    g.softmax("softmax", x)
    return g


def resnet_int8(units, num_stage, filter_list, num_classes, bottle_neck=True, dataset="imagenet", in_ch=3):
    """symbol/resnet_int8.py:83-131: the resnet graph with every conv (incl. conv0) and fc1
    fed by fake-quantized data and weights (int8_api.py:120-171)."""
    g = Graph()
    g.chan["data"] = in_ch
    x = g.bn("bn_data", "data", eps=2e-5, fix_gamma=True)
    if dataset == "imagenet":
        x = g.conv("conv0", x, filter_list[0], (7, 7), (2, 2), (3, 3), quant=True)
        x = g.relu("relu0", g.bn("bn0", x))
        x = g.maxpool("pooling0", x, (3, 3), (2, 2), (1, 1))
    else:
        x = g.conv("conv0", x, filter_list[0], (3, 3), (1, 1), (1, 1), quant=True)
    for i in range(num_stage):
        for j in range(units[i]):
            st = (1, 1) if (i == 0 or j > 0) else (2, 2)
            x = _preact_unit(g, x, filter_list[i + 1], st, j > 0, "stage%d_unit%d" % (i + 1, j + 1), bottle_neck,
                             quant=True)
    x = g.relu("relu1", g.bn("bn1", x))
    x = g.gap("pool1", x)
    x = g.fc("fc1", x, num_classes, quant=True)
    g.softmax("softmax", x)
    return g


def resnet50_imagenet(num_classes=1000):
    return resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], num_classes, True, "imagenet")


def resnet20_cifar():
    return resnet_cifar10([3, 3, 3], 3, [16, 16, 32, 64], 10)


def resnext50_32x4d(num_classes=1000):
    return resnext([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], num_classes, 32)


# ----------------------------------------------------------------------------- execution
def fix_bn(graph):
    """core/graph_optimize.py:114-157 (config.fix_bn, train.py:106-109, test.py:45-48): every
    BatchNorm switched to use_global_stats=True. Returns a new Graph (ops copied)."""
    g = Graph()
    g.params, g.aux, g.chan = dict(graph.params), dict(graph.aux), dict(graph.chan)
    g.ops = [dict(op, global_stats=True) if op["op"] == "bn" else dict(op) for op in graph.ops]
    return g


def attach_quant(graph, skip=None, wbits=8, abits=8):
    """core/graph_optimize.py:199-292 (config.quantize_flag, train.py:111-120) restricted to
    Quantization_int8 on Convolution / FullyConnected: every conv / fc input and weight gets a
    fake-quant node except the first skip[op] of each kind in graph order (skip_quantize_counts,
    edict_config.py default {'Convolution': 1, 'FullyConnected': 1}); one node per quantized tensor,
    named after it, shared by all its consumers. Returns a new Graph."""
    skip = dict(skip or {})
    seen = {"conv": 0, "fc": 0}
    g = Graph()
    g.params, g.aux, g.chan = dict(graph.params), dict(graph.aux), dict(graph.chan)
    for op in graph.ops:
        op = dict(op)
        if op["op"] in ("conv", "fc"):
            seen[op["op"]] += 1
            if seen[op["op"]] > skip.get(op["op"], 0):
                op.update(quant=True, qname=op["x"], wbits=wbits, abits=abits)
        g.ops.append(op)
    return g


def init_params(graph, seed=2, dtype=np.float64):
    """Xavier(gaussian, in, 2) in graph (MXNet arg) order from numpy.random.default_rng(seed)."""
    rng = np.random.default_rng(seed)
    args = {n: ops.init_param(n, s, rng).astype(dtype) for n, s in graph.params.items()}
    aux = {n: ops.init_param(n, s, rng).astype(dtype) for n, s in graph.aux.items()}
    return args, aux


def forward(graph, args, aux, data, label, is_train=True, quant_state=None, first_batch=True, storage=None,
            relu_masks=None, quant_values=None):
    """Returns (prob, tape). Updates aux (moving stats) in place when is_train.

    storage='bf16' emulates a bf16-storage runtime: conv/FC weights and every stored activation
    are rounded to bf16 (logits stay fp32), arithmetic stays in the array dtype.
    relu_masks {relu op name: bool array} replays given ReLU decisions (y = x * mask) instead of
    x > 0 -- parity diagnostics use it to remove rounding-induced decision flips.
    quant_values {'<conv>_data' / '<conv>_weight': array} likewise replays given int8 rounding
    decisions (the fake-quantized tensors) while the quantizer state still updates."""
    rnd = ops.bf16_round if storage == "bf16" else (lambda a: a)
    env = {"data": data}
    tape = []
    qs = quant_state if quant_state is not None else {}
    qdone = {}
    for op in graph.ops:
        t = op["op"]
        if t == "conv" or t == "fc":
            x = env[op["x"]]
            w = args[op["name"] + "_weight"]
            rec = dict(op=op)
            if op["quant"]:
                # the data quantizer node: '<conv>_data' (int8_api.py:133-136), or the quantized tensor's
                # own name when attach_quantize_node shares one node between its consumers
                # (core/graph_optimize.py:247-252): it runs (and updates its EMA) once per forward
                qn = op.get("qname") or op["name"] + "_data"
                key = qn + "_minmax"
                if qn in qdone:
                    xq, mm = qdone[qn]
                else:
                    xq, mm = ops.quant_int8_act(x, qs.get(key, 0.0), is_train, first_batch or key not in qs,
                                                nbits=op.get("abits", 8))
                    if quant_values is not None:
                        xq = quant_values.get(qn, xq).reshape(xq.shape).astype(xq.dtype)
                    qdone[qn] = (xq, mm)
                qs[key] = mm
                wq, _ = ops.quant_int8_weight(w, nbits=op.get("wbits", 8))
                if quant_values is not None:
                    wq = quant_values.get(op["name"] + "_weight", wq).reshape(wq.shape).astype(wq.dtype)
                rec.update(xraw=x, t=mm)
                x, w = xq, wq
            w = rnd(w)
            rec.update(x=x, w=w)
            if t == "conv":
                y = rnd(ops.conv2d_fwd(x, w, op["stride"], op["pad"], op["groups"]))
            else:
                xf = x.reshape(x.shape[0], -1)
                rec["x"] = xf
                y = ops.fc_fwd(xf, w, args[op["name"] + "_bias"])
            env[op["y"]] = y
            tape.append(rec)
        elif t == "bn":
            x = env[op["x"]]
            nm = op["name"]
            if is_train and op.get("global_stats"):
                y, cache = ops.bn_global_fwd(x, args[nm + "_gamma"], args[nm + "_beta"], aux[nm + "_moving_mean"],
                                             aux[nm + "_moving_var"], op["eps"], op["fix_gamma"])
                tape.append(dict(op=op, gcache=cache))
            elif is_train:
                y, cache = ops.bn_train_fwd(x, args[nm + "_gamma"], args[nm + "_beta"], op["eps"], op["fix_gamma"])
                aux[nm + "_moving_mean"], aux[nm + "_moving_var"] = ops.bn_moving_update(
                    aux[nm + "_moving_mean"], aux[nm + "_moving_var"], cache[3], cache[4], op["momentum"])
                tape.append(dict(op=op, cache=cache))
            else:
                y = ops.bn_infer_fwd(x, args[nm + "_gamma"], args[nm + "_beta"], aux[nm + "_moving_mean"],
                                     aux[nm + "_moving_var"], op["eps"], op["fix_gamma"])
                tape.append(dict(op=op))
            env[op["y"]] = rnd(y)
        elif t == "relu":
            x = env[op["x"]]
            mask = relu_masks[op["name"]] if (relu_masks is not None and op["name"] in relu_masks) else (x > 0)
            y = x * mask
            env[op["y"]] = y
            tape.append(dict(op=op, y=y, mask=mask))
        elif t == "maxpool":
            x = env[op["x"]]
            y, arg = ops.maxpool_fwd(x, op["kernel"], op["stride"], op["pad"])
            env[op["y"]] = y
            tape.append(dict(op=op, arg=arg, shape=x.shape))
        elif t == "gap":
            x = env[op["x"]]
            env[op["y"]] = rnd(ops.avgpool_global_fwd(x))
            tape.append(dict(op=op, shape=x.shape))
        elif t == "add":
            env[op["y"]] = rnd(env[op["a"]] + env[op["b"]])
            tape.append(dict(op=op))
        elif t == "softmax":
            prob = ops.softmax_output_fwd(env[op["x"]])
            env[op["y"]] = prob
            tape.append(dict(op=op, prob=prob))
    return env["softmax"], dict(tape=tape, env=env, label=label, rnd=rnd)


def backward(graph, args, fwd_state, grad_scale=1.0, keep=None):
    """Returns grads {param name: array} for one forward tape. If `keep` is a dict, the full
    gradient of every activation tensor is recorded into it (diagnostics)."""
    tape = fwd_state["tape"]
    label = fwd_state["label"]
    rnd = fwd_state.get("rnd", lambda a: a)
    grads = {}
    g = {}

    def acc(name, v):
        v = rnd(v)
        if name in g:
            g[name] = rnd(g[name] + v)
        else:
            g[name] = v

    for rec in reversed(tape):
        op = rec["op"]
        t = op["op"]
        if t == "softmax":
            acc(op["x"], ops.softmax_output_bwd(rec["prob"], label, grad_scale))
            continue
        dy = g.pop(op["y"], None)
        if dy is None:
            continue
        if keep is not None:
            keep[op["y"]] = dy
        if t == "conv":
            need_dx = op["x"] != "data"
            dx, dw = ops.conv2d_bwd(rec["x"], rec["w"], dy, op["stride"], op["pad"], op["groups"], need_dx=need_dx)
            if op["quant"] and need_dx:
                dx = ops.quant_int8_act_bwd(dx, rec["xraw"], rec["t"])
            grads[op["name"] + "_weight"] = dw
            if op["x"] != "data":
                acc(op["x"], dx)
        elif t == "fc":
            dxf, dw, db = ops.fc_bwd(rec["x"], rec["w"], dy)
            if op["quant"]:
                dxf = ops.quant_int8_act_bwd(dxf, rec["xraw"].reshape(dxf.shape), rec["t"])
            grads[op["name"] + "_weight"] = dw
            grads[op["name"] + "_bias"] = db
            acc(op["x"], dxf.reshape(dxf.shape[0], -1, 1, 1))
        elif t == "bn":
            if "gcache" in rec:
                dx, dgamma, dbeta = ops.bn_global_bwd(dy, rec["gcache"], op["fix_gamma"])
            else:
                dx, dgamma, dbeta = ops.bn_train_bwd(dy, rec["cache"], op["fix_gamma"])
            grads[op["name"] + "_gamma"] = dgamma
            grads[op["name"] + "_beta"] = dbeta
            if op["x"] != "data":
                acc(op["x"], dx)
        elif t == "relu":
            acc(op["x"], dy * rec["mask"])
        elif t == "maxpool":
            acc(op["x"], ops.maxpool_bwd(dy, rec["arg"], rec["shape"], op["kernel"], op["stride"], op["pad"]))
        elif t == "gap":
            acc(op["x"], ops.avgpool_global_bwd(dy.reshape(dy.shape[0], -1, 1, 1), rec["shape"]))
        elif t == "add":
            acc(op["a"], dy)
            acc(op["b"], dy)
    return grads


def train_step(graph, args, aux, moms, data, label, lr, momentum=0.9, wd=1e-4, rescale_grad=None,
               num_devices=1, quant_state=None, first_batch=True, storage=None, relu_masks=None, quant_values=None):
    """One Solver iteration (core/solver.py:115-121): forward(is_train) + backward + SGD update.

    num_devices > 1 restates Module's even batch split: per-slice BN statistics, per-slice
    moving-stat updates (returned per slice), gradients summed before the single update.
    Returns (probs, grads, per-device aux list). args/moms are updated in place.
    """
    b = data.shape[0]
    if rescale_grad is None:
        rescale_grad = 1.0 / b
    sl = b // num_devices
    probs, gsum, auxes = [], {}, []
    for d in range(num_devices):
        aux_d = {k: v.copy() for k, v in aux.items()}
        prob, st = forward(graph, args, aux_d, data[d * sl:(d + 1) * sl], label[d * sl:(d + 1) * sl], True,
                           quant_state, first_batch, storage, relu_masks, quant_values)
        grads = backward(graph, args, st)
        for k, v in grads.items():
            gsum[k] = gsum[k] + v if k in gsum else v
        probs.append(prob)
        auxes.append(aux_d)
    for name in graph.params:
        wd_n = wd * ops.wd_mult_for(name)
        ops.sgd_mom_update(args[name], gsum[name], moms[name], lr, wd_n, momentum, rescale_grad)
    return np.concatenate(probs, axis=0), gsum, auxes


def synthetic_batch(batch, shape, num_classes, dtype=np.float64):
    """data/imagenet.py:15-18, seeded: data U(-1,1) from default_rng(0), labels from default_rng(1)."""
    data = np.random.default_rng(0).uniform(-1, 1, (batch,) + tuple(shape)).astype(dtype)
    label = np.random.default_rng(1).integers(0, num_classes, (batch,)).astype(np.float32)
    return data, label
