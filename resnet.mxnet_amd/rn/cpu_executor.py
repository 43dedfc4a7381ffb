"""The mx.cpu() context: the same lowered Plan executed on the host (BASELINE config C1).

The reference's first config trains ResNet-20 on CIFAR-10 with MXNet's CPU executor through
train.py (`devs = [mx.gpu(i) for i in config.gpu_list]`, train.py:34, with
gpu_list=[] meaning no GPU). A Module bound to mx.cpu() contexts runs here: every op of the Plan
(rn/executor.py) as a torch-CPU fp32 operator (oneDNN, the analogue of MXNet's MKL-DNN CPU path),
with MXNet's semantics -- BatchNorm batch statistics with biased variance and momentum moving stats,
fix_gamma / use_global_stats, SoftmaxOutput's p - onehot gradient, Quantization_int8 with EMA
thresholds and the clipped STE, MXNet momentum SGD with wd_mult 0 on biases / betas -- and the same
flat fp32 parameter / gradient / momentum / aux buffers the GPU executor has, so Module,
kvstore (gloo all-reduce over the flat gradient), checkpoints and metrics work unchanged.

This is a device of its own, chosen only by an mx.cpu() context: a Module bound to mx.gpu() never
reaches it (GPU ops have no fallback; rn.lib fails loudly without librn).
"""
import numpy as np
import torch
import torch.nn.functional as F


class _QuantState:
    __slots__ = ("first",)

    def __init__(self):
        self.first = True


def _mx_round(v):
    """mx.nd.round: half away from zero (torch.round is half-to-even)."""
    return torch.sign(v) * torch.floor(v.abs() + 0.5)


class CPUExecutor:
    """Host tensors + a forward over the Plan ops with autograd for the backward."""

    dry_run = False

    def __init__(self, plan, bucket_bytes=None):
        self.plan = plan
        self.device = torch.device("cpu")
        self.bucket_bytes = bucket_bytes or (25 << 20)
        self._build_params()
        self.stats = torch.zeros(4, dtype=torch.float32)
        self._data = torch.zeros(plan.data_tensor.shape, dtype=torch.float32)
        self._label = None
        self._q = _QuantState()
        self._out = {}
        self._head = None
        self.num_update = 0

    # ------------------------------------------------------------------ buffers (MXNet layouts)
    def _build_params(self):
        plan = self.plan
        order, seen = [], set()
        for op in plan.ops:
            names = [getattr(op, k, None) for k in ("weight", "bias", "gamma", "beta")]
            if op.kind == "stem" and op.bn:
                names += [op.bn["gamma"], op.bn["beta"]]
            for nm in names:
                if nm and nm not in seen:
                    order.append(nm)
                    seen.add(nm)
        order = list(reversed(order))  # the GPU executor's order: buckets complete front to back
        self.param_order = order
        self.param_shape = {n: tuple(plan.param_shape(n)) for n in order}
        self.param_off, off = {}, 0
        for n in order:
            self.param_off[n] = off
            off += int(np.prod(self.param_shape[n]))
        self.nparam = off
        self.master = torch.zeros(max(off, 1), dtype=torch.float32)
        self.grad = torch.zeros_like(self.master)
        self.mom = torch.zeros_like(self.master)
        self.aux_off, aoff = {}, 0
        for n in plan.aux_names:
            shp = tuple(plan.param_shape(n))
            self.aux_off[n] = (aoff, shp)
            aoff += int(np.prod(shp))
        self.aux = torch.zeros(max(aoff, 1), dtype=torch.float32)
        self.wd_mult = torch.zeros_like(self.master)
        for n in order:
            if n.endswith("_weight") or n.endswith("_gamma"):
                o = self.param_off[n]
                self.wd_mult[o:o + int(np.prod(self.param_shape[n]))] = 1.0

    def _param(self, master, name, shape=None):
        o = self.param_off[name]
        n = int(np.prod(self.param_shape[name]))
        return master[o:o + n].view(shape if shape is not None else self.param_shape[name])

    def _auxv(self, name):
        o, shp = self.aux_off[name]
        return self.aux[o:o + int(np.prod(shp))]

    # ------------------------------------------------------------------ Module interface
    def set_input(self, data_np, label_np=None):
        d = torch.as_tensor(np.asarray(data_np, dtype=np.float32)) if isinstance(data_np, np.ndarray) else data_np
        self._data = d.detach().to(torch.float32).reshape(self.plan.data_tensor.shape).clone()
        if label_np is not None:
            lab = torch.as_tensor(np.asarray(label_np, dtype=np.float32)) if isinstance(label_np, np.ndarray) \
                else label_np
            self._label = lab.detach().reshape(-1).to(torch.float32).clone()

    def forward(self, is_train=True):
        with torch.enable_grad() if is_train else torch.no_grad():
            self._master_leaf = self.master.detach().requires_grad_(is_train)
            self._run(self._master_leaf, is_train)
        if is_train:
            self._q.first = False

    def backward(self, hooks=None):
        """Autograd from SoftmaxOutput's gradient (p - onehot) * grad_scale into the flat gradient; the
        bucket hooks (kvstore all-reduce) run once it is complete."""
        self.grad.zero_()
        if self._head is not None:
            logits, g = self._head
            logits.backward(g)
            if self._master_leaf.grad is not None:
                self.grad.copy_(self._master_leaf.grad)
        for i in sorted((hooks or {}).keys()):
            hooks[i]()

    def repack_weights(self):
        pass

    def sgd_update(self, lr, wd, momentum, rescale_grad, clip=-1.0):
        """MXNet SGD (multi_precision fp32): mom = momentum*mom - lr*(clip(rescale*g) + wd*wd_mult*w);
        w += mom (oracle/ops.py sgd_mom_update, train.py:186-203)."""
        with torch.no_grad():
            g = self.grad * rescale_grad
            if clip is not None and clip > 0:
                g = g.clamp(-clip, clip)
            g = g + wd * self.wd_mult * self.master
            self.mom.mul_(momentum).sub_(lr * g)
            self.master.add_(self.mom)
        self.num_update += 1

    def set_param(self, name, value):
        v = np.asarray(value, dtype=np.float32)
        if tuple(v.shape) != self.param_shape[name]:
            raise ValueError("shape mismatch for %s: %s vs %s" % (name, v.shape, self.param_shape[name]))
        self._param(self.master, name).copy_(torch.from_numpy(np.ascontiguousarray(v)))

    def get_param(self, name, grad=False):
        return self._param(self.grad if grad else self.master, name).detach().numpy().copy()

    def set_aux(self, name, value):
        self._auxv(name).copy_(torch.from_numpy(np.asarray(value, dtype=np.float32).reshape(-1)))

    def get_aux(self, name):
        return self._auxv(name).numpy().reshape(self.aux_off[name][1]).copy()

    def output(self, i=0):
        t = self.plan.outputs[i]
        return self._out[id(t)].detach()

    def buckets(self):
        """~bucket_bytes slices of the flat gradient, all launched once the backward is complete."""
        out, s = [], 0
        step = max(1, self.bucket_bytes // 4)
        while s < self.nparam:
            out.append((s, min(self.nparam, s + step), 0))
            s += step
        return out

    # ------------------------------------------------------------------ the ops
    def _run(self, m, train):
        env = {}
        P = lambda name, shape=None: self._param(m, name, shape)  # noqa: E731
        self._head = None

        def get(t):
            return env[id(t)]

        for op in self.plan.ops:
            k = op.kind
            if k == "stem":
                x = self._data
                if op.bn:
                    b = op.bn
                    x = self._bn(x, None, P(b["beta"]), b["mean"], b["var"], b["eps"], b["momentum"], True,
                                 b["use_global_stats"], train)
                if op.quant:
                    x = self._quant_act(x, op.quant, train)
                w = self._weight(P(op.weight), op.qweight, train)
                env[id(op.y)] = F.conv2d(x, w, stride=op.stride, padding=op.pad)
            elif k == "conv":
                w = self._weight(P(op.weight), op.qweight, train)
                y = F.conv2d(get(op.x), w, stride=op.stride, padding=op.pad, groups=op.groups)
                env[id(op.y)] = y + get(op.res) if op.res is not None else y
            elif k == "bn":
                y = self._bn(get(op.x), None if op.fix_gamma else P(op.gamma), P(op.beta), op.mean, op.var, op.eps,
                             op.momentum, op.fix_gamma, op.use_global_stats, train)
                env[id(op.y)] = F.relu(y) if op.relu else y
            elif k == "affine":
                c = op.x.c
                y = get(op.x)
                if op.gamma:
                    y = y * P(op.gamma, (1, c, 1, 1))
                if op.beta:
                    y = y + P(op.beta, (1, c, 1, 1))
                env[id(op.y)] = F.relu(y) if op.relu else y
            elif k == "relu":
                env[id(op.y)] = F.relu(get(op.x))
            elif k == "quant":
                env[id(op.y)] = self._quant_act(get(op.x), op.q, train)
            elif k == "add":
                y = get(op.a) + get(op.b)
                env[id(op.y)] = F.relu(y) if op.relu else y
            elif k == "pool":
                x = get(op.x)
                if op.global_pool:
                    y = x.mean(dim=(2, 3), keepdim=True) if op.type == "avg" else x.amax(dim=(2, 3), keepdim=True)
                elif op.type == "max":  # 'valid' convention, padding never wins (-inf)
                    y = F.max_pool2d(x, op.kernel, op.stride, op.pad)
                else:  # MXNet avg pooling counts the padding (count_include_pad)
                    y = F.avg_pool2d(x, op.kernel, op.stride, op.pad, count_include_pad=True)
                env[id(op.y)] = y
            elif k == "fc":
                x = get(op.x).reshape(op.x.n, -1)
                w = self._weight(P(op.weight), op.qweight, train)
                env[id(op.y)] = F.linear(x, w, P(op.bias) if op.bias else None)
            elif k == "softmax":
                z = get(op.x)
                prob = torch.softmax(z.detach(), dim=1)
                env[id(op.y)] = prob
                lab = self._label.long() if self._label is not None else None
                if train and lab is not None:
                    onehot = F.one_hot(lab, prob.shape[1]).to(prob.dtype)
                    self._head = (z, (prob - onehot) * op.grad_scale)
                    with torch.no_grad():  # device-metric counters: CE sum, top-1 / top-5 hits
                        pl = prob.gather(1, lab[:, None]).clamp_min(1e-30)
                        top = prob.topk(min(5, prob.shape[1]), dim=1).indices
                        self.stats += torch.tensor([float(-pl.log().sum()), float((top[:, 0] == lab).sum()),
                                                    float((top == lab[:, None]).any(1).sum()), 0.0])
            else:
                raise RuntimeError("CPU executor: op kind %s" % k)
        self._out = {id(t): env[id(t)] for t in self.plan.outputs}

    def _bn(self, x, gamma, beta, mean_name, var_name, eps, momentum, fix_gamma, use_global, train):
        """mx.sym.BatchNorm over axis 1 (fix_gamma: gamma := 1, no gradient)."""
        c = x.shape[1]
        g = torch.ones(c, dtype=x.dtype) if (fix_gamma or gamma is None) else gamma
        mm, mv = self._auxv(mean_name), self._auxv(var_name)
        if train and not use_global:
            dims = (0, 2, 3) if x.dim() == 4 else (0,)
            with torch.no_grad():  # moving = moving*momentum + batch*(1 - momentum), biased batch variance
                bm = x.mean(dim=dims)
                bv = x.var(dim=dims, unbiased=False)
                mm.mul_(momentum).add_(bm * (1 - momentum))
                mv.mul_(momentum).add_(bv * (1 - momentum))
            return F.batch_norm(x, None, None, g, beta, training=True, eps=eps)
        return F.batch_norm(x, mm.clone(), mv.clone(), g, beta, training=False, eps=eps)

    def _qthreshold(self, x, q, train, is_weight):
        """quant_state_update: weights t = max|w|; activations t = EMA(max|x|) from the first batch."""
        mm = self._auxv(q["minmax"])
        with torch.no_grad():
            cur = x.detach().abs().max()
            if is_weight:
                if train:
                    mm.fill_(float(cur))
                return cur
            if train:
                mm.fill_(float(cur) if self._q.first else float(mm[0]) * q["ema"] + float(cur) * (1 - q["ema"]))
            return mm[0].clone()

    def _quant_act(self, x, q, train):
        """Quantization_int8 on data: clip to +-t, round to the t/qmax grid; STE masked by |x| < t
        (symbol/clip_grad_quantization_int8.py:37-67)."""
        t = self._qthreshold(x, q, train, False)
        qmax = float(2 ** (q["nbits"] - 1) - 1)
        unit = t / qmax
        with torch.no_grad():
            v = _mx_round(x.detach().clamp(-float(t), float(t)) / unit) * unit if unit > 0 else torch.zeros_like(x)
            mask = ((x.detach() > -t) & (x.detach() < t)).to(x.dtype)
        return x * mask + (v - x.detach() * mask)

    def _weight(self, w, qw, train):
        """Quantization_int8 on a weight (per tensor, no clip, plain STE: symbol/quant_ops.py:17-31)."""
        if qw is None:
            return w
        t = self._qthreshold(w, qw, train, True)
        unit = t / float(2 ** (qw["nbits"] - 1) - 1)
        with torch.no_grad():
            v = _mx_round(w.detach() / unit) * unit if unit > 0 else torch.zeros_like(w)
        return w + (v - w.detach())
