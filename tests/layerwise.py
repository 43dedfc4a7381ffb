"""Layer-by-layer parity of one training step at any size (test infrastructure).

A randomly initialised ResNet-50 v2 is chaotic under rounding end to end (the
forward error of ANY bf16 storage grows ~1.17x per BatchNorm+ReLU layer, 0.2 % at the stem to 25 %
at stage 4, on the CPU emulation itself), so whole-step bf16 parity at the bench configuration can
only be relative. Per layer it is absolute: every kernel of the step is re-computed in fp32 on the
GPU with plain torch ops (unfold + GEMM, no MIOpen) from the SAME inputs the device kernel read (its
own stored bf16 activations, the bf16 compute copies of the weights, its saved BatchNorm statistics),
and its output must match within the rounding of its output type.

Forward: every conv (including BatchNorm+ReLU applied on load, the residual add, the BN statistics of
the epilogue via the BatchNorm coefficients), every BatchNorm's statistics / coefficients / stored
output, the stem (bn_data + conv0 over the zero-bordered NHWC4 image), pooling, FullyConnected,
SoftmaxOutput. Backward: every call of the backward plan, checked in a hook right after it runs
(the executor runs serialised on one stream while checking): data gradients (with the fused BN-backward
reductions they emit), weight gradients (split-M slabs, BN+ReLU on load), BatchNorm backward (dx,
dgamma, dbeta), gradient fan-in adds, pooling backward (through the device's own arg-max taps), the FC
bias gradient. References follow the ops' MXNet semantics (oracle/ops.py restated in torch).
"""
import types

import numpy as np

import torch
import torch.nn.functional as F

BF16_BAR = {"fro": 4e-3, "max": 8e-3}     # outputs stored in bf16 (one rounding of 2^-9)
F32_BAR = {"fro": 1e-4, "max": 2e-3}      # fp32 outputs of long fp32 reductions
# weight gradients: sums of up to N*P*Q = 802,816 products that cancel heavily, so the relative error of
# the result is not the measure; cond = error per element / the sum of its terms' magnitudes
WGRAD_BAR = {"fro": 1e-4, "max": 1e-3, "cond": 2e-6}


def _fro(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _maxr(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _bf16(t):
    return t.to(torch.bfloat16).to(torch.float32)


def _fma(x, a, b):
    """fp32 fmaf(x, a, b) as the kernels compute it (one rounding: the fp64 product of two fp32 values
    is exact). A mul-then-add reference differs in 1 of ~60,000 elements after the bf16 rounding, and
    in a weight gradient whose dy cancels those few flips are a 4e-5 error (tools/diag/xf_wgrad.py)."""
    return (x.double() * a.double() + b.double()).float()


def _chunks(n, per_image_bytes, budget=1 << 30):
    step = max(1, min(n, budget // max(per_image_bytes, 1)))
    return range(0, n, step), step


def ref_fwd(x, w, stride, pad):
    """fp32 conv forward: x (n,c,h,w), w (k,c,r,s)."""
    n, c, h, wd = x.shape
    k, _, r, s = w.shape
    p = (h + 2 * pad[0] - r) // stride[0] + 1
    q = (wd + 2 * pad[1] - s) // stride[1] + 1
    out = torch.empty(n, k, p, q, device=x.device, dtype=torch.float32)
    wm = w.reshape(k, -1)
    rng, step = _chunks(n, c * r * s * p * q * 4)
    for i in rng:
        cols = F.unfold(x[i:i + step], (r, s), padding=pad, stride=stride)
        out[i:i + step] = torch.matmul(wm, cols).view(-1, k, p, q)
    return out


def ref_dgrad(dy, w, hw, stride, pad):
    """fp32 data gradient: dy (n,k,p,q), w (k,c,r,s) -> (n,c,h,w)."""
    n, k, p, q = dy.shape
    _, c, r, s = w.shape
    out = torch.empty(n, c, hw[0], hw[1], device=dy.device, dtype=torch.float32)
    wt = w.reshape(k, -1).t()
    rng, step = _chunks(n, c * r * s * p * q * 4)
    for i in rng:
        cols = torch.matmul(wt, dy[i:i + step].reshape(-1, k, p * q))
        out[i:i + step] = F.fold(cols, hw, (r, s), padding=pad, stride=stride)
    return out


def ref_wgrad(x, dy, rs, stride, pad, with_abs=False):
    """Weight gradient (k,c,r,s) in fp64 (a sum over N*P*Q terms that cancels heavily: the BatchNorm
    backward makes dy zero-mean per channel). with_abs: also sum |dy| |x| (fp32), the scale that
    bounds any fp32 summation's error."""
    n, c = x.shape[:2]
    k, p, q = dy.shape[1:]
    acc = torch.zeros(k, c * rs[0] * rs[1], device=x.device, dtype=torch.float64)
    accb = torch.zeros(k, c * rs[0] * rs[1], device=x.device, dtype=torch.float32) if with_abs else None
    rng, step = _chunks(n, 4 * c * rs[0] * rs[1] * p * q * 4)
    for i in rng:
        cols = F.unfold(x[i:i + step], rs, padding=pad, stride=stride)  # (ch, crs, pq)
        ch = cols.shape[0]
        a = dy[i:i + step].reshape(ch, k, p * q).permute(1, 0, 2).reshape(k, ch * p * q)
        b = cols.permute(1, 0, 2).reshape(-1, ch * p * q)
        acc += torch.matmul(a.double(), b.double().t())
        if with_abs:
            accb += torch.matmul(a.abs(), b.abs().t())
    out = acc.view(k, c, rs[0], rs[1])
    return (out, accb.view(k, c, rs[0], rs[1])) if with_abs else out


class Checker:
    def __init__(self, ex):
        self.ex = ex
        self.rec = []  # (kind, layer, metrics dict, bar dict)
        self.byptr = {}
        for b in list(ex._acts.values()) + list(ex._grads.values()):
            self.byptr[b.data_ptr()] = b
        for op in ex.plan.ops:
            if op.kind == "stem":
                self.byptr[op.x8.data_ptr()] = op.x8
        self.wc_op = {}
        self.wk_op = {}
        for op in ex.plan.ops:
            if getattr(op, "wc", None) is not None:
                self.wc_op[op.wc.data_ptr()] = op
            if getattr(op, "wk", None) is not None:
                self.wk_op[op.wk.data_ptr()] = op
        self.bn_by_sm = {op.sm.value: op for op in ex.plan.ops if op.kind == "bn"}

    # ------------------------------------------------------------------ helpers
    def t(self, ptr):
        v = ptr.value if hasattr(ptr, "value") else ptr
        return None if v is None else self.byptr[v]

    def add(self, kind, layer, dev, ref, bar):
        m = {"fro": _fro(dev, ref), "max": _maxr(dev, ref)}
        self.rec.append((kind, layer, m, bar))

    def add_metric(self, kind, layer, m, bar):
        self.rec.append((kind, layer, m, bar))

    @staticmethod
    def nchw(buf, n, h, w, cs, c):
        return buf.view(n, h, w, cs)[..., :c].permute(0, 3, 1, 2).float()

    def act_nchw(self, t):
        return self.nchw(self.ex.act(t), t.n, t.h, t.w, t.cp, t.c)

    def param(self, name):
        return self.ex.pview(name)

    def grad_name(self, ptr):
        off = (ptr.value - self.ex.grad.data_ptr()) // 4
        for nm, o in self.ex.param_off.items():
            if o == off:
                return nm
        raise KeyError(ptr.value)

    @staticmethod
    def w_from_krsc(wk, d):
        return wk.view(d.k, d.r, d.s, d.c)[..., :d.c_real].permute(0, 3, 1, 2).float()

    @staticmethod
    def w_from_crsk(wc, d):
        return wc.view(d.c, d.r, d.s, d.k_pad)[:d.c_real, :, :, :d.k].permute(3, 0, 1, 2).float()

    def bn_coefs(self, op):
        cp = op.x.cp
        b = op.buf
        return b[0:cp], b[cp:2 * cp], b[2 * cp:3 * cp], b[3 * cp:4 * cp]

    def conv_input(self, op):
        """What the conv's kernel multiplies: its stored input, or relu(bn(x)) rounded to bf16 as the
        BN+ReLU-on-load transform produces it."""
        if op.xf is None:
            return self.act_nchw(op.x)
        return self.bn_relu_input(op.xf)

    def bn_relu_input(self, bn):
        _, _, sc, sh = self.bn_coefs(bn)
        x = self.act_nchw(bn.x)
        c = bn.x.c
        v = torch.relu(_fma(x, sc[:c].view(1, c, 1, 1), sh[:c].view(1, c, 1, 1)))
        return _bf16(v) if self.ex.dtype == 0 else v

    # ------------------------------------------------------------------ forward
    def check_forward(self):
        ex = self.ex
        bar = BF16_BAR if ex.dtype == 0 else F32_BAR
        for op in ex.plan.ops:
            if op.kind == "conv":
                if op.groups != 1 or getattr(op, "int8", False):
                    continue
                d = op.desc
                w = self.w_from_krsc(op.wk, d)
                y = ref_fwd(self.conv_input(op), w, op.stride, op.pad)
                if op.res is not None:
                    y = y + self.act_nchw(op.res)
                self.add("conv_fwd", op.name, self.act_nchw(op.y), y, bar)
            elif op.kind == "stem" and op.bn is not None and op.quant is None:
                x = op.x
                b = op.bnbuf
                sc, sh = b[16:16 + x.c], b[24:24 + x.c]
                data = ex._in_bufs[ex._in_idx].view(x.n, x.c, x.h, x.w).float()
                # bn_data (fix_gamma): batch statistics of the NCHW input, biased variance
                mean = data.double().mean(dim=(0, 2, 3))
                var = data.double().var(dim=(0, 2, 3), unbiased=False)
                inv = 1.0 / torch.sqrt(var + op.bn["eps"])
                self.add_metric("bn_fwd", "bn_data", {"mean": float(((b[0:x.c].double() - mean).abs() /
                                                                       torch.sqrt(var)).max()),
                                                      "invstd": _maxr(b[8:8 + x.c], inv)},
                                {"mean": 1e-5, "invstd": 1e-5})
                want = data * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
                k = op.y.c
                if op.p4 is not None:  # the zero-bordered NHWC4 image, 8 x 8 taps of 4 channels
                    hp, wp = op.p4
                    x4 = op.x8.view(x.n, hp, wp, 4).permute(0, 3, 1, 2).float()
                    ph, pw = op.pad
                    self.add("stem_prepare", "bn_data", x4[:, :x.c, ph:ph + x.h, pw:pw + x.w], _bf16(want), BF16_BAR)
                    w = op.wk.view(k, 8, 8, 4)[:, :op.kernel[0], :op.kernel[1], :].permute(0, 3, 1, 2).float()
                    y = ref_fwd(x4, w, op.stride, (0, 0))[:, :, :op.y.h, :op.y.w]
                else:  # NHWC with 8 channels (3 real)
                    x8 = self.nchw(op.x8, x.n, x.h, x.w, 8, x.c)
                    self.add("stem_prepare", "bn_data", x8, _bf16(want) if ex.dtype == 0 else want, bar)
                    y = ref_fwd(x8, self.w_from_krsc(op.wk, op.dfull), op.stride, op.pad)
                self.add("conv_fwd", op.name, self.act_nchw(op.y), y, bar)
            elif op.kind == "bn" and not op.use_global_stats:
                x = self.act_nchw(op.x).double()
                c = op.x.c
                mean = x.mean(dim=(0, 2, 3))
                var = x.var(dim=(0, 2, 3), unbiased=False)
                sm, si, sc, sh = self.bn_coefs(op)
                inv = 1.0 / torch.sqrt(var + op.eps)
                g = torch.ones_like(mean) if op.fix_gamma else self.param(op.gamma).double()
                beta = self.param(op.beta).double()
                m = {"mean": float(((sm[:c].double() - mean).abs() / torch.sqrt(var + op.eps)).max()),
                     "invstd": _maxr(si[:c], inv), "scale": _maxr(sc[:c], g * inv),
                     "shift": float((sh[:c].double() - (beta - mean * g * inv)).abs().max() /
                                    max(1.0, float((beta - mean * g * inv).abs().max())))}
                self.add_metric("bn_fwd", op.name, m, {"mean": 1e-5, "invstd": 1e-5, "scale": 1e-5,
                                                       "shift": 1e-5})
                if not (getattr(op, "apply_fused", False) or getattr(op, "apply_in_quant", False)):
                    v = _fma(x.float(), sc[:c].view(1, c, 1, 1), sh[:c].view(1, c, 1, 1))
                    if op.relu:
                        v = torch.relu(v)
                    self.add("bn_apply", op.name, self.act_nchw(op.y), v, bar)
            elif op.kind == "pool":
                x = self.act_nchw(op.x)
                if op.type == "max":
                    y = F.max_pool2d(x, op.kernel, op.stride, op.pad)
                else:
                    y = x.mean(dim=(2, 3), keepdim=True) if op.global_pool else F.avg_pool2d(x, op.kernel, op.stride,
                                                                                            op.pad)
                self.add("pool_fwd", op.name, self.act_nchw(op.y), y, bar if op.type != "max" else {"fro": 0.0,
                                                                                                   "max": 0.0})
            elif op.kind == "fc":
                d = op.desc
                x = self.act_nchw(op.x).reshape(op.x.n, -1)
                w = op.wk.view(d.k, d.c)[:, :d.c_real].float()
                y = x @ w.t() + self.param(op.bias).view(1, -1)
                dev = ex.act(op.y).view(op.y.n, op.y.cp)[:, :op.nh]
                self.add("fc_fwd", op.name, dev, y, F32_BAR)
            elif op.kind == "softmax":
                x = op.x
                logits = ex.act(x).view(x.n, x.cp)[:, :x.c].double()
                p = torch.softmax(logits, dim=1)
                self.add("softmax", op.name, ex.act(op.y).view(x.n, x.c), p, {"fro": 1e-5, "max": 1e-5})
                lab = ex.act(op.label).view(-1).long()
                g = p.clone()
                g[torch.arange(x.n, device=g.device), lab] -= 1.0
                dl = ex.grad_buf(x).view(x.n, x.cp)[:, :x.c]
                self.add("softmax_grad", op.name, dl.float(), g * op.grad_scale, bar)

    # ------------------------------------------------------------------ backward (hooks)
    def backward_hooks(self):
        ex = self.ex
        pre, post = {}, {}
        self.covered, self.skipped = {}, {}
        for i, (name, fn, args) in enumerate(ex._bwd):
            h = getattr(self, "_h_" + name, None)
            if h is None:
                self.skipped[name] = self.skipped.get(name, 0) + 1
                continue
            self.covered[name] = self.covered.get(name, 0) + 1
            state = {}
            pre_fn, post_fn = h(args, state)
            if pre_fn is not None:
                pre.setdefault(i, []).append(pre_fn)
            post.setdefault(i + 1, []).append(post_fn)
        hooks = {}
        for k in set(pre) | set(post):
            fns = post.get(k, []) + pre.get(k, [])
            hooks[k] = (lambda fs: lambda: [f() for f in fs])(fns)
        if 0 in pre:
            raise RuntimeError("a check needs a snapshot before the first backward call")
        return hooks

    def _snap(self, ptr, state, key):
        t = self.t(ptr) if ptr is not None else None

        def f():
            state[key] = None if t is None else t.clone()
        return f

    def _dgrad(self, args, state, bnred=False):
        d = args[0]._obj
        dyp, wcp, outp, addp = args[1], args[2], args[3], args[4]
        op = self.wc_op[wcp.value]

        def post():
            n, p, q = d.n, d.p, d.q
            dy = self.nchw(self.t(dyp), n, p, q, d.k_pad, d.k)
            w = self.w_from_crsk(op.wc, d)
            ref = ref_dgrad(dy, w, (d.h, d.w), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w))
            if state.get("add") is not None:
                ref = ref + self.nchw(state["add"], n, d.h, d.w, d.c, d.c_real)
            dev = self.nchw(self.t(outp), n, d.h, d.w, d.c, d.c_real)
            self.add("dgrad_bnred" if bnred else "dgrad", op.name, dev,
                     ref, BF16_BAR if self.ex.dtype == 0 else F32_BAR)
        return (self._snap(addp, state, "add") if addp is not None else None), post

    def _h_rn_conv_bwd_data(self, args, state):
        return self._dgrad(args, state)

    def _h_rn_conv_bwd_data_bnred(self, args, state):
        if args[3] is None:  # reduction only (the first pass of the recompute): nothing stored; its partials
            return None, (lambda: None)  # are checked through dgamma / dbeta / dx of the apply below
        return self._dgrad(args, state, bnred=True)

    def _h_rn_bn_bwd_finalize(self, args, state):
        return None, (lambda: None)  # (dgamma / dbeta: checked after rn_conv_bwd_data_bnapply)

    def _h_rn_conv_bwd_data_bnapply(self, args, state):
        """the dgrad recomputed with the BN backward applied: dx vs the fp32 dgrad of the device's dy,
        rounded to bf16 as rn_conv_bwd_data would store it, through the BN(+ReLU) backward (+ add)."""
        if not hasattr(self, "bn_by_sm_x"):
            self.bn_by_sm_x = {self.ex.act(op.x).data_ptr(): op for op in self.ex.plan.ops if op.kind == "bn"}
        d = args[0]._obj
        dyp, wcp, dxp, addp, xp = args[1], args[2], args[3], args[4], args[5]
        cop, op = self.wc_op[wcp.value], self.bn_by_sm_x[xp.value]

        def post():
            dy = self.nchw(self.t(dyp), d.n, d.p, d.q, d.k_pad, d.k)
            w = self.w_from_crsk(cop.wc, d)
            g = ref_dgrad(dy, w, (d.h, d.w), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w))
            self._bn_bwd_check(op, _bf16(g).double(), state.get("add"), dxp)
        return (self._snap(addp, state, "add") if addp is not None else None), post

    def _wgrad(self, args, state, xf=False, p4=False):
        d = args[0]._obj
        xp, dyp, dwp = args[1], args[2], args[3]
        name = self.grad_name(dwp)

        def post():
            n = d.n
            dy = self.nchw(self.t(dyp), n, d.p, d.q, d.k_pad, d.k)
            if p4:
                op = [o for o in self.ex.plan.ops if o.kind == "stem"][0]
                hp, wp = op.p4
                x = op.x8.view(n, hp, wp, 4).permute(0, 3, 1, 2).float()
                x = x[:, :, :(d.p - 1) * d.stride_h + d.r, :(d.q - 1) * d.stride_w + d.s]  # exactly p x q windows
                ref, rab = ref_wgrad(x, dy, (d.r, d.s), (d.stride_h, d.stride_w), (0, 0), with_abs=True)
                ref, rab = ref[:, :d.c_real], rab[:, :d.c_real]
            else:
                if xf:
                    x = self.bn_relu_input(self.bn_by_sm_x[xp.value])
                else:
                    x = self.nchw(self.t(xp), n, d.h, d.w, d.c, d.c_real)
                ref, rab = ref_wgrad(x, dy, (d.r, d.s), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w), with_abs=True)
            dev = self.ex.gview(name).view(d.k, d.r, d.s, d.c_real).permute(0, 3, 1, 2)
            if self.ex.param_layout[name] != "krsc":  # FC: (k, c)
                dev = self.ex.gview(name).view(d.k, d.c_real, 1, 1)
            # cond: |dev - ref| per element over sum |dy| |x| of its terms (an fp32 summation of n terms
            # errs by at most ~n * 2^-24 of that; blocked / split sums far less)
            m = {"fro": _fro(dev, ref), "max": _maxr(dev, ref),
                 "cond": float(((dev.double() - ref).abs() / (rab.double() + 1e-30)).max())}
            self.add_metric("wgrad", name, m, WGRAD_BAR)
        return None, post

    def _h_rn_conv_bwd_filter(self, args, state):
        return self._wgrad(args, state)

    def _h_rn_conv_bwd_filter_ws(self, args, state):
        return self._wgrad(args, state)

    def _h_rn_conv_bwd_filter_x(self, args, state):
        if not hasattr(self, "bn_by_sm_x"):
            self.bn_by_sm_x = {self.ex.act(op.x).data_ptr(): op for op in self.ex.plan.ops if op.kind == "bn"}
        return self._wgrad(args, state, xf=True)

    def _h_rn_stem_conv_wgrad_p4(self, args, state):
        d = args[0]._obj
        op = [o for o in self.ex.plan.ops if o.kind == "stem"][0]
        if d.n == op.dfull.n:
            return self._wgrad(args, state, p4=True)
        # an image chunk (executor._stem_chunks): dW is complete after the last one -> check it there
        # against the whole batch
        hp, wp = op.p4
        i = (args[1].value - op.x8.data_ptr()) // (d.n * hp * wp * 4 * 2)
        if (i + 1) * d.n < op.dfull.n:
            return None, (lambda: None)
        dy0 = args[2].value - i * d.n * d.p * d.q * d.k_pad * 2
        full = (types.SimpleNamespace(_obj=op.dfull), types.SimpleNamespace(value=op.x8.data_ptr()),
                types.SimpleNamespace(value=dy0), args[3])
        return self._wgrad(full, state, p4=True)

    def _h_rn_bn_bwd_apply_rows(self, args, state):
        """dx rows of a BN backward whose reductions rn_bn_bwd did (dx = NULL): the whole dx checked
        after the last row chunk."""
        d = args[0]._obj
        if args[8] + args[9] < d.m:
            return None, (lambda: None)
        if not hasattr(self, "bn_by_sm_x"):
            self.bn_by_sm_x = {self.ex.act(op.x).data_ptr(): op for op in self.ex.plan.ops if op.kind == "bn"}
        op = self.bn_by_sm_x[args[1].value]
        xp, dyp, dxp = args[1], args[2], args[3]
        assert args[4] is None

        def post():
            t = op.x
            self._bn_bwd_check(op, self.nchw(self.t(dyp), t.n, t.h, t.w, t.cp, t.c).double(), None, dxp)
        return None, post

    def _bn_bwd(self, args, state, part):
        if part:
            d, xp, dyp, dxp, addp, gp, smp = args[0]._obj, args[3], args[4], args[5], args[6], args[7], args[8]
            dgp, dbp = args[12], args[13]
        else:
            d, xp, dyp, dxp, addp, gp, smp = args[0]._obj, args[1], args[2], args[3], args[4], args[5], args[6]
            dgp, dbp = args[10], args[11]
        op = self.bn_by_sm[smp.value]

        def post():
            t = op.x
            self._bn_bwd_check(op, self.nchw(self.t(dyp), t.n, t.h, t.w, t.cp, t.c).double(), state.get("add"), dxp)
        return (self._snap(addp, state, "add") if addp is not None else None), post

    def _bn_bwd_check(self, op, dy, add, dxp):
        """BN(+ReLU) backward of `op` from its output gradient dy (fp64, NCHW): dx (+ add) vs the device's
        dxp, dgamma / dbeta vs the gradient buffers."""
        t = op.x
        c = t.c
        sm, si, sc, sh = self.bn_coefs(op)
        x = self.act_nchw(t).double()
        mu, inv = sm[:c].double().view(1, c, 1, 1), si[:c].double().view(1, c, 1, 1)
        dz = dy
        if op.relu:
            dz = dy * ((x * sc[:c].double().view(1, c, 1, 1) + sh[:c].double().view(1, c, 1, 1)) > 0)
        xc = x - mu
        m = t.n * t.h * t.w
        s = dz.sum(dim=(0, 2, 3))
        q = (dz * xc).sum(dim=(0, 2, 3))
        g = torch.ones(c, device=x.device, dtype=torch.float64) if op.fix_gamma else \
            self.param(op.gamma).double()
        gi = (g.view(1, c, 1, 1) * inv)
        # dx = g*invstd*(dz - mean(dz) - xhat*mean(dz*xhat)), xhat = (x - mean)*invstd
        dx = gi * (dz - (s / m).view(1, c, 1, 1)) - gi * inv * inv * (q / m).view(1, c, 1, 1) * xc
        if add is not None:
            dx = dx + self.nchw(add, t.n, t.h, t.w, t.cp, c).double()
        if dxp is not None:
            dev = self.nchw(self.t(dxp), t.n, t.h, t.w, t.cp, c)
            self.add("bn_bwd_dx", op.name, dev, dx, BF16_BAR if self.ex.dtype == 0 else F32_BAR)
        # fp32 sums: bounded by the sum of the magnitudes of their terms
        sa = dz.abs().sum(dim=(0, 2, 3))
        qa = (dz * xc).abs().sum(dim=(0, 2, 3)) * inv.view(-1)
        db = self.ex.gview(op.beta)[:c].double()
        mb = {"dbeta": float(((db - s).abs() / (sa + 1e-30)).max())}
        if not op.fix_gamma:
            dgv = self.ex.gview(op.gamma)[:c].double()
            mb["dgamma"] = float(((dgv - q * inv.view(-1)).abs() / (qa + 1e-30)).max())
        self.add_metric("bn_bwd_params", op.name, mb, {k: 1e-5 for k in mb})

    def _h_rn_bn_bwd_part(self, args, state):
        return self._bn_bwd(args, state, True)

    def _h_rn_bn_bwd(self, args, state):
        return self._bn_bwd(args, state, False)

    def _h_rn_eltwise_add(self, args, state):
        n, _, ap, bp, dp = args[0], args[1], args[2], args[3], args[4]
        sa, sb = self._snap(ap, state, "a"), self._snap(bp, state, "b")

        def pre():
            sa()
            sb()

        def post():
            ref = state["a"].float() + (state["b"].float() if state["b"] is not None else 0.0)
            if args[5]:
                ref = torch.relu(ref)
            self.add("grad_fanin_add", "add", self.t(dp)[:n].float(), ref, BF16_BAR)
        return pre, post

    def _h_rn_pool_bwd(self, args, state):
        d, dyp, amp, dxp, addp = args[0]._obj, args[1], args[2], args[3], args[4]
        op = [o for o in self.ex.plan.ops if o.kind == "pool" and o.argmax is not None and
              amp.value == o.argmax.data_ptr()] if amp is not None else []

        def post():
            n, c = d.n, d.c
            dy = self.t(dyp).view(n, d.p, d.q, c).float()
            ref = torch.zeros(n, d.h, d.w, c, device=dy.device, dtype=torch.float64)
            if op:
                am = op[0].argmax.view(n, d.p, d.q, c).long()
                tr, ts = am // d.s, am % d.s
                ii = torch.arange(d.p, device=dy.device).view(1, -1, 1, 1) * d.stride_h - d.pad_h + tr
                jj = torch.arange(d.q, device=dy.device).view(1, 1, -1, 1) * d.stride_w - d.pad_w + ts
                nn = torch.arange(n, device=dy.device).view(-1, 1, 1, 1).expand_as(ii)
                cc = torch.arange(c, device=dy.device).view(1, 1, 1, -1).expand_as(ii)
                ok = (ii >= 0) & (ii < d.h) & (jj >= 0) & (jj < d.w)
                ref.index_put_((nn[ok], ii[ok], jj[ok], cc[ok]), dy[ok].double(), accumulate=True)
            else:  # global average
                ref += (dy / (d.h * d.w)).double()
            if state.get("add") is not None:
                ref += state["add"].view(n, d.h, d.w, c).double()
            self.add("pool_bwd", "pool", self.t(dxp).view(n, d.h, d.w, c).float(), ref, BF16_BAR)
        return (self._snap(addp, state, "add") if addp is not None else None), post

    def _h_rn_col_sum(self, args, state):
        _, m, c, ld, xp, outp = args[:6]

        def post():
            x = self.t(xp).view(m, ld)[:, :c].double()
            off = (outp.value - self.ex.grad.data_ptr()) // 4
            dev = self.ex.grad[off:off + c]
            self.add("fc_bias_grad", "fc1_bias", dev, x.sum(0), F32_BAR)
        return None, post

    def _h_rn_stem_shift_grad(self, args, state):
        """bn_data's beta gradient without the stem's data gradient: dbeta[c] = sum over the image of
        conv0's data gradient (fix_gamma BatchNorm), from the fp32 master weights."""
        d, dyp, wmp, dbp = args[0]._obj, args[1], args[2], args[3]
        name = self.grad_name(dbp)

        def post():
            dy = self.nchw(self.t(dyp), d.n, d.p, d.q, d.k_pad, d.k)
            off = (wmp.value - self.ex.master.data_ptr()) // 4
            w = self.ex.master[off:off + d.k * d.r * d.s * d.c_real].view(d.k, d.r, d.s, d.c_real).permute(0, 3, 1, 2)
            args_ = ((d.h, d.w), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w))
            ref = ref_dgrad(dy, w.float(), *args_).double().sum(dim=(0, 2, 3))
            rab = ref_dgrad(dy.abs(), w.float().abs(), *args_).double().sum(dim=(0, 2, 3))
            dev = self.ex.gview(name)[:d.c_real].double()
            self.add_metric("stem_dbeta", name, {"cond": float(((dev - ref).abs() / rab).max()),
                                                 "fro": _fro(dev, ref)}, {"cond": 2e-6, "fro": 1e-3})
        return None, post

    # ------------------------------------------------------------------ results
    def failures(self):
        bad = []
        for kind, layer, m, bar in self.rec:
            for k, lim in bar.items():
                if not (m[k] <= lim):
                    bad.append((kind, layer, k, m[k], lim))
        return bad

    def table(self):
        out = {}
        for kind, layer, m, bar in self.rec:
            e = out.setdefault(kind, {"n": 0})
            e["n"] += 1
            for k, v in m.items():
                if v > e.get(k, (-1.0, None))[0]:
                    e[k] = (v, layer)
        return out
