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

ResNeXt (C4): grouped convolutions (direct v_dot2 and block-diagonal MFMA kernels) against the bf16
rounding of the fp32 master weights, per group; the post-activation unit tail (rn_bn_apply_add) and
its backward (rn_relu_bwd_bnred). Int8 QAT (C5): every quantizer bit for bit -- the activation codes,
fake-quantized values, units and EMA threshold states (symbol/quant_ops.py:17-31,
clip_grad_quantization_int8.py:37-54), every weight quantizer's threshold, unit, codes and copies
(rn_weight_quant_pack) -- the int8 convolutions as exact fp64 sums of the device's own codes times
the two units, and the straight-through clips folded into the BatchNorm backwards, the stem's and
the FullyConnected input's.
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


def ref_fwd(x, w, stride, pad, groups=1):
    """conv forward in x's dtype (fp32, or fp64 for the exact integer sums of int8 codes): x (n,c,h,w),
    w (k,c/groups,r,s); a grouped conv multiplies each group's unfolded channels with its own filters."""
    n, c, h, wd = x.shape
    k, cg, r, s = w.shape
    p = (h + 2 * pad[0] - r) // stride[0] + 1
    q = (wd + 2 * pad[1] - s) // stride[1] + 1
    out = torch.empty(n, k, p, q, device=x.device, dtype=x.dtype)
    wm = w.to(x.dtype).reshape(groups, k // groups, cg * r * s)
    rng, step = _chunks(n, c * r * s * p * q * x.element_size())
    for i in rng:
        cols = F.unfold(x[i:i + step], (r, s), padding=pad, stride=stride)  # (ch, c*r*s, pq), channel-major
        cols = cols.view(cols.shape[0], groups, cg * r * s, p * q)
        out[i:i + step] = torch.einsum("gkj,ngjl->ngkl", wm, cols).reshape(-1, k, p, q)
    return out


def ref_dgrad(dy, w, hw, stride, pad, groups=1):
    """fp32 data gradient: dy (n,k,p,q), w (k,c/groups,r,s) -> (n,c,h,w)."""
    n, k, p, q = dy.shape
    _, cg, r, s = w.shape
    c = cg * groups
    out = torch.empty(n, c, hw[0], hw[1], device=dy.device, dtype=torch.float32)
    wt = w.reshape(groups, k // groups, cg * r * s).transpose(1, 2)  # (g, cg*r*s, k/g)
    rng, step = _chunks(n, c * r * s * p * q * 4)
    for i in rng:
        d = dy[i:i + step].reshape(-1, groups, k // groups, p * q)
        cols = torch.einsum("gjk,ngkl->ngjl", wt, d).reshape(d.shape[0], c * r * s, p * q)
        out[i:i + step] = F.fold(cols, hw, (r, s), padding=pad, stride=stride)
    return out


def ref_wgrad(x, dy, rs, stride, pad, with_abs=False, groups=1):
    """Weight gradient (k,c/groups,r,s) in fp64 (a sum over N*P*Q terms that cancels heavily: the
    BatchNorm backward makes dy zero-mean per channel). with_abs: also sum |dy| |x| (fp32), the scale
    that bounds any fp32 summation's error."""
    n, c = x.shape[:2]
    k, p, q = dy.shape[1:]
    cg, kg, crs = c // groups, k // groups, c // groups * rs[0] * rs[1]
    acc = torch.zeros(groups, kg, crs, device=x.device, dtype=torch.float64)
    accb = torch.zeros(groups, kg, crs, device=x.device, dtype=torch.float32) if with_abs else None
    rng, step = _chunks(n, 4 * c * rs[0] * rs[1] * p * q * 4)
    for i in rng:
        cols = F.unfold(x[i:i + step], rs, padding=pad, stride=stride)  # (ch, c*r*s, pq)
        ch = cols.shape[0]
        b = cols.view(ch, groups, crs, p * q).permute(1, 2, 0, 3).reshape(groups, crs, ch * p * q)
        a = dy[i:i + step].reshape(ch, groups, kg, p * q).permute(1, 2, 0, 3).reshape(groups, kg, ch * p * q)
        acc += torch.matmul(a.double(), b.double().transpose(1, 2))
        if with_abs:
            accb += torch.matmul(a.abs(), b.abs().transpose(1, 2))
    out = acc.view(k, cg, rs[0], rs[1])
    return (out, accb.view(k, cg, rs[0], rs[1])) if with_abs else out


def _round_away(v):
    """mx.nd.round / roundf: half away from zero (torch.round is half to even)."""
    return torch.sign(v) * torch.floor(v.abs() + 0.5)


def f32(v):
    """Round an fp64 result to fp32 once: for one +, -, * or / of fp32 operands this IS the correctly
    rounded fp32 operation (53 >= 2 * 24 + 2 bits: no double-rounding error)."""
    return v.float()


def quant_ref(y, t, qmax=127.0, clip=True):
    """Quantization_int8 of the fp32 tensor y with threshold t as the device computes it
    (symbol/quant_ops.py:17-31 with mx.round half away from zero): unit = t / qmax,
    code = roundf(clip(y, -t, t) / unit), value = code * unit, each an fp32 operation.
    Returns (codes fp64, values fp32, unit fp32 scalar tensor)."""
    tt = torch.tensor(float(t), dtype=torch.float32)
    unit = f32(tt.double() / qmax)
    v = torch.clamp(y.float(), -float(t), float(t)) if clip else y.float()
    if float(unit) <= 0.0:
        z = torch.zeros_like(v, dtype=torch.float64)
        return z, z.float(), unit
    u = unit.to(v.device)
    qf = f32(v.double() / u.double())
    code = _round_away(qf.double())
    return code, f32(code * u.double()), unit


def ema_refs(prev, cur, decay):
    """The quantizer's EMA state update (quant_state_update: minmax * decay + curmax * (1 - decay)) in
    fp32, both as two rounded products and a rounded sum and as the contracted fma the compiler may
    form: the device's value must be one of them."""
    d = torch.tensor(decay, dtype=torch.float32).double()
    p, c = torch.tensor(prev, dtype=torch.float32).double(), torch.tensor(cur, dtype=torch.float32).double()
    om = f32(1.0 - d).double()
    b = f32(c * om).double()
    return {float(f32(f32(p * d).double() + b)), float(f32(p * d + b)), float(f32(c * om + f32(p * d).double())),
            float(f32(c * om + p * d))}


EXACT = {"mismatch": 0.0}  # bit-identical: the fraction of differing elements


class Checker:
    def __init__(self, ex, prev_aux=None, first_batch=True):
        """prev_aux: {aux name: fp32 tensor} snapshot taken before the checked forward (the quantizers'
        EMA states); first_batch: whether that forward was the executor's first training forward."""
        self.ex = ex
        self.prev_aux = prev_aux or {}
        self.first_batch = first_batch
        self.rec = []  # (kind, layer, metrics dict, bar dict)
        self.byptr = {}
        for b in list(ex._acts.values()) + list(ex._grads.values()):
            self.byptr[b.data_ptr()] = b
        for op in ex.plan.ops:
            if op.kind == "stem":
                self.byptr[op.x8.data_ptr()] = op.x8
        self.aux_by_ptr = {ex._ap(nm).value: nm for nm in ex.aux_off}
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

    def aux_val(self, ptr):
        """The fp32 value an aux pointer (a quantizer's threshold state) holds."""
        v = ptr.value if hasattr(ptr, "value") else ptr
        return float(self.ex.aview(self.aux_by_ptr[v])[0])

    def master_oihw(self, name, groups=1):
        """An fp32 master weight (KRSC in the flat buffer) as OIHW (k, c/groups, r, s)."""
        shp = self.ex.param_shape[name]
        m = self.param(name)
        if len(shp) == 2:
            return m.view(shp[0], shp[1], 1, 1)
        k, cg, r, s_ = shp
        return m.view(k, r, s_, cg).permute(0, 3, 1, 2)

    def mismatch(self, dev, ref):
        dev, ref = dev.double(), ref.double()
        return {"mismatch": float((dev != ref).double().mean()) if dev.numel() else 0.0}

    def conv_input(self, op):
        """What the conv's kernel multiplies (or the pooling reduces): its stored input, or relu(bn(x))
        rounded to bf16 as the BN+ReLU-on-load transform produces it."""
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
            if getattr(op, "qweight", None) is not None:
                self.check_weight_quant(op)
            if op.kind == "conv":
                d = op.desc
                if getattr(op, "int8", False):
                    # exact fp64 sums of the device's own int8 codes, times the two units
                    qs, x = op.qsrc, op.x
                    xc = self.nchw(qs.codes, x.n, x.h, x.w, x.cp, x.c).double()
                    wc = self.w_from_krsc(op.wk8, d).double()
                    y = ref_fwd(xc, wc, op.stride, op.pad) * (float(qs.unit[0]) * float(op.wunit[0]))
                    kind = "conv_fwd_i8"
                elif op.groups != 1:
                    # grouped: against the bf16 rounding of the fp32 master, group by group (the compact /
                    # block-diagonal compute copies themselves are the kernel's business)
                    w = _bf16(self.master_oihw(op.weight, op.groups))
                    y = ref_fwd(self.conv_input(op), w, op.stride, op.pad, op.groups)
                    kind = "conv_fwd_grouped"
                else:
                    w = self.w_from_krsc(op.wk, d)
                    if not getattr(op, "qweight", None):  # the compute copies ARE the master rounded once
                        wm = self.master_oihw(op.weight)
                        ref = _bf16(wm) if ex.dtype == 0 else wm
                        self.add_metric("weight_copy", op.name + ":krsc", self.mismatch(w, ref), EXACT)
                        self.add_metric("weight_copy", op.name + ":crsk", self.mismatch(self.w_from_crsk(op.wc, d), ref),
                                        EXACT)
                    y = ref_fwd(self.conv_input(op), w, op.stride, op.pad)
                    kind = "conv_fwd"
                if op.res is not None:
                    y = y + self.act_nchw(op.res).to(y.dtype)
                self.add(kind, op.name, self.act_nchw(op.y), y, bar)
            elif op.kind == "quant":
                self.check_quant(op)
            elif op.kind == "add":
                self.check_add(op, bar)
            elif op.kind == "relu":
                self.add_metric("relu_fwd", op.name, self.mismatch(self.act_nchw(op.y), torch.relu(self.act_nchw(op.x))),
                                EXACT)
            elif op.kind == "stem" and op.bn is not None and op.quant is not None:
                self.check_stem_quant(op, bar)
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
                x = self.conv_input(op)  # (rn_pool_fwd_x: relu(bn(x)) as the load transform rounds it)
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

    def check_add(self, op, bar):
        """Residual add (+ ReLU); with BatchNorms applied inside it (rn_bn_apply_add, the post-activation
        unit tail): each BN output rounded to the storage type as rn_bn_apply stores it, then the add."""
        ex = self.ex

        def side(key):
            bn = None
            if getattr(op, "bn_a", None) is not None:
                if op.bn_a_key == key:
                    bn = op.bn_a
                elif op.bn_b is not None:
                    bn = op.bn_b
            if bn is None:
                return self.act_nchw(getattr(op, key))
            _, _, sc, sh = self.bn_coefs(bn)
            c = bn.x.c
            v = _fma(self.act_nchw(bn.x), sc[:c].view(1, c, 1, 1), sh[:c].view(1, c, 1, 1))
            return _bf16(v) if ex.dtype == 0 else v
        y = side("a") + side("b")
        if op.relu:
            y = torch.relu(y)
        self.add("bn_apply_add" if getattr(op, "bn_a", None) is not None else "add_fwd", op.name,
                 self.act_nchw(op.y), _bf16(y) if ex.dtype == 0 else y, bar)

    def _quant_state(self, q, cur, is_weight=False):
        """|device state - the state the update must produce| / state: 0 when it is one of the fp32
        evaluations (first batch / weights: the max itself; else the EMA, ema_refs)."""
        dev = float(self.ex.aview(q["minmax"])[0])
        if is_weight or self.first_batch:
            want = {float(torch.tensor(cur, dtype=torch.float32))}
        else:
            want = ema_refs(float(self.prev_aux[q["minmax"]][0]), cur, q["ema"])
        if dev in want:
            return 0.0, dev
        return min(abs(dev - w) for w in want) / max(abs(dev), 1e-30), dev

    def check_quant(self, op):
        """An activation Quantization_int8, bit for bit from the device's own input: max|y| -> threshold
        state (EMA), unit, int8 codes, fake-quantized values. y = the stored input, or the BatchNorm(+ReLU)
        output the quantizer applies on load (rn_quant_int8_fwd_codes_bn[2]), rounded as rn_bn_apply
        stores it."""
        x = op.x
        # (the second quantizer of a pair is written by its lead's call, rn_quant_int8_fwd_codes_bn2)
        bn = op.bn_src if op.bn_src is not None else (op.bn_lead.bn_src if op.bn_lead is not None else None)
        if bn is not None:
            _, _, sc, sh = self.bn_coefs(bn)
            c = bn.x.c
            v = _fma(self.act_nchw(bn.x), sc[:c].view(1, c, 1, 1), sh[:c].view(1, c, 1, 1))
            if bn.relu:
                v = torch.relu(v)
            y = _bf16(v) if self.ex.dtype == 0 else v
        else:
            y = self.act_nchw(x)
        cur = float(y.abs().max()) if y.numel() else 0.0
        st, t = self._quant_state(op.q, cur)
        code, val, unit = quant_ref(y, t, float((1 << (int(op.q["nbits"]) - 1)) - 1))
        val = _bf16(val) if self.ex.dtype == 0 else val
        if getattr(op, "defer_values", False):
            # the forward writes codes only: the values are checked where rn_quant_int8_expand writes them
            if not hasattr(self, "deferred_vals"):
                self.deferred_vals = {}
            self.deferred_vals[self.ex.act(op.y).data_ptr()] = (op, val)
            m = {"state": st}
        elif getattr(op, "codes_wgrad", False):  # codes only: the weight gradients multiply them (unit * code)
            m = {"state": st}
        else:
            m = {"state": st, "values": self.mismatch(self.act_nchw(op.y), val)["mismatch"]}
        if getattr(op, "codes", None) is not None:
            m["codes"] = self.mismatch(self.nchw(op.codes, x.n, x.h, x.w, x.cp, x.c), code)["mismatch"]
            m["unit"] = 0.0 if float(op.unit[0]) == float(unit) else 1.0
        self.add_metric("quant", op.q["name"], m, {k: 0.0 for k in m})

    def check_weight_quant(self, op):
        """A weight Quantization_int8 (rn_weight_quant_pack / the per-weight calls): threshold = max|w| of
        the fp32 master, the fake-quantized fp32 copy, and for int8 convolutions the unit, the int8 KRSC
        codes and the bf16 CRSK data-gradient copy; else the compute copy = the fake-quantized values
        rounded once."""
        ex = self.ex
        q = op.qweight
        wm = self.master_oihw(op.weight)
        cur = float(wm.abs().max())
        st, t = self._quant_state(q, cur, is_weight=True)
        code, val, unit = quant_ref(wm, t, float((1 << (int(q["nbits"]) - 1)) - 1), clip=False)
        shp = ex.param_shape[op.weight]
        k, cr = shp[0], shp[1]
        r_, s_ = (shp[2], shp[3]) if len(shp) == 4 else (1, 1)
        qw = op.qw.view(k, r_, s_, cr).permute(0, 3, 1, 2)
        m = {"state": st, "values": self.mismatch(qw, val)["mismatch"]}
        low = _bf16(val) if ex.dtype == 0 else val
        d = op.dfull if op.kind == "stem" else op.desc
        if getattr(op, "int8", False):
            m["unit"] = 0.0 if float(op.wunit[0]) == float(unit) else 1.0
            m["codes"] = self.mismatch(self.w_from_krsc(op.wk8, d), code)["mismatch"]
            m["crsk"] = self.mismatch(self.w_from_crsk(op.wc, d), low)["mismatch"]
        elif op.kind == "fc":
            m["krsc"] = self.mismatch(op.wk.view(d.k, d.c)[:, :d.c_real].float(), low.view(k, cr))["mismatch"]
        elif op.kind == "stem" and op.p4 is None:
            m["krsc"] = self.mismatch(self.w_from_krsc(op.wk, d), low)["mismatch"]
        self.add_metric("weight_quant", q["name"], m, {kk: 0.0 for kk in m})

    def check_stem_quant(self, op, bar):
        """The quantized stem (symbol/resnet_int8.py:96-98): bn_data's statistics, the NHWC-8 copy
        quantized in place (the stored bf16 affine input through Quantization_int8, bit for bit) and conv0
        over it."""
        ex = self.ex
        x = op.x
        b = op.bnbuf
        sc, sh = b[16:16 + x.c], b[24:24 + x.c]
        data = ex._in_bufs[ex._in_idx].view(x.n, x.c, x.h, x.w).float()
        mean = data.double().mean(dim=(0, 2, 3))
        var = data.double().var(dim=(0, 2, 3), unbiased=False)
        inv = 1.0 / torch.sqrt(var + op.bn["eps"])
        self.add_metric("bn_fwd", "bn_data", {"mean": float(((b[0:x.c].double() - mean).abs() /
                                                               torch.sqrt(var)).max()),
                                              "invstd": _maxr(b[8:8 + x.c], inv)},
                        {"mean": 1e-5, "invstd": 1e-5})
        aff = _fma(data, sc.view(1, -1, 1, 1), sh.view(1, -1, 1, 1))
        y = _bf16(aff) if ex.dtype == 0 else aff
        cur = float(y.abs().max())
        st, t = self._quant_state(op.quant, cur)
        _, val, _ = quant_ref(y, t, float((1 << (int(op.quant["nbits"]) - 1)) - 1))
        val = _bf16(val) if ex.dtype == 0 else val
        x8 = self.nchw(op.x8, x.n, x.h, x.w, 8, x.c)
        self.add_metric("quant", op.quant["name"], {"state": st, "values": self.mismatch(x8, val)["mismatch"]},
                        {"state": 0.0, "values": 0.0})
        y0 = ref_fwd(x8, self.w_from_krsc(op.wk, op.dfull), op.stride, op.pad)
        self.add("conv_fwd", op.name, self.act_nchw(op.y), y0, bar)

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
            if d.groups > 1:  # the bf16 rounding of the master, per group (as the forward)
                w = _bf16(self.master_oihw(op.weight, d.groups))
            else:
                w = self.w_from_crsk(op.wc, d)
            ref = ref_dgrad(dy, w, (d.h, d.w), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w), d.groups)
            if state.get("add") is not None:
                ref = ref + self.nchw(state["add"], n, d.h, d.w, d.c, d.c_real)
            dev = self.nchw(self.t(outp), n, d.h, d.w, d.c, d.c_real)
            self.add(("dgrad_bnred" if bnred else "dgrad") + ("_grouped" if d.groups > 1 else ""), op.name, dev,
                     ref, BF16_BAR if self.ex.dtype == 0 else F32_BAR)
        return (self._snap(addp, state, "add") if addp is not None else None), post

    def _h_rn_conv_bwd_data(self, args, state):
        return self._dgrad(args, state)

    def _h_rn_conv_bwd_data_bnred(self, args, state):
        if args[3] is None:  # reduction only (the first pass of the recompute): nothing stored; its partials
            return None, (lambda: None)  # are checked through dgamma / dbeta / dx of the apply below
        return self._dgrad(args, state, bnred=True)

    def _h_rn_conv_bwd_data_bnred_clip(self, args, state):
        # (its reduction carries the folded quantizer clip: checked through the BN backward it feeds)
        return self._dgrad(args, state, bnred=True)

    def _h_rn_conv_bwd_data_bnred_clip2(self, args, state):
        """A quantizer pair's later data gradient: dx = [y < t1] * its dgrad + [y < t2] * the other
        quantizer's stored gradient, y = bf16(BN output) (clip_grad_quantization_int8.py's STE of each, as
        rn_bn_bwd's relu_clip2_dz sums them) -- vs the fp32 dgrad of the device's dy (its BN reduction:
        checked through the BN backward it feeds)."""
        d = args[0]._obj
        dyp, wcp, dxp, otp, xp, c1p, c2p = args[1], args[2], args[3], args[4], args[5], args[9], args[10]
        op = self.wc_op[wcp.value]
        if not hasattr(self, "bn_by_sm_x"):
            self.bn_by_sm_x = {self.ex.act(o.x).data_ptr(): o for o in self.ex.plan.ops if o.kind == "bn"}
        bn = self.bn_by_sm_x[xp.value]
        snap = self._snap(otp, state, "other")

        def post():
            n = d.n
            dy = self.nchw(self.t(dyp), n, d.p, d.q, d.k_pad, d.k)
            w = self.w_from_crsk(op.wc, d)
            g = ref_dgrad(dy, w, (d.h, d.w), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w))
            _, _, sc, sh = self.bn_coefs(bn)
            c = d.c_real
            y = _bf16(_fma(self.act_nchw(bn.x), sc[:c].view(1, c, 1, 1), sh[:c].view(1, c, 1, 1)))
            other = self.nchw(state["other"], n, d.h, d.w, d.c, d.c_real)
            ref = g * (y < self.aux_val(c1p)) + other * (y < self.aux_val(c2p))
            dev = self.nchw(self.t(dxp), n, d.h, d.w, d.c, d.c_real)
            self.add("dgrad_bnred_clip2", op.name, dev, ref, BF16_BAR)
        return snap, post

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

    def _wgrad(self, args, state, xf=False, p4=False, xval=None):
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
                if xval is not None:
                    x = xval()
                elif xf:
                    x = self.bn_relu_input(self.bn_by_sm_x[xp.value])
                else:
                    x = self.nchw(self.t(xp), n, d.h, d.w, d.c, d.c_real)
                ref, rab = ref_wgrad(x, dy, (d.r, d.s), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w), with_abs=True,
                                     groups=d.groups)
            dev = self.ex.gview(name).view(d.k, d.r, d.s, d.c_real // d.groups).permute(0, 3, 1, 2)
            if self.ex.param_layout[name] != "krsc":  # FC: (k, c)
                dev = self.ex.gview(name).view(d.k, d.c_real, 1, 1)
            # cond: |dev - ref| per element over sum |dy| |x| of its terms (an fp32 summation of n terms
            # errs by at most ~n * 2^-24 of that; blocked / split sums far less)
            m = {"fro": _fro(dev, ref), "max": _maxr(dev, ref),
                 "cond": float(((dev.double() - ref).abs() / (rab.double() + 1e-30)).max())}
            self.add_metric("wgrad_grouped" if d.groups > 1 else "wgrad", name, m, WGRAD_BAR)
        return None, post

    def _h_rn_conv_bwd_filter(self, args, state):
        return self._wgrad(args, state)

    def _h_rn_conv_bwd_filter_ws(self, args, state):
        return self._wgrad(args, state)

    def _h_rn_conv_bwd_filter_x(self, args, state):
        if not hasattr(self, "bn_by_sm_x"):
            self.bn_by_sm_x = {self.ex.act(op.x).data_ptr(): op for op in self.ex.plan.ops if op.kind == "bn"}
        return self._wgrad(args, state, xf=True)

    def _h_rn_conv_bwd_filter_i8(self, args, state):
        """The weight gradient of an int8 conv from its input's codes (rn_conv_bwd_filter_i8): against the
        oracle on x = unit * code (the codes themselves are checked bit for bit at the quantizer)."""
        d = args[0]._obj
        cp_, up_ = args[1], args[2]
        q = {o.codes.data_ptr(): o for o in self.ex.plan.ops
             if o.kind == "quant" and getattr(o, "codes", None) is not None}[cp_.value]
        assert q.unit.data_ptr() == up_.value

        def xval():
            return self.nchw(q.codes, d.n, d.h, d.w, d.c, d.c_real) * float(q.unit[0])  # (fp32, as the values)
        return self._wgrad((args[0], None, args[3], args[4]), state, xval=xval)

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
        desc = op.desc
        if op.relu and desc.clip:
            # the folded straight-through clips of the quantizer(s) that read this BN's output
            # (rn_bn_desc.clip / clip2 / dy2): dz = [y > 0] * [y < t] * dy (two: rounded sum), y as stored
            yv = torch.relu(_fma(x.float(), sc[:c].view(1, c, 1, 1), sh[:c].view(1, c, 1, 1)))
            yv = _bf16(yv) if self.ex.dtype == 0 else yv
            g = dy * (yv < self.aux_val(desc.clip))
            if desc.dy2:
                dy2 = self.nchw(self.byptr[desc.dy2], t.n, t.h, t.w, t.cp, c).double()
                g = g + dy2 * (yv < self.aux_val(desc.clip2))
                g = (_bf16(g.float()) if self.ex.dtype == 0 else g.float()).double()
            dz = g * (yv > 0)
        elif op.relu:
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

    def _h_rn_relu_bwd_bnred(self, args, state):
        """The post-activation unit tail's backward: g = dy * [y > 0] (exact); its BatchNorm reductions are
        checked through the rn_bn_bwd_part calls that finish those BNs (dgamma, dbeta, dx)."""
        d, yp, dyp, gp = args[0]._obj, args[1], args[2], args[3]
        snap = self._snap(dyp, state, "dy")

        def post():
            m, cp = d.m, d.c
            y = self.t(yp)[:m * cp].float()
            ref = state["dy"][:m * cp].float() * (y > 0)
            self.add_metric("relu_bwd_bnred", "add", self.mismatch(self.t(gp)[:m * cp].float(), ref), EXACT)
        return snap, post

    def _h_rn_relu_bwd(self, args, state):
        n, yp, dyp, dxp, addp = args[0], args[2], args[3], args[4], args[5]
        sd, sa = self._snap(dyp, state, "dy"), self._snap(addp, state, "add")

        def pre():
            sd()
            sa()

        def post():
            ref = state["dy"][:n].float() * (self.t(yp)[:n].float() > 0)
            if state["add"] is not None:
                ref = ref + state["add"][:n].float()
            self.add("relu_bwd", "relu", self.t(dxp)[:n].float(), ref, BF16_BAR if self.ex.dtype == 0 else F32_BAR)
        return pre, post

    def _h_rn_quant_int8_expand(self, args, state):
        """A quantizer's deferred fake-quantized values (expanded from its codes on the weight-gradient
        stream): bit for bit the values the oracle's quantizer gives for the forward's input."""
        outp = args[4]

        def post():
            op, val = self.deferred_vals.pop(outp.value)
            m = {"values": self.mismatch(self.act_nchw(op.y), val)["mismatch"]}
            self.add_metric("quant_expand", op.q["name"], m, {"values": 0.0})
        return None, post

    def _h_rn_quant_int8_bwd(self, args, state):
        """A Quantization_int8's straight-through backward that is not folded into a BatchNorm (the
        FullyConnected input's): dx = dy * [-t < x < t] (+ add) (clip_grad_quantization_int8.py:55-67)."""
        n, xp, dyp, dxp, mmp, is_w, addp = args[1], args[2], args[3], args[4], args[5], args[6], args[7]
        sd, sa = self._snap(dyp, state, "dy"), self._snap(addp, state, "add")

        def pre():
            sd()
            sa()

        def post():
            x = self.t(xp)[:n].float()
            t = float("inf") if (is_w or mmp is None) else self.aux_val(mmp)
            ref = state["dy"][:n].float() * ((x > -t) & (x < t))
            if state["add"] is not None:
                ref = ref + state["add"][:n].float()
            ref = _bf16(ref) if self.ex.dtype == 0 else ref
            self.add_metric("quant_bwd", "ste", self.mismatch(self.t(dxp)[:n].float(), ref), EXACT)
        return pre, post

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

    # (its BN reduction: checked through the BN backward it feeds, rn_bn_bwd_part's dx / dgamma / dbeta)
    _h_rn_pool_bwd_bnred = _h_rn_pool_bwd

    def _h_rn_col_sum(self, args, state):
        _, m, c, ld, xp, outp = args[:6]

        def post():
            x = self.t(xp).view(m, ld)[:, :c].double()
            off = (outp.value - self.ex.grad.data_ptr()) // 4
            dev = self.ex.grad[off:off + c]
            self.add("fc_bias_grad", "fc1_bias", dev, x.sum(0), F32_BAR)
        return None, post

    def _stem_weight(self, wmp, d):
        """conv0's fp32 KRSC weight behind a pointer: the master, or (int8 graph) its fake-quantized copy."""
        n = d.k * d.r * d.s * d.c_real
        for buf in [self.ex.master] + [op.qw for op in self.ex.plan.ops if getattr(op, "qw", None) is not None]:
            off = (wmp.value - buf.data_ptr()) // 4
            if 0 <= off and off + n <= buf.numel():
                return buf[off:off + n].view(d.k, d.r, d.s, d.c_real).permute(0, 3, 1, 2).float()
        raise KeyError(wmp.value)

    def _stem_dbeta(self, d, dyp, wmp, dbp, clip=None):
        name = self.grad_name(dbp)
        dy = self.nchw(self.t(dyp), d.n, d.p, d.q, d.k_pad, d.k)
        w = self._stem_weight(wmp, d)
        args_ = ((d.h, d.w), (d.stride_h, d.stride_w), (d.pad_h, d.pad_w))
        g = ref_dgrad(dy, w, *args_).double()
        ga = ref_dgrad(dy.abs(), w.abs(), *args_).double()
        if clip is not None:  # the input quantizer's straight-through clip: no gradient where it clipped
            g, ga = g * clip, ga * clip
        ref, rab = g.sum(dim=(0, 2, 3)), ga.sum(dim=(0, 2, 3))
        dev = self.ex.gview(name)[:d.c_real].double()
        # dbeta[c] sums ~n h w data-gradient terms that cancel to 1e-3 .. 1e-7 of their magnitudes (cancel =
        # sum |terms| / |sum|: 7e3 .. 3e6 measured at 256 x 224^2), so its relative (fro) error is fp32
        # summation noise times that factor -- informational: any change of summation order moves it by a
        # random factor of that size. The int8 stem's four image chunks (rn_stem_clip_wgrad_chunk: each
        # chunk's clip-mask weight gradient, then the chunks' dot products added in chunk order) changed the
        # order, and the relative error with it (2.75e-4 -> 3.36e-3), while the error
        # stayed ~1e3 x under the fp32 summation bound (cond 7e-10: an fp32 tree over 1.3e7 terms may
        # reach ~24 x 6e-8 = 1.4e-6 of sum |terms|). The bars: cond (|dev - ref| over the sum of the
        # magnitudes, the summation bound) and err_terms (|dev - ref| in units of the mean |term|: a clip
        # mask flipped at one input moves its channel by about one term; measured 2e-5 .. 1.6e-2, the bar
        # three times the largest)
        nterm = float(d.n * d.h * d.w)
        self.add_metric("stem_dbeta", name, {"cond": float(((dev - ref).abs() / rab).max()),
                                             "fro": _fro(dev, ref),
                                             "cancel": float((rab / (ref.abs() + 1e-300)).max()),
                                             "err_terms": float(((dev - ref).abs() / (rab / nterm)).max())},
                        {"cond": 2e-6, "err_terms": 0.05})

    def _h_rn_stem_shift_grad(self, args, state):
        """bn_data's beta gradient without the stem's data gradient: dbeta[c] = sum over the image of
        conv0's data gradient (fix_gamma BatchNorm), from the weights conv0 ran with. With an input
        quantizer the clip gradient that follows completes it (checked there)."""
        d, dyp, wmp, dbp = args[0]._obj, args[1], args[2], args[3]
        if any(nm in ("rn_stem_quant_clip_grad", "rn_stem_clip_dbeta") for nm, _, _ in self.ex._bwd):
            return None, (lambda: None)
        return None, (lambda: self._stem_dbeta(d, dyp, wmp, dbp))

    def _h_rn_stem_clip_mask(self, args, state):
        return None, (lambda: None)  # (its masks: checked through the clip gradient they produce)

    def _h_rn_stem_clip_wgrad(self, args, state):
        """The int8 stem's weight gradient over the real and clip-mask channels: dW (real channels) vs the
        oracle's; the mask part is checked through bn_data's beta gradient (rn_stem_clip_dbeta)."""
        self._stem_dy = args[2]
        return self._wgrad(args, state)

    def _h_rn_stem_clip_wgrad_chunk(self, args, state):
        """The same over image chunks (executor._stem_chunks): dW is complete after the last chunk, checked
        there against the whole batch."""
        d = args[0]._obj
        op = [o for o in self.ex.plan.ops if o.kind == "stem"][0]
        i = (args[1].value - op.x8.data_ptr()) // (d.n * d.h * d.w * 8 * 2)
        if not args[8]:
            return None, (lambda: None)
        dy0 = types.SimpleNamespace(value=args[2].value - i * d.n * d.p * d.q * d.k_pad * 2)
        full = (types.SimpleNamespace(_obj=op.dfull), types.SimpleNamespace(value=op.x8.data_ptr()), dy0, args[3])
        self._stem_dy = dy0
        return self._wgrad(full, state)

    def _h_rn_stem_clip_dbeta(self, args, state):
        """rn_stem_shift_grad + rn_stem_clip_wgrad's mask part + this == the clipped beta gradient of
        _h_rn_stem_quant_clip_grad, with the same bars."""
        d, wmp, dbp = args[0]._obj, args[2], args[3]
        op = [o for o in self.ex.plan.ops if o.kind == "stem"][0]

        def post():
            x = op.x
            data = self.ex._in_bufs[self.ex._in_idx].view(x.n, x.c, x.h, x.w).float()
            sc, sh = op.bnbuf[16:16 + x.c], op.bnbuf[24:24 + x.c]
            v = _fma(data, sc.view(1, -1, 1, 1), sh.view(1, -1, 1, 1))
            t = self.aux_val(self.ex._ap(op.quant["minmax"]))
            self._stem_dbeta(d, self._stem_dy, wmp, dbp, clip=((v > -t) & (v < t)).double())
        return None, post

    def _h_rn_stem_quant_clip_grad(self, args, state):
        """rn_stem_shift_grad + this: dbeta[c] = sum of conv0's data gradient over the unclipped inputs,
        clipped = !(-t < fmaf(x, scale, shift) < t) on the fp32 input (the STE of
        clip_grad_quantization_int8.py on bn_data's fp32 output)."""
        d, xp, scp, shp, mmp, dyp, wmp, dbp = args[0]._obj, args[1], args[2], args[3], args[4], args[5], args[6], args[7]
        op = [o for o in self.ex.plan.ops if o.kind == "stem"][0]

        def post():
            x = op.x
            data = self.ex._in_bufs[self.ex._in_idx].view(x.n, x.c, x.h, x.w).float()
            sc, sh = op.bnbuf[16:16 + x.c], op.bnbuf[24:24 + x.c]
            v = _fma(data, sc.view(1, -1, 1, 1), sh.view(1, -1, 1, 1))
            t = self.aux_val(mmp)
            self._stem_dbeta(d, dyp, wmp, dbp, clip=((v > -t) & (v < t)).double())
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
