"""Per-op numpy restatement of the MXNet 1.x semantics used by the reference's hot path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py); parity against MXNet is unpinned.
Layout here is MXNet's own: NCHW activations, OIHW weights.

MXNet semantics restated (the [MXNet 1.x, un-vendored] items of SURVEY.md section 8c):
 (1) BatchNorm training: batch mean and BIASED variance over (N,H,W); moving stats
     m = momentum*m + (1-momentum)*batch; fix_gamma => gamma treated as 1 and dgamma = 0.
 (2) SoftmaxOutput backward = grad_scale*(p - onehot(label)), normalization 'null' (no 1/B);
     the 1/B comes from the optimizer's rescale_grad.
 (3) SGD momentum: mom = momentum*mom - lr*(rescale*g + wd*w); w += mom.
 (4) wd_mult = 0 for parameters not ending in _weight / _gamma.
 (5) Xavier(rnd_type='gaussian', factor_type='in', magnitude=2): N(0, sqrt(2/fan_in)).
 (6) Pooling 'valid' output size floor((H+2p-k)/s)+1; max-pool gradient goes to the first
     maximal element of the window in (r, s) scan order; global pooling ignores kernel.
 (7) FullyConnected has a bias unless no_bias.
 (8) Convolution: cross-correlation, no bias (no_bias=True in every reference conv).
 (9) The scheduler is called with num_update starting at 1.
"""
import numpy as np


# ----------------------------------------------------------------------------- precision emulation
def bf16_round(x):
    """Round to the nearest bf16 (ties to even) and widen back -- emulates bf16 storage."""
    x = np.asarray(x)
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return r.view(np.float32).astype(x.dtype)


# ----------------------------------------------------------------------------- convolution
def _windows(xp, r, s, sh, sw, p, q):
    """(N,C,Hp,Wp) padded input -> strided view (N,C,P,Q,R,S)."""
    n, c, hp, wp = xp.shape
    st = xp.strides
    return np.lib.stride_tricks.as_strided(
        xp, shape=(n, c, p, q, r, s),
        strides=(st[0], st[1], st[2] * sh, st[3] * sw, st[2], st[3]), writeable=False)


def conv_out_hw(h, w, r, s, stride, pad):
    return (h + 2 * pad[0] - r) // stride[0] + 1, (w + 2 * pad[1] - s) // stride[1] + 1


def conv2d_fwd(x, w, stride=(1, 1), pad=(0, 0), groups=1):
    """mx.sym.Convolution(no_bias=True) forward. x (N,C,H,W), w (K,C/g,R,S) -> (N,K,P,Q)."""
    n, c, h, wd = x.shape
    k, cg, r, s = w.shape
    p, q = conv_out_hw(h, wd, r, s, stride, pad)
    xp = np.pad(x, ((0, 0), (0, 0), (pad[0], pad[0]), (pad[1], pad[1])))
    win = _windows(xp, r, s, stride[0], stride[1], p, q)
    kg = k // groups
    outs = []
    for g in range(groups):
        wg = w[g * kg:(g + 1) * kg]
        wing = win[:, g * cg:(g + 1) * cg]
        # (N,Cg,P,Q,R,S) x (Kg,Cg,R,S) -> (N,P,Q,Kg)
        outs.append(np.tensordot(wing, wg, axes=([1, 4, 5], [1, 2, 3])))
    y = np.concatenate(outs, axis=3) if groups > 1 else outs[0]
    return np.ascontiguousarray(y.transpose(0, 3, 1, 2))


def conv2d_bwd(x, w, dy, stride=(1, 1), pad=(0, 0), groups=1, need_dx=True):
    """Returns (dx, dw) of conv2d_fwd."""
    n, c, h, wd = x.shape
    k, cg, r, s = w.shape
    p, q = dy.shape[2], dy.shape[3]
    xp = np.pad(x, ((0, 0), (0, 0), (pad[0], pad[0]), (pad[1], pad[1])))
    win = _windows(xp, r, s, stride[0], stride[1], p, q)
    kg = k // groups
    dw = np.empty_like(w)
    dxp = np.zeros_like(xp) if need_dx else None
    for g in range(groups):
        dyg = dy[:, g * kg:(g + 1) * kg]              # (N,Kg,P,Q)
        wing = win[:, g * cg:(g + 1) * cg]            # (N,Cg,P,Q,R,S)
        dw[g * kg:(g + 1) * kg] = np.tensordot(dyg, wing, axes=([0, 2, 3], [0, 2, 3]))
        if need_dx:
            wg = w[g * kg:(g + 1) * kg]
            # dcols (N,P,Q,Cg,R,S)
            dcols = np.tensordot(dyg, wg, axes=([1], [0]))
            for rr in range(r):
                for ss in range(s):
                    dxp[:, g * cg:(g + 1) * cg,
                        rr:rr + stride[0] * (p - 1) + 1:stride[0],
                        ss:ss + stride[1] * (q - 1) + 1:stride[1]] += \
                        dcols[:, :, :, :, rr, ss].transpose(0, 3, 1, 2)
    dx = None
    if need_dx:
        dx = dxp[:, :, pad[0]:pad[0] + h, pad[1]:pad[1] + wd]
    return dx, dw


# ----------------------------------------------------------------------------- batchnorm
def bn_train_fwd(x, gamma, beta, eps, fix_gamma):
    """mx.sym.BatchNorm training forward over axis 1. Returns y, cache."""
    axes = (0, 2, 3) if x.ndim == 4 else (0,)
    shp = (1, -1, 1, 1) if x.ndim == 4 else (1, -1)
    mean = x.mean(axis=axes)
    var = x.var(axis=axes)  # biased
    invstd = 1.0 / np.sqrt(var + eps)
    g = np.ones_like(gamma) if fix_gamma else gamma
    xhat = (x - mean.reshape(shp)) * invstd.reshape(shp)
    y = xhat * g.reshape(shp) + beta.reshape(shp)
    return y, (xhat, invstd, g, mean, var)


def bn_train_bwd(dy, cache, fix_gamma):
    xhat, invstd, g, mean, var = cache
    axes = (0, 2, 3) if dy.ndim == 4 else (0,)
    shp = (1, -1, 1, 1) if dy.ndim == 4 else (1, -1)
    m = dy.size // dy.shape[1]
    dbeta = dy.sum(axis=axes)
    dg_raw = (dy * xhat).sum(axis=axes)
    dgamma = np.zeros_like(dg_raw) if fix_gamma else dg_raw
    dx = (g * invstd).reshape(shp) * (dy - (dbeta / m).reshape(shp) - xhat * (dg_raw / m).reshape(shp))
    return dx, dgamma, dbeta


def bn_moving_update(moving_mean, moving_var, mean, var, momentum):
    return (moving_mean * momentum + mean * (1 - momentum),
            moving_var * momentum + var * (1 - momentum))


def bn_infer_fwd(x, gamma, beta, moving_mean, moving_var, eps, fix_gamma):
    shp = (1, -1, 1, 1) if x.ndim == 4 else (1, -1)
    g = np.ones_like(gamma) if fix_gamma else gamma
    return (x - moving_mean.reshape(shp)) / np.sqrt(moving_var.reshape(shp) + eps) * g.reshape(shp) + beta.reshape(shp)


def bn_global_fwd(x, gamma, beta, moving_mean, moving_var, eps, fix_gamma):
    """BatchNorm(use_global_stats=True) in training (fix_bn, core/graph_optimize.py:114-157;
    MXNet 1.x batch_norm backward, un-vendored): normalised with the moving statistics, which are
    constants (no moving-stat update). Returns y, cache."""
    shp = (1, -1, 1, 1) if x.ndim == 4 else (1, -1)
    invstd = 1.0 / np.sqrt(moving_var + eps)
    g = np.ones_like(gamma) if fix_gamma else gamma
    xhat = (x - moving_mean.reshape(shp)) * invstd.reshape(shp)
    return xhat * g.reshape(shp) + beta.reshape(shp), (xhat, invstd, g)


def bn_global_bwd(dy, cache, fix_gamma):
    """dx = gamma*invstd*dy (no batch-statistic terms), dgamma = sum(dy*xhat), dbeta = sum(dy)."""
    xhat, invstd, g = cache
    axes = (0, 2, 3) if dy.ndim == 4 else (0,)
    shp = (1, -1, 1, 1) if dy.ndim == 4 else (1, -1)
    dbeta = dy.sum(axis=axes)
    dg_raw = (dy * xhat).sum(axis=axes)
    dgamma = np.zeros_like(dg_raw) if fix_gamma else dg_raw
    return (g * invstd).reshape(shp) * dy, dgamma, dbeta


# ----------------------------------------------------------------------------- activation
def relu_fwd(x):
    return np.maximum(x, 0)


def relu_bwd(dy, y):
    return dy * (y > 0)


# ----------------------------------------------------------------------------- pooling
def pool_out_hw(h, w, kernel, stride, pad, global_pool):
    if global_pool:
        return 1, 1
    return (h + 2 * pad[0] - kernel[0]) // stride[0] + 1, (w + 2 * pad[1] - kernel[1]) // stride[1] + 1


def maxpool_fwd(x, kernel, stride, pad):
    n, c, h, w = x.shape
    p, q = pool_out_hw(h, w, kernel, stride, pad, False)
    xp = np.pad(x, ((0, 0), (0, 0), (pad[0], pad[0]), (pad[1], pad[1])), constant_values=-np.inf)
    win = _windows(xp, kernel[0], kernel[1], stride[0], stride[1], p, q).reshape(n, c, p, q, -1)
    arg = win.argmax(axis=-1)  # first maximal tap in (r, s) scan order
    y = np.take_along_axis(win, arg[..., None], axis=-1)[..., 0]
    return y, arg


def maxpool_bwd(dy, arg, x_shape, kernel, stride, pad):
    n, c, h, w = x_shape
    p, q = dy.shape[2], dy.shape[3]
    dxp = np.zeros((n, c, h + 2 * pad[0], w + 2 * pad[1]), dtype=dy.dtype)
    rr, ss = np.divmod(arg, kernel[1])
    hi = np.arange(p).reshape(1, 1, p, 1) * stride[0] + rr
    wi = np.arange(q).reshape(1, 1, 1, q) * stride[1] + ss
    ni = np.arange(n).reshape(n, 1, 1, 1)
    ci = np.arange(c).reshape(1, c, 1, 1)
    np.add.at(dxp, (np.broadcast_to(ni, dy.shape), np.broadcast_to(ci, dy.shape), hi, wi), dy)
    return dxp[:, :, pad[0]:pad[0] + h, pad[1]:pad[1] + w]


def avgpool_global_fwd(x):
    return x.mean(axis=(2, 3), keepdims=True)


def avgpool_global_bwd(dy, x_shape):
    n, c, h, w = x_shape
    return np.broadcast_to(dy / (h * w), x_shape).copy()


# ----------------------------------------------------------------------------- FC / softmax
def fc_fwd(x, w, b):
    return x @ w.T + (b if b is not None else 0)


def fc_bwd(x, w, dy):
    return dy @ w, dy.T @ x, dy.sum(axis=0)


def softmax_output_fwd(z):
    zm = z - z.max(axis=1, keepdims=True)
    e = np.exp(zm)
    return e / e.sum(axis=1, keepdims=True)


def softmax_output_bwd(prob, label, grad_scale=1.0):
    g = prob.copy()
    g[np.arange(prob.shape[0]), label.astype(np.int64)] -= 1.0
    return g * grad_scale


def cross_entropy(prob, label):
    return float(-np.log(np.maximum(prob[np.arange(prob.shape[0]), label.astype(np.int64)], 1e-30)).sum())


# ----------------------------------------------------------------------------- optimizer / init
def wd_mult_for(name):
    return 1.0 if (name.endswith("_weight") or name.endswith("_gamma")) else 0.0


def sgd_mom_update(w, g, mom, lr, wd, momentum, rescale_grad, clip_gradient=-1.0):
    """MXNet sgd_mom_update (in place on w and mom)."""
    gr = rescale_grad * g
    if clip_gradient is not None and clip_gradient > 0:
        gr = np.clip(gr, -clip_gradient, clip_gradient)
    mom *= momentum
    mom -= lr * (gr + wd * w)
    w += mom
    return w, mom


def xavier_gaussian_in(shape, rng, magnitude=2.0):
    fan_in = shape[1] * (int(np.prod(shape[2:])) if len(shape) > 2 else 1)
    return rng.normal(0.0, np.sqrt(magnitude / fan_in), size=shape)


def init_param(name, shape, rng):
    """mx.init.Xavier dispatch by name suffix."""
    if name.endswith("_weight"):
        return xavier_gaussian_in(shape, rng)
    if name.endswith("_gamma") or name.endswith("moving_var"):
        return np.ones(shape)
    return np.zeros(shape)  # _bias, _beta, moving_mean


# ----------------------------------------------------------------------------- schedulers
class MultiFactorScheduler:
    """mx.lr_scheduler.MultiFactorScheduler (used via core/scheduler.py:5-7)."""

    def __init__(self, step, factor=1.0, base_lr=0.01):
        self.step, self.factor, self.base_lr = list(step), factor, base_lr
        self.cur_step_ind, self.count = 0, 0

    def __call__(self, num_update):
        while self.cur_step_ind <= len(self.step) - 1:
            if num_update > self.step[self.cur_step_ind]:
                self.count = self.step[self.cur_step_ind]
                self.cur_step_ind += 1
                self.base_lr *= self.factor
            else:
                return self.base_lr
        return self.base_lr


class WarmupMultiFactorScheduler:
    """Restatement of core/scheduler.py:9-56 (WarmupMultiFactorScheduler)."""

    def __init__(self, base_lr, step, factor=1, warmup=False, warmup_type='constant', warmup_lr=0,
                 warmup_step=0):
        self.base_lr, self.step, self.factor = base_lr, list(step), factor
        self.cur_step_ind = 0
        self.warmup, self.warmup_type = warmup, warmup_type
        self.warmup_lr, self.warmup_step = warmup_lr, warmup_step

    def __call__(self, num_update):
        if self.warmup and num_update <= self.warmup_step:
            if self.warmup_type == 'constant':
                return self.warmup_lr
            return (self.base_lr - self.warmup_lr) / self.warmup_step * num_update + self.warmup_lr
        while self.cur_step_ind <= len(self.step) - 1:
            if num_update > self.step[self.cur_step_ind]:
                self.cur_step_ind += 1
                self.base_lr *= self.factor
            else:
                return self.base_lr
        return self.base_lr


# ----------------------------------------------------------------------------- int8 fake quant
def mx_round(x):
    """mx.nd.round: half away from zero (numpy's round is half-to-even)."""
    return np.sign(x) * np.floor(np.abs(x) + 0.5)


def quant_int8_weight(w, nbits=8):
    """symbol/quant_ops.py:17-31 (per-tensor): unit = max|w|/qmax, round(w/unit)*unit."""
    qmax = 2 ** (nbits - 1) - 1
    t = np.abs(w).max()
    unit = t / qmax
    return (mx_round(w / unit) * unit if unit > 0 else np.zeros_like(w)), t


def quant_int8_act(x, minmax, is_train, first, ema_decay=0.99, nbits=8):
    """symbol/clip_grad_quantization_int8.py:37-54: EMA(max|x|) initialised from the first batch,
    clip to +-t then round. Returns (out, new_minmax)."""
    qmax = 2 ** (nbits - 1) - 1
    if is_train:
        cur = np.abs(x).max()
        minmax = cur if first else minmax * ema_decay + cur * (1 - ema_decay)
    t = minmax
    unit = t / qmax
    xc = np.clip(x, -t, t)
    return (mx_round(xc / unit) * unit if unit > 0 else np.zeros_like(x)), minmax


def quant_int8_act_bwd(dy, x, t):
    """clip_grad_quantization_int8.py:56-67: STE masked to the open clip range."""
    return dy * ((x > -t) & (x < t))
