"""librn (fp32 parity path) against the committed golden fixtures (tests/golden/golden_fp64.npz,
torch-CPU fp64, see tests/golden/make_golden.py). Tolerance: 2e-5 of max |ref| (fp32
accumulation order vs fp64), 1e-4 for reductions over a whole batch (BN dgamma/dbeta)."""
import ctypes as C
import os

import numpy as np
import pytest
import torch

from rn import lib as L
from gpu_util import F32, from_nhwc, p, pad8, rel_err, stream, to_nhwc

pytestmark = pytest.mark.gpu
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_fp64.npz"))
TOL = 2e-5


def _f(a, dev):
    return torch.tensor(np.asarray(a, dtype=np.float32), device=dev)


@pytest.mark.parametrize("name", ["conv3x3", "conv1x1s2", "conv7x7s2", "gconv3x3s2"])
def test_conv_golden_gpu(gpu, name):
    n, c, h, w, k, r, st, pd, g = (int(v) for v in G[name + "/cfg"])
    x, wt, dy = G[name + "/x"], G[name + "/w"], G[name + "/dy"]
    cp = c if g > 1 else pad8(c)
    kp = k if g > 1 else pad8(k)
    d = L.ConvDesc(dtype=F32, n=n, h=h, w=w, c=cp, c_real=c, k=k, k_pad=kp, r=r, s=r, stride_h=st, stride_w=st,
                   pad_h=pd, pad_w=pd, groups=g)
    L.call("rn_conv_desc_init", C.byref(d))
    lib = L.load()
    master = _f(wt.transpose(0, 2, 3, 1), gpu).reshape(-1)
    wk = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 0), dtype=torch.float32, device=gpu)
    wc = torch.zeros(lib.rn_conv_pack_numel(C.byref(d), 1), dtype=torch.float32, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(master), p(wk), p(wc), stream())
    xd, dyd = to_nhwc(x, F32, gpu, cp), to_nhwc(dy, F32, gpu, kp)
    y = torch.zeros((n, d.p, d.q, kp), dtype=torch.float32, device=gpu)
    L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(y), F32, None, None, stream())
    dw = torch.zeros(master.numel(), dtype=torch.float32, device=gpu)
    dx = torch.zeros((n, h, w, cp), dtype=torch.float32, device=gpu)
    if c % 8 == 0 or r * r == 1:
        L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dyd), p(dw), stream())
    L.call("rn_conv_bwd_data", C.byref(d), p(dyd), p(wc), p(dx), None, stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(y, k), G[name + "/y"]) < TOL
    assert rel_err(from_nhwc(dx, c), G[name + "/dx"]) < TOL
    if c % 8 == 0 or r * r == 1:  # the 3-channel stem's wgrad runs through im2col (test_kernels_gpu)
        dw_h = dw.cpu().numpy().reshape(k, r, r, c // g).transpose(0, 3, 1, 2)
        assert rel_err(dw_h, G[name + "/dw"]) < TOL


@pytest.mark.parametrize("name", ["bn0", "bn1"])
def test_bn_golden_gpu(gpu, name):
    fix_gamma, relu = (int(v) for v in G[name + "/cfg"])
    x, dy = G[name + "/x"], G[name + "/dy"]
    n, c, h, w = x.shape
    cp = pad8(c)
    d = L.BNDesc(dtype=F32, m=n * h * w, c=cp, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=fix_gamma, relu=relu)
    pad = lambda a: _f(np.pad(a, (0, cp - c)), gpu)
    gam, bet = pad(G[name + "/gamma"]), pad(G[name + "/beta"])
    mm, mv = pad(G[name + "/moving_mean0"]), pad(G[name + "/moving_var0"])
    sm, si, sc, sh = [torch.zeros(cp, dtype=torch.float32, device=gpu) for _ in range(4)]
    ws = torch.zeros(L.load().rn_bn_workspace_bytes(C.byref(d)) // 4 + 16, dtype=torch.float32, device=gpu)
    xd = to_nhwc(x, F32, gpu)
    yd = torch.zeros_like(xd)
    L.call("rn_bn_fwd_train", C.byref(d), p(xd), p(yd), p(gam), p(bet), p(mm), p(mv), p(sm), p(si), p(sc), p(sh),
           p(ws), stream())
    dyd = to_nhwc(dy, F32, gpu)
    dxd = torch.zeros_like(xd)
    dg, db = torch.zeros(cp, dtype=torch.float32, device=gpu), torch.zeros(cp, dtype=torch.float32, device=gpu)
    L.call("rn_bn_bwd", C.byref(d), p(xd), p(dyd), p(dxd), None, p(gam), p(sm), p(si), p(sc), p(sh), p(dg), p(db),
           p(ws), stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(yd, c), G[name + "/y"]) < TOL
    assert rel_err(from_nhwc(dxd, c), G[name + "/dx"]) < 1e-4
    assert rel_err(db.cpu().numpy()[:c], G[name + "/dbeta"]) < 1e-4
    if fix_gamma:
        assert np.all(dg.cpu().numpy() == 0)
    else:
        assert rel_err(dg.cpu().numpy()[:c], G[name + "/dgamma"]) < 1e-4
    assert rel_err(mm.cpu().numpy()[:c], G[name + "/moving_mean"]) < 1e-5
    assert rel_err(mv.cpu().numpy()[:c], G[name + "/moving_var"]) < 1e-5


def test_pool_golden_gpu(gpu):
    x, dy = G["maxpool/x"], G["maxpool/dy"]
    n, c, h, w = x.shape
    d = L.PoolDesc(dtype=F32, n=n, h=h, w=w, c=pad8(c), r=3, s=3, stride_h=2, stride_w=2, pad_h=1, pad_w=1,
                   type=L.RN_POOL_MAX, global_pool=0)
    L.call("rn_pool_desc_init", C.byref(d))
    xd = to_nhwc(x, F32, gpu)
    yd = torch.zeros((n, d.p, d.q, pad8(c)), dtype=torch.float32, device=gpu)
    am = torch.zeros(yd.numel(), dtype=torch.uint8, device=gpu)
    L.call("rn_pool_fwd", C.byref(d), p(xd), p(yd), p(am), stream())
    dxd = torch.zeros_like(xd)
    L.call("rn_pool_bwd", C.byref(d), p(to_nhwc(dy, F32, gpu)), p(am), p(dxd), None, stream())
    xg, dyg = G["gap/x"], G["gap/dy"]
    gd = L.PoolDesc(dtype=F32, n=xg.shape[0], h=xg.shape[2], w=xg.shape[3], c=pad8(xg.shape[1]), type=L.RN_POOL_AVG,
                    global_pool=1)
    L.call("rn_pool_desc_init", C.byref(gd))
    xgd = to_nhwc(xg, F32, gpu)
    ygd = torch.zeros((xg.shape[0], 1, 1, pad8(xg.shape[1])), dtype=torch.float32, device=gpu)
    L.call("rn_pool_fwd", C.byref(gd), p(xgd), p(ygd), None, stream())
    dxg = torch.zeros_like(xgd)
    L.call("rn_pool_bwd", C.byref(gd), p(to_nhwc(dyg, F32, gpu)), None, p(dxg), None, stream())
    torch.cuda.synchronize()
    assert rel_err(from_nhwc(yd, c), G["maxpool/y"]) < 1e-7
    assert rel_err(from_nhwc(dxd, c), G["maxpool/dx"]) < 1e-7
    assert rel_err(from_nhwc(ygd, xg.shape[1]), G["gap/y"]) < TOL
    assert rel_err(from_nhwc(dxg, xg.shape[1]), G["gap/dx"]) < TOL


def test_fc_softmax_golden_gpu(gpu):
    x, wt, b, label = G["softmax/x"], G["softmax/w"], G["softmax/b"], G["softmax/label"]
    n, cin = x.shape
    k = wt.shape[0]
    d = L.ConvDesc(dtype=F32, n=n, h=1, w=1, c=pad8(cin), c_real=cin, k=k, k_pad=pad8(k), r=1, s=1, stride_h=1,
                   stride_w=1, pad_h=0, pad_w=0, groups=1)
    L.call("rn_conv_desc_init", C.byref(d))
    master = _f(wt, gpu).reshape(-1)
    wk = torch.zeros(k * pad8(cin), dtype=torch.float32, device=gpu)
    wc = torch.zeros(pad8(cin) * pad8(k), dtype=torch.float32, device=gpu)
    L.call("rn_conv_weight_pack", C.byref(d), p(master), p(wk), p(wc), stream())
    xd = to_nhwc(x[:, :, None, None], F32, gpu)
    bd = _f(b, gpu)
    z = torch.zeros((n, pad8(k)), dtype=torch.float32, device=gpu)
    L.call("rn_conv_fwd", C.byref(d), p(xd), p(wk), p(z), F32, None, p(bd), stream())
    lab = _f(label, gpu)
    prob = torch.zeros((n, k), dtype=torch.float32, device=gpu)
    dz = torch.zeros((n, pad8(k)), dtype=torch.float32, device=gpu)
    stats = torch.zeros(4, dtype=torch.float32, device=gpu)
    L.call("rn_softmax_output", F32, n, k, pad8(k), p(z), p(lab), p(prob), p(dz), C.c_float(1.0), p(stats), stream())
    dx = torch.zeros((n, 1, 1, pad8(cin)), dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_data", C.byref(d), p(dz), p(wc), p(dx), None, stream())
    dw = torch.zeros(k * cin, dtype=torch.float32, device=gpu)
    L.call("rn_conv_bwd_filter", C.byref(d), p(xd), p(dz), p(dw), stream())
    db = torch.zeros(k, dtype=torch.float32, device=gpu)
    L.call("rn_col_sum", F32, n, k, pad8(k), p(dz), p(db), 0, stream())
    torch.cuda.synchronize()
    assert rel_err(z.cpu().numpy()[:, :k], G["softmax/logits"]) < TOL
    assert rel_err(prob.cpu().numpy(), G["softmax/prob"]) < TOL
    assert rel_err(dz.cpu().numpy()[:, :k], G["softmax/dlogits"]) < TOL
    assert rel_err(dx.cpu().numpy().reshape(n, -1)[:, :cin], G["softmax/dx"]) < TOL
    assert rel_err(dw.cpu().numpy().reshape(k, cin), G["softmax/dw"]) < TOL
    assert rel_err(db.cpu().numpy(), G["softmax/db"]) < TOL
    assert abs(stats.cpu().numpy()[0] - float(G["softmax/loss"])) < 1e-4 * float(G["softmax/loss"])


def test_sgd_golden_gpu(gpu):
    w, g, m = G["sgd/w"], G["sgd/g"], G["sgd/mom"]
    lr, wd, mom, rescale = (float(v) for v in G["sgd/hyper"])
    wd_, gd, md = _f(w, gpu), _f(g, gpu), _f(m, gpu)
    offs = torch.tensor([0], dtype=torch.int64, device=gpu)
    sizes = torch.tensor([w.size], dtype=torch.int64, device=gpu)
    wds = torch.tensor([wd], dtype=torch.float32, device=gpu)
    L.call("rn_sgd_mom_update", 1, p(offs), p(sizes), p(wds), p(wd_), p(gd), p(md), None, F32, C.c_float(lr), None,
           C.c_float(mom), C.c_float(rescale), C.c_float(-1.0), stream())
    torch.cuda.synchronize()
    assert rel_err(wd_.cpu().numpy(), G["sgd/w_new"]) < 1e-6
    assert rel_err(md.cpu().numpy(), G["sgd/mom_new"]) < 1e-5
