"""Generate tests/golden/golden_fp64.npz: seeded inputs and fp64 expected outputs for the ops and
one whole network on the training path, computed with torch-CPU fp64 (torch.nn.functional +
autograd) -- an implementation independent of the numpy oracle.

The reference ships no tests or golden vectors and MXNet is not importable here (SURVEY.md 8c;
importing the reference's symbol files was refused), so these fixtures pin the
MXNet semantics the oracle restates (biased BN variance, SoftmaxOutput grad = p - onehot with
normalization 'null', SGD momentum form, first-max pooling) through a second implementation.

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.dirname(os.path.dirname(HERE))]
from torch_ref import T, torch_net_grads  # noqa: E402

# n, c, h, w, k, r, stride, pad, groups -- ResNet 3x3 / strided 1x1 shortcut / 7x7 stem / ResNeXt group conv
CONV = {"conv3x3": (2, 16, 9, 9, 24, 3, 1, 1, 1), "conv1x1s2": (2, 32, 8, 8, 16, 1, 2, 0, 1),
        "conv7x7s2": (1, 3, 15, 15, 8, 7, 2, 3, 1), "gconv3x3s2": (2, 32, 9, 9, 32, 3, 2, 1, 8)}


def conv_cases(out):
    for i, (name, (n, c, h, w, k, r, st, pd, g)) in enumerate(CONV.items()):
        rng = np.random.default_rng(100 + i)
        x = rng.standard_normal((n, c, h, w))
        wt = rng.standard_normal((k, c // g, r, r)) / np.sqrt(c // g * r * r)
        xt, wtt = T(x, True), T(wt, True)
        y = F.conv2d(xt, wtt, stride=st, padding=pd, groups=g)
        dy = rng.standard_normal(tuple(y.shape))
        y.backward(T(dy))
        out.update({name + "/x": x, name + "/w": wt, name + "/dy": dy, name + "/y": y.detach().numpy(),
                    name + "/dx": xt.grad.numpy(), name + "/dw": wtt.grad.numpy(),
                    name + "/cfg": np.array([n, c, h, w, k, r, st, pd, g])})


def bn_cases(out):
    for i, (fix_gamma, relu) in enumerate([(False, True), (True, False)]):
        name = "bn%d" % i
        rng = np.random.default_rng(200 + i)
        x = rng.standard_normal((3, 16, 5, 5)) * 2 + 0.5
        gamma, beta = rng.uniform(0.5, 1.5, 16), rng.standard_normal(16) * 0.1
        mm0, mv0 = rng.standard_normal(16) * 0.1, rng.uniform(0.5, 1.5, 16)
        dy = rng.standard_normal(x.shape)
        xt, gt, bt = T(x, True), T(np.ones(16) if fix_gamma else gamma, True), T(beta, True)
        z = F.batch_norm(xt, None, None, gt, bt, training=True, eps=1e-5)
        y = F.relu(z) if relu else z
        y.backward(T(dy))
        mean = x.mean(axis=(0, 2, 3))
        var = ((x - mean[None, :, None, None]) ** 2).mean(axis=(0, 2, 3))  # biased: MXNet BatchNorm
        out.update({name + "/x": x, name + "/gamma": gamma, name + "/beta": beta, name + "/dy": dy,
                    name + "/moving_mean0": mm0, name + "/moving_var0": mv0, name + "/y": y.detach().numpy(),
                    name + "/dx": xt.grad.numpy(), name + "/dgamma": np.zeros(16) if fix_gamma else gt.grad.numpy(),
                    name + "/dbeta": bt.grad.numpy(), name + "/moving_mean": 0.9 * mm0 + 0.1 * mean,
                    name + "/moving_var": 0.9 * mv0 + 0.1 * var, name + "/cfg": np.array([int(fix_gamma), int(relu)])})


def pool_cases(out):
    rng = np.random.default_rng(300)
    x = rng.standard_normal((2, 8, 11, 11))  # continuous values: no ties, the arg-max is unique
    xt = T(x, True)
    y = F.max_pool2d(xt, 3, 2, 1)
    dy = rng.standard_normal(tuple(y.shape))
    y.backward(T(dy))
    out.update({"maxpool/x": x, "maxpool/dy": dy, "maxpool/y": y.detach().numpy(), "maxpool/dx": xt.grad.numpy()})
    x = rng.standard_normal((2, 16, 7, 7))
    xt = T(x, True)
    y = xt.mean(dim=(2, 3), keepdim=True)
    dy = rng.standard_normal(tuple(y.shape))
    y.backward(T(dy))
    out.update({"gap/x": x, "gap/dy": dy, "gap/y": y.detach().numpy(), "gap/dx": xt.grad.numpy()})


def softmax_cases(out):
    rng = np.random.default_rng(400)
    x, w, b = rng.standard_normal((6, 20)), rng.standard_normal((10, 20)) * 0.3, rng.standard_normal(10) * 0.1
    label = rng.integers(0, 10, 6).astype(np.float64)
    xt, wt, bt = T(x, True), T(w, True), T(b, True)
    z = F.linear(xt, wt, bt)
    zt = z.detach().clone().requires_grad_(True)
    loss = F.cross_entropy(zt, torch.tensor(label.astype(np.int64)), reduction="sum")
    loss.backward()
    z.backward(zt.grad)
    out.update({"softmax/x": x, "softmax/w": w, "softmax/b": b, "softmax/label": label,
                "softmax/logits": z.detach().numpy(), "softmax/prob": F.softmax(zt.detach(), 1).numpy(),
                "softmax/dlogits": zt.grad.numpy(), "softmax/dx": xt.grad.numpy(), "softmax/dw": wt.grad.numpy(),
                "softmax/db": bt.grad.numpy(), "softmax/loss": np.array(loss.item())})


def sgd_cases(out):
    rng = np.random.default_rng(500)
    w, g, m = rng.standard_normal(37), rng.standard_normal(37), rng.standard_normal(37) * 0.1
    lr, wd, mom, rescale = 0.1, 1e-4, 0.9, 1.0 / 256
    # MXNet sgd_mom_update: mom = momentum*mom - lr*(rescale*grad + wd*weight); weight += mom
    m1 = mom * m - lr * (rescale * g + wd * w)
    out.update({"sgd/w": w, "sgd/g": g, "sgd/mom": m, "sgd/hyper": np.array([lr, wd, mom, rescale]),
                "sgd/w_new": w + m1, "sgd/mom_new": m1})


def network_case(out):
    from oracle import net as onet  # parameter init + graph description only; expected values from torch
    g = onet.resnet20_cifar()
    args, _ = onet.init_params(g, seed=4)
    data, label = onet.synthetic_batch(3, (3, 16, 16), 10)
    grads, loss, prob = torch_net_grads(g, args, data, label, want_loss=True)
    out["resnet20/args_abs_sum"] = np.array([np.abs(args[k]).sum() for k in g.params])
    out.update({"resnet20/data": data, "resnet20/label": label, "resnet20/loss": np.array(loss),
                "resnet20/prob": prob})
    for k in ("conv0_weight", "bn0_gamma", "stage1_unit1_conv1_weight", "stage2_unit1_sc_weight",
              "stage3_unit3_bn2_beta", "fc1_weight", "fc1_bias"):
        out["resnet20/grad/" + k] = grads[k]


def main():
    out = {}
    conv_cases(out)
    bn_cases(out)
    pool_cases(out)
    softmax_cases(out)
    sgd_cases(out)
    network_case(out)
    path = os.path.join(HERE, "golden_fp64.npz")
    np.savez_compressed(path, **out)
    print("wrote %s: %d arrays, %d bytes" % (path, len(out), os.path.getsize(path)))


if __name__ == "__main__":
    main()
