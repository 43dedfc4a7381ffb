"""Stock-stack comparison point (measurement only, not part of the product): the same ResNet-50 v2
convolutions / training step through PyTorch-ROCm's own kernels (MIOpen convolutions, channels_last,
bf16) on the same GPU.

python tools/torch_ref_bench.py convs   [--batch 256] [--iters 20]   per unique conv shape: fwd / dgrad / wgrad
python tools/torch_ref_bench.py step    [--batch 256] [--steps 10]   whole train step (bf16 weights, SGD momentum)
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd")]


def unique_convs(batch):
    from rn import graphs
    from rn.executor import Plan
    plan = Plan(graphs.resnet50(), [("data", (batch, 3, 224, 224))], [("softmax_label", (batch,))])
    shapes = {}
    for op in plan.ops:
        if op.kind != "conv":
            continue
        x, y = op.x, op.y
        key = (x.n, x.h, x.w, x.c, y.c, op.kernel, op.stride, op.pad, op.groups)
        shapes.setdefault(key, [op.name, 0])[1] += 1
    return shapes


def time_fn(torch, fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def convs(a):
    import torch
    import torch.nn.functional as F
    dev = torch.device("cuda:0")
    cl = torch.channels_last
    tot = [0.0, 0.0, 0.0]
    for (n, h, w, c, k, kern, stride, pad, g), (name, cnt) in unique_convs(a.batch).items():
        x = torch.randn(n, c, h, w, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
        wt = (torch.randn(k, c // g, *kern, device=dev) * 0.05).to(torch.bfloat16).to(memory_format=cl)
        y = F.conv2d(x, wt, None, stride, pad, 1, g)
        dy = torch.randn_like(y).contiguous(memory_format=cl)
        fwd = lambda: F.conv2d(x, wt, None, stride, pad, 1, g)
        bwd = lambda mask: torch.ops.aten.convolution_backward(dy, x, wt, None, list(stride), list(pad), [1, 1],
                                                               False, [0, 0], g, mask)
        ms = [time_fn(torch, fwd, a.iters), time_fn(torch, lambda: bwd([True, False, False]), a.iters),
              time_fn(torch, lambda: bwd([False, True, False]), a.iters)]
        flops = 2.0 * n * y.shape[2] * y.shape[3] * k * (c // g) * kern[0] * kern[1]
        for i in range(3):
            tot[i] += ms[i] * cnt
        print("%-26s %3d %dx%dx%d>%d k%d s%d  " % (name[:26], cnt, h, w, c, k, kern[0], stride[0]) +
              "".join("%8.1fus %5.0fT" % (m * 1e3, flops / m / 1e9) for m in ms), flush=True)
    print("per-step totals (MIOpen, bf16 channels_last): fwd %.3f ms  dgrad %.3f ms  wgrad %.3f ms" % tuple(tot))


def build_resnet50_v2(torch, nn):
    """Pre-activation ResNet-50 with the layer structure of symbol/resnet.py (bottle_neck=True)."""
    class Unit(nn.Module):
        def __init__(s, cin, cout, stride, dim_match):
            super().__init__()
            mid = cout // 4
            s.bn1, s.bn2, s.bn3 = nn.BatchNorm2d(cin, eps=2e-5), nn.BatchNorm2d(mid, eps=2e-5), nn.BatchNorm2d(mid, eps=2e-5)
            s.c1 = nn.Conv2d(cin, mid, 1, bias=False)
            s.c2 = nn.Conv2d(mid, mid, 3, stride, 1, bias=False)
            s.c3 = nn.Conv2d(mid, cout, 1, bias=False)
            s.sc = None if dim_match else nn.Conv2d(cin, cout, 1, stride, bias=False)

        def forward(s, x):
            a1 = torch.relu(s.bn1(x))
            y = s.c1(a1)
            y = s.c2(torch.relu(s.bn2(y)))
            y = s.c3(torch.relu(s.bn3(y)))
            return y + (x if s.sc is None else s.sc(a1))

    layers = [nn.BatchNorm2d(3, eps=2e-5), nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64, eps=2e-5),
              nn.ReLU(), nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for i, (units, cout) in enumerate(zip([3, 4, 6, 3], [256, 512, 1024, 2048])):
        for j in range(units):
            layers.append(Unit(cin, cout, (1 if i == 0 else 2) if j == 0 else 1, j > 0))
            cin = cout
    layers += [nn.BatchNorm2d(cin, eps=2e-5), nn.ReLU(), nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(cin, 1000)]
    return nn.Sequential(*layers)


def step(a):
    import torch
    import torch.nn as nn
    dev = torch.device("cuda:0")
    model = build_resnet50_v2(torch, nn).to(dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.rand(a.batch, 3, 224, 224, device=dev, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
    lab = torch.randint(0, 1000, (a.batch,), device=dev)
    lossf = nn.CrossEntropyLoss()

    def one():
        opt.zero_grad(set_to_none=True)
        loss = lossf(model(x).float(), lab)
        loss.backward()
        opt.step()
    for _ in range(a.warmup):
        one()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / a.steps
    print('{"stack": "pytorch-rocm eager (MIOpen), bf16 weights, channels_last", "batch": %d, '
          '"ms_per_step": %.3f, "images_per_sec": %.1f}' % (a.batch, ms, a.batch * 1e3 / ms))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["convs", "step"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    {"convs": convs, "step": step}[a.what](a)
