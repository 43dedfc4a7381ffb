"""HBM streaming reference points on one MI355X: torch copy (read + write) and the BatchNorm backward
apply (rn_bn_bwd's apply pass at the stage-1 shape: read x, dy, write dx) -- achieved GB/s."""
import ctypes as C
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "resnet.mxnet_amd")
from rn import lib as L  # noqa: E402
from gpu_util import BF16, p  # noqa: E402

dev = torch.device("cuda:0")


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


a = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
b = torch.empty_like(a)
t = timeit(lambda: b.copy_(a))
print("torch copy 512 MiB: %.1f GB/s (read + write)" % (2 * a.numel() / t / 1e9), flush=True)
for m, c in ((802816, 256), (200704, 512), (50176, 1024)):
    x = torch.randn(m, c, device=dev).to(torch.bfloat16)
    dy = torch.randn(m, c, device=dev).to(torch.bfloat16)
    dx = torch.empty_like(x)
    d = L.BNDesc(dtype=BF16, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    f = lambda v: torch.full((c,), v, dtype=torch.float32, device=dev)
    g, sm, si, sc, sh, dg, db = f(1.0), f(0.0), f(1.0), f(0.5), f(0.1), f(0.0), f(0.0)
    ws = torch.zeros(L.load().rn_bn_workspace_bytes(C.byref(d)) // 4 + 16, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    t = timeit(lambda: L.call("rn_bn_bwd", C.byref(d), p(x), p(dy), p(dx), None, p(g), p(sm), p(si), p(sc), p(sh),
                              p(dg), p(db), p(ws), s))
    nb = m * c * 2
    print("rn_bn_bwd m=%d c=%d: %.1f us, %.1f GB/s (reduce: read x, dy; apply: read x, dy, write dx = 5 tensor passes)"
          % (m, c, t * 1e6, 5 * nb / t / 1e9), flush=True)
