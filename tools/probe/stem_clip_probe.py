"""Time rn_stem_quant_clip_grad at the ResNet-50 stem size (256 x 3 x 224 x 224, 7x7/2 -> 64) for
thresholds clipping 0, ~0.1 %, ~1 % and ~5 % of the inputs (U(-1,1) data, identity BN)."""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "resnet.mxnet_amd")
from rn import lib as L  # noqa: E402
from gpu_util import BF16, conv_desc, p  # noqa: E402

n, c, h, w, k, r, st, pd = 256, 3, 224, 224, 64, 7, 2, 3
d = conv_desc(BF16, n, 8, h, w, k, r, r, st, pd, c_real=c)
dev = torch.device("cuda:0")
x = torch.rand(n, c, h, w, device=dev) * 2 - 1
dy = torch.randn(n, d.p, d.q, d.k_pad, device=dev).to(torch.bfloat16)
wq = torch.randn(k * r * r * c, device=dev) * 0.05
dbeta = torch.zeros(c, device=dev)
s = torch.cuda.current_stream()
for frac in (0.0, 0.001, 0.01, 0.05):
    t = torch.tensor([1e30 if frac == 0 else 1.0 - frac], device=dev)
    for _ in range(2):
        L.call("rn_stem_quant_clip_grad", C.byref(d), p(x), None, None, p(t), p(dy), p(wq), p(dbeta), s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        L.call("rn_stem_quant_clip_grad", C.byref(d), p(x), None, None, p(t), p(dy), p(wq), p(dbeta), s.cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    clipped = int((x.abs() >= t).sum().item())
    print("clip fraction %.4f (%d elements): %.3f ms" % (frac, clipped, e0.elapsed_time(e1) / 10), flush=True)
