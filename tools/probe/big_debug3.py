"""Debug the 256-row igemm tile: residual add and dgrad."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch
import torch.nn.functional as F
from rn import lib as L
from gpu_util import BF16, conv_desc, p, stream

dev = torch.device("cuda:0")
torch.manual_seed(0)
for (n, h, w, c, k, r, pad), mode, use_res in [((2, 14, 14, 128, 256, 3, 1), 2, False),
                                               ((2, 14, 14, 128, 256, 3, 1), 2, True),
                                               ((2, 14, 14, 128, 256, 3, 1), 0, True)]:
    d = conv_desc(BF16, n, c, h, w, k, r, r, 1, pad)
    x = torch.randn(n, h, w, c, device=dev).to(torch.bfloat16)
    wm = torch.randn(k, r, r, c, device=dev) * 0.1
    wk = torch.zeros(k * r * r * c, dtype=torch.bfloat16, device=dev)
    wc = torch.zeros(k * r * r * c, dtype=torch.bfloat16, device=dev)
    L.call("rn_conv_weight_pack", C.byref(d), p(wm), p(wk), p(wc), stream())
    y = torch.zeros(n, d.p, d.q, k, dtype=torch.bfloat16, device=dev)
    res = torch.randn(n, d.p, d.q, k, device=dev).to(torch.bfloat16)
    dy = torch.randn(n, d.p, d.q, k, device=dev).to(torch.bfloat16)
    dx = torch.zeros(n, h, w, c, dtype=torch.bfloat16, device=dev)
    L.call("rn_set_tuning", 4, mode)
    L.call("rn_conv_fwd", C.byref(d), p(x), p(wk), p(y), BF16, p(res) if use_res else None, None, stream())
    L.call("rn_conv_bwd_data", C.byref(d), p(dy), p(wc), p(dx), None, stream())
    torch.cuda.synchronize()
    L.call("rn_set_tuning", 4, 0)
    wf = wk.view(k, r, r, c).float().permute(0, 3, 1, 2)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wf, padding=pad).permute(0, 2, 3, 1)
    if use_res:
        ref = ref + res.float()
    err = (y.float() - ref).abs()
    dref = torch.nn.grad.conv2d_input((n, c, h, w), wf, dy.float().permute(0, 3, 1, 2), padding=pad).permute(0, 2, 3, 1)
    derr = (dx.float() - dref).abs()
    print("case", (n, h, w, c, k, r, pad), "mode", mode, "res", use_res, "fwd max err %.4f (ref %.2f)" % (
        err.max().item(), ref.abs().max().item()), "dgrad max err %.4f (ref %.2f)" % (derr.max().item(), dref.abs().max().item()))
    e = err.reshape(-1, k).cpu().numpy()
    badrows = np.nonzero(e.max(axis=1) > 0.05)[0]
    badcols = np.nonzero(e.max(axis=0) > 0.05)[0]
    if len(badrows):
        print("  bad rows", len(badrows), badrows[:20].tolist(), " bad cols", len(badcols), badcols[:20].tolist())
