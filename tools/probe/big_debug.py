"""Debug the 256-row igemm tile: 1x1 convs as plain GEMMs, error structure per row/column block."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd"), os.path.join(REPO, "tests")]
import numpy as np
import torch
from rn import lib as L
from gpu_util import BF16, conv_desc, p, stream

dev = torch.device("cuda:0")
torch.manual_seed(0)
for (n, h, w, c, k), mode in [((1, 16, 16, 64, 256), 2), ((1, 16, 16, 64, 256), 3), ((1, 16, 16, 128, 256), 2),
                              ((2, 16, 16, 64, 256), 2), ((1, 16, 16, 64, 256), 0)]:
    d = conv_desc(BF16, n, c, h, w, k, 1, 1, 1, 0)
    x = torch.randn(n * h * w, c, device=dev).to(torch.bfloat16)
    wm = torch.randn(k, c, device=dev) * 0.1
    wk = torch.zeros(k * c, dtype=torch.bfloat16, device=dev)
    L.call("rn_conv_weight_pack", C.byref(d), p(wm), p(wk), None, stream())
    y = torch.zeros(n * h * w, k, dtype=torch.bfloat16, device=dev)
    L.call("rn_set_tuning", 4, mode)
    L.call("rn_set_tuning", 1, 1 if mode == 0 else 0)
    L.call("rn_conv_fwd", C.byref(d), p(x), p(wk), p(y), BF16, None, None, stream())
    torch.cuda.synchronize()
    L.call("rn_set_tuning", 4, 0)
    L.call("rn_set_tuning", 1, 0)
    ref = x.float() @ wk.view(k, c).float().t()
    err = (y.float() - ref).abs()
    M = n * h * w
    print("case", (n, h, w, c, k), "mode", mode, "max err", err.max().item(), "ref max", ref.abs().max().item())
    e = err.cpu().numpy()
    rb = e.reshape(M // 16, 16, k // 16, 16).max(axis=(1, 3))
    print(" bad 16x16 blocks (row blk, col blk):", np.argwhere(rb > 0.05)[:12].tolist(), "count", int((rb > 0.05).sum()),
          "of", rb.size)
    bad = np.argwhere(e > 0.05)
    if len(bad):
        r0, c0 = bad[0]
        print(" first bad", (int(r0), int(c0)), "got", float(y[r0, c0]), "ref", float(ref[r0, c0]))
        # which column of the reference matches the bad output row?
        yr = y[r0].float()
        cand = ((ref - yr[None, :]).abs().max(dim=1).values < 0.05).nonzero().flatten().tolist()
        print(" row", int(r0), "matches reference rows", cand[:8])
        yc = y[:, c0].float()
        candc = ((ref - yc[:, None]).abs().max(dim=0).values < 0.05).nonzero().flatten().tolist()
        print(" col", int(c0), "matches reference cols", candc[:8])
