"""Debug the 256-row igemm tile on 3x3 convs: which configurations fail."""
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
for (n, h, w, c, k, r, pad), mode in [((1, 16, 16, 64, 256, 3, 0), 2), ((1, 16, 16, 64, 256, 3, 1), 2),
                                      ((1, 16, 16, 128, 256, 3, 1), 2), ((1, 16, 16, 64, 256, 1, 0), 2),
                                      ((1, 16, 16, 64, 256, 3, 1), 3), ((2, 14, 14, 128, 256, 3, 1), 2),
                                      ((1, 16, 16, 64, 256, 3, 1), 0), ((1, 16, 16, 64, 256, 2, 0), 2)]:
    d = conv_desc(BF16, n, c, h, w, k, r, r, 1, pad)
    x = torch.randn(n, h, w, c, device=dev).to(torch.bfloat16)
    wm = torch.randn(k, r, r, c, device=dev) * 0.1
    wk = torch.zeros(k * r * r * c, dtype=torch.bfloat16, device=dev)
    L.call("rn_conv_weight_pack", C.byref(d), p(wm), p(wk), None, stream())
    y = torch.zeros(n, d.p, d.q, k, dtype=torch.bfloat16, device=dev)
    L.call("rn_set_tuning", 4, mode)
    L.call("rn_set_tuning", 1, 1 if mode == 0 else 0)
    L.call("rn_conv_fwd", C.byref(d), p(x), p(wk), p(y), BF16, None, None, stream())
    torch.cuda.synchronize()
    L.call("rn_set_tuning", 4, 0)
    L.call("rn_set_tuning", 1, 0)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wk.view(k, r, r, c).float().permute(0, 3, 1, 2), padding=pad)
    ref = ref.permute(0, 2, 3, 1)
    err = (y.float() - ref).abs()
    print("case", (n, h, w, c, k, r, pad), "mode", mode, "max err %.4f" % err.max().item(),
          "ref max %.3f" % ref.abs().max().item())
    e = err.reshape(-1, k).cpu().numpy()
    badrows = np.nonzero(e.max(axis=1) > 0.05)[0]
    badcols = np.nonzero(e.max(axis=0) > 0.05)[0]
    if len(badrows):
        print("  bad rows", len(badrows), badrows[:20].tolist(), " bad cols", len(badcols), badcols[:20].tolist())
