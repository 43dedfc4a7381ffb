"""Per-shape timing of the conv kernels (fwd / dgrad / wgrad) over the unique convolutions of a
graph (default ResNet-50 v2, batch 256, bf16) -- the inner loop for conv-kernel work.

python tools/conv_bench.py [--graph resnet50|resnext50|resnet50_int8] [--iters 20] [--only fwd,dgrad,wgrad]
Prints one line per unique shape (count = occurrences per step) and the per-step totals.
"""
import argparse
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="fwd,dgrad,wgrad", help="modes among fwd, dgrad, wgrad, dgbn (dgrad + BN reduction)")
    ap.add_argument("--filter", default="")
    ap.add_argument("--cold", action="store_true", help="evict L2/MALL (write 512 MB) before every timed call")
    a = ap.parse_args()
    import torch
    from rn import graphs
    from rn import lib as L
    from rn.executor import Plan, _pad8
    sym = {"resnet50": graphs.resnet50, "resnext50": graphs.resnext50_32x4d,
           "resnet50_int8": graphs.resnet50_int8}[a.graph]()
    plan = Plan(sym, [("data", (a.batch, 3, 224, 224))], [("softmax_label", (a.batch,))])
    lib = L.load()
    shapes = {}
    for op in plan.ops:
        if op.kind != "conv":
            continue
        x, y = op.x, op.y
        key = (x.n, x.h, x.w, x.cp, x.c, y.c, op.kernel, op.stride, op.pad, op.groups, op.res is not None)
        if key not in shapes:
            shapes[key] = [op.name, 0]
        shapes[key][1] += 1
    dev = torch.device("cuda:0")
    flush = torch.empty(128 << 20, dtype=torch.float32, device=dev) if a.cold else None
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    modes = a.only.split(",")
    tot = {m: 0.0 for m in modes}
    flops_tot = 0.0
    print("%-26s %3s %-22s %-5s" % ("layer", "n", "shape", "") + "".join("%23s" % m for m in modes))
    for key, (name, cnt) in shapes.items():
        if a.filter and a.filter not in name:
            continue
        n, h, w, cp, c, k, kern, stride, pad, g, res = key
        d = L.ConvDesc(dtype=L.RN_BF16, n=n, h=h, w=w, c=cp, c_real=c, k=k, k_pad=_pad8(k), r=kern[0], s=kern[1],
                       stride_h=stride[0], stride_w=stride[1], pad_h=pad[0], pad_w=pad[1], groups=g)
        L.check(lib.rn_conv_desc_init(C.byref(d)), "desc")
        x = torch.randn(n * h * w * cp, device=dev).to(torch.bfloat16)
        yv = torch.randn(n * d.p * d.q * d.k_pad, device=dev).to(torch.bfloat16)
        y = torch.empty_like(yv)
        dx = torch.empty_like(x)
        wm = torch.randn(k * kern[0] * kern[1] * (c // g), device=dev) * 0.05
        wk = torch.empty(lib.rn_conv_pack_numel(C.byref(d), 0), device=dev, dtype=torch.bfloat16)
        wc = torch.empty(lib.rn_conv_pack_numel(C.byref(d), 1), device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(wm.numel(), device=dev)
        P = lambda t: C.c_void_p(t.data_ptr())
        ws_bytes = int(lib.rn_conv_wgrad_ws_bytes(C.byref(d)))  # split-M slab workspace, as the executor uses
        ws = torch.empty(max(ws_bytes, 16) // 4, device=dev)
        bnv = torch.rand(cp, device=dev) * 0.5 + 0.5
        bnpart = torch.empty(int(lib.rn_conv_bnred_blocks(C.byref(d))) * cp * 2 + 16, device=dev)
        L.check(lib.rn_conv_weight_pack(C.byref(d), P(wm), P(wk), P(wc), st), "pack")
        calls = {
            "fwd": lambda: lib.rn_conv_fwd(C.byref(d), P(x), P(wk), P(y), L.RN_BF16, P(yv) if res else None, None, st),
            "dgrad": lambda: lib.rn_conv_bwd_data(C.byref(d), P(yv), P(wc), P(dx), None, st),
            "wgrad": lambda: lib.rn_conv_bwd_filter_ws(C.byref(d), P(x), P(yv), P(dw), P(ws), ws_bytes, st),
            # the data gradient with the BatchNorm-backward reduction of its output in the epilogue (EPI 2,
            # how the step runs it): bn_x = the dgrad output's shape
            "dgbn": lambda: lib.rn_conv_bwd_data_bnred(C.byref(d), P(yv), P(wc), P(dx), None, P(x), P(bnv), P(bnv),
                                                       P(bnv), 1, P(bnpart), st),
        }
        flops = 2.0 * n * d.p * d.q * k * (c // g) * kern[0] * kern[1]
        # algorithmic HBM bytes (bf16): x + w + y (+ residual for fwd); per-mode roofline time
        xb, yb, wb = 2.0 * n * h * w * c, 2.0 * n * d.p * d.q * k, 2.0 * k * kern[0] * kern[1] * (c // g)
        algb = {"fwd": xb + wb + yb * (2 if res else 1), "dgrad": yb + wb + xb, "wgrad": xb + yb + 2 * wb,
                "dgbn": yb + wb + 2 * xb}
        row = "%-26s %3d %-22s %-5s" % (name[:26], cnt, "%dx%dx%d>%d k%d s%d" % (h, w, c, k, kern[0], stride[0]),
                                       "g%d" % g if g > 1 else ("+res" if res else ""))
        for m in modes:
            fn = calls[m]
            for _ in range(3):
                L.check(fn(), m)
            if flush is None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.iters
            else:
                evs = []
                for _ in range(a.iters):
                    flush.fill_(1.0)
                    dw.zero_()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    evs.append((e0, e1))
                torch.cuda.synchronize()
                ms = sum(x.elapsed_time(y) for x, y in evs) / a.iters
            tot[m] += ms * cnt
            roof = max(flops / 2.5e15, algb[m] / 8e12) * 1e3
            row += "%8.1fus %6.0fT %3.0f%%" % (ms * 1e3, flops / ms / 1e9, 100 * roof / ms)
        flops_tot += flops * cnt
        print(row, flush=True)
    print("per-step totals: " + "  ".join("%s %.3f ms" % (m, tot[m]) for m in modes) +
          "  (conv flops fwd %.1f GF -> %s)" % (flops_tot / 1e9, "  ".join(
              "%s %.0f TF/s" % (m, flops_tot / tot[m] / 1e9) for m in modes if tot[m] > 0)))


if __name__ == "__main__":
    main()
