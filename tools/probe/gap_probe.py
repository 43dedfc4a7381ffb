"""Kernel-boundary gaps on one stream: what a dependent launch waits for after a given producer.

python tools/probe/gap_probe.py            (under rocprofv3 --kernel-trace; then --report <trace.csv>)
Each sequence is captured in its own hipGraph and replayed 5 times: a 1x1 conv forward on the 224-row
tile writing 411 MB (stage 1) or 51 MB (stage 4), the BatchNorm apply pass (411 MB, nontemporal stores by
default), and a trivial 256-element kernel between them. The report prints the mean gap between each
(previous, next) kernel pair on the queue: a gap that follows the producer's output size is its dirty L2
lines' write-back at the boundary; a gap that follows the consumer is its own launch cost.
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd")]


def report(path):
    import collections
    import csv
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    agg = collections.defaultdict(list)
    short = lambda n: n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]
    for a, b in zip(rows, rows[1:]):
        if a["Queue_Id"] != b["Queue_Id"]:
            continue
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        if g < 100:  # (not across replays)
            agg[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append(g)
    for (pa, pb), v in sorted(agg.items()):
        print("%7.2f us  n=%3d  %-48s -> %s" % (sum(v) / len(v), len(v), pa, pb))


def main():
    import torch
    from rn import lib as L
    lib = L.load()
    dev = torch.device("cuda:0")
    st = C.c_void_p(0)
    P = lambda t: C.c_void_p(t.data_ptr())

    def conv(n, h, c, k):
        d = L.ConvDesc(dtype=L.RN_BF16, n=n, h=h, w=h, c=c, c_real=c, k=k, k_pad=k, r=1, s=1, stride_h=1, stride_w=1,
                       pad_h=0, pad_w=0, groups=1)
        L.check(lib.rn_conv_desc_init(C.byref(d)), "desc")
        x = torch.randn(n * h * h * c, device=dev).to(torch.bfloat16)
        y = torch.empty(n * h * h * k, device=dev, dtype=torch.bfloat16)
        wm = torch.randn(k * c, device=dev) * 0.05
        wk = torch.empty(lib.rn_conv_pack_numel(C.byref(d), 0), device=dev, dtype=torch.bfloat16)
        L.check(lib.rn_conv_weight_pack(C.byref(d), P(wm), P(wk), None, st), "pack")
        return lambda s: L.check(lib.rn_conv_fwd(C.byref(d), P(x), P(wk), P(y), L.RN_BF16, None, None, s), "fwd")

    conv56 = conv(256, 56, 64, 256)   # 411 MB out
    conv7 = conv(256, 7, 512, 2048)   # 51 MB out
    m, c = 256 * 56 * 56, 256
    bd = L.BNDesc(dtype=L.RN_BF16, m=m, c=c, c_real=c, eps=1e-5, momentum=0.9, fix_gamma=0, relu=1)
    bx = torch.randn(m * c, device=dev).to(torch.bfloat16)
    by = torch.empty_like(bx)
    sc, sh = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1
    bnapply = lambda s: L.check(lib.rn_bn_apply(C.byref(bd), P(bx), P(by), P(sc), P(sh), s), "bn_apply")
    tiny_t = torch.zeros(256, device=dev)

    def tiny(s):
        tiny_t.add_(1.0)

    seqs = {"conv56": [conv56] * 6, "conv7": [conv7] * 6, "bnapply": [bnapply] * 6, "tiny": [tiny] * 6,
            "conv56_tiny": [conv56, tiny] * 4, "conv7_tiny": [conv7, tiny] * 4, "bnapply_tiny": [bnapply, tiny] * 4,
            "conv56_bnapply": [conv56, bnapply] * 3}
    graphs = {}
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for name, seq in seqs.items():
            for fn in seq:  # warm
                fn(C.c_void_p(s.cuda_stream))
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for fn in seq:
                    fn(C.c_void_p(s.cuda_stream))
            graphs[name] = g
    torch.cuda.synchronize()
    for name, g in graphs.items():
        for _ in range(5):
            g.replay()
            torch.cuda.synchronize()
        print("replayed", name, flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        main()
