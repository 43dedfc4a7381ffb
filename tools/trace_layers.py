"""Map the conv dispatch durations (igemm*/wgrad* kernels) of the LAST training step in a rocprofv3
kernel trace onto the ResNet-50 layers (plan call order) and print per-layer TFLOP/s and the
fraction of each layer's own roofline max(FLOP/2.5 PF, algorithmic bytes/8 TB/s). CPU-only tool.
usage: python tools/trace_layers.py <run_kernel_trace.csv> [batch] [resnet50|resnext50|resnet50_int8]"""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd")]
from rn import graphs  # noqa: E402
from rn.executor import Executor, Plan  # noqa: E402
from bench import conv_call_bytes  # noqa: E402

CONV_CALLS = ("rn_conv_fwd", "rn_conv_fwd_bnstats", "rn_conv_fwd_x", "rn_conv_bwd_data",
              "rn_conv_bwd_data_bnred", "rn_conv_bwd_filter", "rn_conv_bwd_filter_x", "rn_conv_bwd_filter_ws",
              "rn_stem_conv_fwd_p4", "rn_stem_conv_wgrad_p4")


def kernel_short(name):
    """'void (anonymous namespace)::igemm_big_kernel<256, 2, 1, false, 224, 0>(IgemmArgs)' ->
    'igemm_big_kernel<256, 2, 1, false, 224, 0>'."""
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0].replace("unsigned short", "bf16")[:48]


def main():
    trace = sys.argv[1]
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    gname = sys.argv[3] if len(sys.argv) > 3 else "resnet50"
    sym = {"resnet50": graphs.resnet50, "resnext50": graphs.resnext50_32x4d, "resnet50_int8": graphs.resnet50_int8}[gname]()
    plan = Plan(sym, [("data", (batch, 3, 224, 224))], [("softmax_label", (batch,))])
    ex = Executor(plan, "cpu")
    names = {}
    for op in plan.ops:
        for attr in ("desc", "dfull", "d1"):
            if hasattr(op, attr):
                names[id(getattr(op, attr))] = op.name
    calls = [(n, a) for n, f, a in ex._fwd_train + ex._bwd if n in CONV_CALLS]
    # host submission order (Dispatch_Id) = the plan's call order on both streams; start times are
    # not, once the weight gradients run on the side stream beside the data-gradient chain
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Dispatch_Id"]))
    step_end = [i for i, r in enumerate(rows) if "sgd_mom" in r["Kernel_Name"]]
    rows = rows[step_end[-2] + 1:step_end[-1]]
    conv_rows = []
    for r in rows:  # a slab reduction pass belongs to the weight gradient launched just before it
        if "slab_reduce" in r["Kernel_Name"] and conv_rows:
            conv_rows[-1] = dict(conv_rows[-1], End_Timestamp=str(int(conv_rows[-1]["End_Timestamp"]) + int(
                r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        elif "igemm" in r["Kernel_Name"] or "wgrad" in r["Kernel_Name"]:
            conv_rows.append(r)
    rows = conv_rows
    assert len(rows) == len(calls), (len(rows), len(calls))
    tot, out = {}, []
    for (n, a), r in zip(calls, rows):
        d = a[0]._obj
        flops = 2.0 * d.n * d.p * d.q * d.k * (d.c_real // d.groups) * d.r * d.s
        kind = "wgrad" if ("filter" in n or "wgrad" in n) else "dgrad" if "bwd_data" in n else "fwd"
        # algorithmic bytes as bench.py counts them: every operand once, + residual / BN input reads
        algb = float(conv_call_bytes(ex, n, a)) if n.startswith("rn_conv") else \
            2.0 * (d.n * d.h * d.w * d.c + d.n * d.p * d.q * d.k_pad) + 8.0 * d.k * d.r * d.s * d.c
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        roof = max(flops / 2.5e15, algb / 8e12) * 1e6
        out.append((us, names.get(id(d), "?"), kind, flops / us / 1e6, algb / us / 1e6, roof / us,
                    flops / algb, kernel_short(r["Kernel_Name"])))
        tot[kind] = tot.get(kind, 0) + us
    print("    time  layer                  kind    TFLOP/s   TB/s  roof%  FLOP/B  kernel")
    for us, lname, kind, tf, tb, fr, ai, kn in sorted(out, reverse=True):
        print("%8.1f us  %-22s %-5s %7.1f TF %5.2f %4.0f%% %6.0f  %s" % (us, lname, kind, tf, tb, 100 * fr, ai, kn))
    print({k: round(v / 1e3, 3) for k, v in tot.items()}, "ms")
    # time above a practical bound: memory-side layers at 5.5 TB/s, MFMA-side at 60 % of peak
    excess = sum(max(0.0, o[0] - max(o[3] * o[0] / 2.5e3 / 0.6 * 0 + (o[0] * o[4] / 5.5), 0)) for o in out)
    print("time above max(bytes / 5.5 TB/s, FLOP / 1.5 PF): %.3f ms" % (sum(
        max(0.0, o[0] - max(o[0] * o[4] / 5.5, o[0] * o[3] / 1.5e3)) for o in out) / 1e3))


if __name__ == "__main__":
    main()
