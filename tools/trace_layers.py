"""Map igemm/wgrad dispatch durations of the last training step in a rocprofv3 kernel trace
onto the ResNet-50 layers (plan call order), and print per-layer TFLOP/s. CPU-only tool."""
import csv
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd")]
from rn import graphs  # noqa: E402
from rn.executor import Executor, Plan  # noqa: E402

trace = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
plan = Plan(graphs.resnet50(), [("data", (batch, 3, 224, 224))], [("softmax_label", (batch,))])
ex = Executor(plan, "cpu")
calls = [(n, a) for n, f, a in ex._fwd_train + ex._bwd if n in ("rn_conv_fwd", "rn_conv_bwd_data", "rn_conv_bwd_filter")]
names = {}
for op in plan.ops:
    if hasattr(op, "desc"):
        names[id(op.desc)] = op.name
    if hasattr(op, "d1"):
        names[id(op.d1)] = op.name
rows = [r for r in csv.DictReader(open(trace)) if "igemm_kernel" in r["Kernel_Name"] or "wgrad_kernel" in r["Kernel_Name"]]
rows = rows[-len(calls):]
tot = {}
out = []
for (n, a), r in zip(calls, rows):
    d = a[0]._obj
    flops = 2 * d.n * d.p * d.q * d.k * d.c_real * d.r * d.s
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    lname = names.get(id(d), "?")
    kind = {"rn_conv_fwd": "fwd", "rn_conv_bwd_data": "dgrad", "rn_conv_bwd_filter": "wgrad"}[n]
    out.append((us, lname, kind, flops / us / 1e6, d.n * d.p * d.q, d.k, d.c_real, d.r))
    tot[kind] = tot.get(kind, 0) + us
for us, lname, kind, tf, m, k, c, r in sorted(out, reverse=True)[:40]:
    print("%8.1f us  %-28s %-5s %7.1f TF  M=%d K=%d C=%d R=%d" % (us, lname, kind, tf, m, k, c, r))
print({k: round(v / 1e3, 3) for k, v in tot.items()}, "ms")
