"""GPU diagnostic: shim step vs oracle (fp64, fp32, bf16-storage) -- prints error summaries."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd"), os.path.join(REPO, "tests")]
import numpy as np

from oracle import net as onet
from rn import graphs
from step_util import module_step, oracle_step


def fro(a, b):
    return float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))


def mrel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def cos_all(ga, gb):
    ks = sorted(gb)
    a = np.concatenate([ga[k].ravel() for k in ks])
    b = np.concatenate([gb[k].ravel() for k in ks])
    return float(a @ b / (np.linalg.norm(a) * np.linalg.norm(b)))


def report(tag, res_prob, res_g, ref):
    g = ref["grads"][0]
    errs = sorted(((fro(res_g[k], g[k]), k) for k in g), reverse=True)
    print("  %-26s prob mrel %.2e | grad cos %.6f | worst fro %s" % (
        tag, mrel(res_prob, ref["prob"][0]), cos_all(res_g, g), ["%s %.2e" % (k, e) for e, k in errs[:3]]),
        flush=True)


cases = [
    ("r50_4x64", onet.resnet50_imagenet(16), lambda: graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16),
     4, 64, 16),
    ("r20_8x32", onet.resnet20_cifar(), graphs.resnet20_cifar, 8, 32, 10),
]
for name, g, symf, n, hw, ncls in cases:
    args, aux = onet.init_params(g)
    data, label = onet.synthetic_batch(n, (3, hw, hw), ncls)
    r64 = oracle_step(g, args, aux, data, label)
    r32 = oracle_step(g, args, aux, data, label, dtype=np.float32)
    rbf = oracle_step(g, args, aux, data, label, dtype=np.float32, storage="bf16")
    print(name, flush=True)
    report("oracle fp32 vs fp64", r32["prob"][0], r32["grads"][0], r64)
    report("oracle bf16st vs fp64", rbf["prob"][0], rbf["grads"][0], r64)
    for prec in ("float32", "bfloat16"):
        res = module_step(symf(), args, aux, data, label, prec)
        report("gpu %s vs fp64" % prec, res["prob"][0], res["grads"][0], r64)
        if prec == "bfloat16":
            report("gpu bf16 vs oracle bf16st", res["prob"][0], res["grads"][0], rbf)
