"""Run the R20 two-step parity body several times in one process; print worst errors per run."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd"), os.path.join(REPO, "tests")]
import numpy as np

from oracle import net as onet
from rn import graphs
from step_util import max_rel, module_step, oracle_state, oracle_step

g = onet.resnet20_cifar()
args, aux = oracle_state(g)
data, label = onet.synthetic_batch(8, (3, 32, 32), 10)
ref = oracle_step(g, args, aux, data, label, steps=2)
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    res = module_step(graphs.resnet20_cifar(), args, aux, data, label, "float32", steps=2)
    ga = sorted(((max_rel(res["grads"][0][n], ref["grads"][0][n]), n) for n in ref["grads"][0]), reverse=True)[:2]
    gb = sorted(((max_rel(res["grads"][1][n], ref["grads"][1][n]), n) for n in ref["grads"][1]), reverse=True)[:2]
    wa = sorted(((max_rel(res["args"][n], ref["args"][n]), n) for n in ref["args"]), reverse=True)[:2]
    print(it, "g0", ga, "g1", gb, "w", wa, "p1 %.1e" % max_rel(res["prob"][1], ref["prob"][1]), flush=True)
