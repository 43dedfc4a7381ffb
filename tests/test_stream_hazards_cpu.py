"""Cross-stream hazards of the two-stream backward (CPU dry run of the bound call plan, no GPU).

With the weight-gradient stream on (rn/executor.py `_route_wgrads`), every weight-gradient call
runs on a side stream after a fork from the compute stream, and the compute stream only joins the
side stream at the end of the backward. A fork orders the side call after everything the compute
stream enqueued BEFORE it, nothing after it. So for every side call S forked at plan index i:
  * no compute-stream call j > i may WRITE memory S reads or writes (S may run after j), and
  * no compute-stream call j > i may READ memory S writes (j may run before S).
Reads and writes come from `include/rn.h` itself: `const T*` parameters are read, non-const pointer
parameters written. Pointers are resolved to the executor's allocations (one tensor per graph
activation / gradient, the flat parameter / gradient / momentum / aux buffers split per parameter,
scratch workspaces), so two calls conflict when they touch the same allocation (or the same
parameter's slice of a flat buffer) in overlapping byte ranges -- the whole allocation, except for the
entry points that work on a known row / image range of it (_extent).

The reference's engine (MXNet) gets this ordering from its dependency engine; here it is a static
property of the plan, checked for every graph family and both precisions."""
import bisect
import ctypes as C
import os
import re

import numpy as np
import pytest
import torch

from rn import graphs
from rn.executor import Executor, Plan

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _signatures():
    """{entry point: [(param name, 'r' | 'w' | None)]} parsed from include/rn.h."""
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(REPO, "include", "rn.h")).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|int32_t|int64_t|void|size_t)\s+(rn_\w+)\s*\(([^)]*)\)\s*;", src):
        body = m.group(2).strip()
        params = [] if body in ("", "void") else [p.strip() for p in body.split(",")]
        kinds = []
        for p in params:
            if "*" not in p or "desc" in p:
                kinds.append((p, None))
            else:
                kinds.append((p, "r" if p.startswith("const ") else "w"))
        out[m.group(1)] = kinds
    return out


class _Regions:
    """Map a device pointer to a region label: the allocation holding it (flat buffers per param)."""

    def __init__(self, ex):
        spans = []
        seen = set()

        def add(t, label):
            if not isinstance(t, torch.Tensor) or t.numel() == 0 or t.data_ptr() in seen:
                return
            seen.add(t.data_ptr())
            spans.append((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size(), label))

        flats = {"master": ex.master, "grad": ex.grad, "mom": ex.mom}
        for fname, flat in flats.items():
            seen.add(flat.data_ptr())
            for n in ex.param_order:
                o = flat.data_ptr() + 4 * ex.param_off[n]
                spans.append((o, o + 4 * int(np.prod(ex.param_shape[n])), "%s:%s" % (fname, n)))
        seen.add(ex.aux.data_ptr())
        for n, (o, shp) in ex.aux_off.items():
            a = ex.aux.data_ptr() + 4 * o
            spans.append((a, a + 4 * int(np.prod(shp)), "aux:%s" % n))
        for k, v in vars(ex).items():
            vals = v.values() if isinstance(v, dict) else v if isinstance(v, (list, tuple)) else [v]
            for j, t in enumerate(vals):
                add(t, "%s[%d]" % (k, j))
        spans.sort()
        self.spans = spans
        self.starts = [s for s, _, _ in spans]

    def label(self, p):
        j = bisect.bisect_right(self.starts, p) - 1
        if j >= 0 and p < self.spans[j][1]:
            return self.spans[j][2]
        return "ptr:%x" % p  # an allocation outside the executor (exact-pointer identity)


def _extent(name, pname, v, args):
    """Byte range [lo, hi) a pointer argument touches: the whole allocation, except where an entry
    point works on a known sub-range (the stem's image chunks: rn_bn_bwd_apply_rows rows,
    rn_stem_conv_wgrad_p4 over its descriptor's n images)."""
    whole = (float("-inf"), float("inf"))
    if name == "rn_bn_bwd_apply_rows" and pname.split()[-1].lstrip("*") in ("x", "dy", "dx", "add_src"):
        d = args[0]._obj
        row = d.c * (2 if d.dtype == 0 else 4)
        return v + args[8] * row, v + (args[8] + args[9]) * row
    if name == "rn_stem_conv_wgrad_p4":
        d = args[0]._obj
        arg = pname.split()[-1].lstrip("*")
        if arg == "x4":
            return v, v + d.n * args[4] * args[5] * 4 * 2
        if arg == "dy":
            return v, v + d.n * d.p * d.q * d.k_pad * 2
    return whole


def _accesses(ex, sigs, regions, name, args):
    kinds = sigs[name]
    assert len(kinds) == len(args), (name, len(kinds), len(args))
    rd, wr = set(), set()
    for (pname, kind), a in zip(kinds, args):
        if kind is None or a is None:
            continue
        v = a.value if isinstance(a, C.c_void_p) else None
        if not v:
            continue
        (rd if kind == "r" else wr).add((regions.label(v),) + _extent(name, pname, v, args))
    return rd, wr


def _conflicts(a, b):
    """Labels of the accesses in a and b that touch the same allocation in overlapping byte ranges."""
    return {x[0] for x in a for y in b if x[0] == y[0] and x[1] < y[2] and y[1] < x[2]}


CASES = {
    "resnet20": (lambda: graphs.resnet20_cifar(), (8, 3, 32, 32)),
    "resnet50": (lambda: graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16), (2, 3, 64, 64)),
    "resnext50": (lambda: graphs.resnext([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16, "float32", 32),
                  (2, 3, 64, 64)),
    "resnet_int8": (lambda: graphs.resnet_int8([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16), (2, 3, 64, 64)),
}


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("graph", sorted(CASES))
def test_no_cross_stream_hazard(graph, dtype):
    symf, shp = CASES[graph]
    ex = Executor(Plan(symf(), [("data", shp)], [("softmax_label", (shp[0],))], dtype=dtype), "cpu")
    bad = _hazards(ex)
    assert not bad, bad[:10]


def _hazards(ex):
    sigs = _signatures()
    regions = _Regions(ex)
    calls = ex._bwd
    # the side-stream calls: _route_wgrads' rule (a weight-gradient call bound to the compute stream)
    side = [i for i, (n, f, a) in enumerate(calls) if n in Executor.WGRAD_CALLS]
    assert side, "no weight-gradient calls in the plan"
    acc = [_accesses(ex, sigs, regions, n, a) if n in sigs else (set(), set()) for n, f, a in calls]
    bad = []
    for i in side:
        s_rd, s_wr = acc[i]
        for j in range(i + 1, len(calls)):
            if j in side:
                continue  # same stream, plan order
            c_rd, c_wr = acc[j]
            war = _conflicts(c_wr, s_rd | s_wr)
            raw = _conflicts(c_rd, s_wr)
            if war or raw:
                bad.append((calls[i][0], i, calls[j][0], j, sorted(war | raw)[:3]))
    return bad


def test_hazard_check_sees_row_overlap():
    """The range-aware check still flags a compute-stream write into rows a side-stream call reads:
    the stem's second dx chunk moved onto the first chunk's rows (read by that chunk's wgrad)."""
    symf, shp = CASES["resnet20"]
    ex = Executor(Plan(symf(), [("data", shp)], [("softmax_label", (shp[0],))], dtype="bfloat16"), "cpu")
    assert not _hazards(ex)
    idx = [i for i, c in enumerate(ex._bwd) if c[0] == "rn_bn_bwd_apply_rows"]
    assert len(idx) == 4
    name, fn, args = ex._bwd[idx[1]]
    ex._bwd[idx[1]] = (name, fn, args[:8] + (0,) + args[9:])
    bad = _hazards(ex)
    assert bad and all(b[0] == "rn_stem_conv_wgrad_p4" and b[2] == "rn_bn_bwd_apply_rows" for b in bad)


def test_signature_parse_covers_plan():
    """Every call bound in a plan is declared in include/rn.h with a matching argument count (the
    hazard check above reads its access modes from there)."""
    sigs = _signatures()
    ex = Executor(Plan(CASES["resnet50"][0](), [("data", (2, 3, 64, 64))], [("softmax_label", (2,))],
                       dtype="bfloat16"), "cpu")
    for name, f, args in ex._fwd_train + ex._bwd:
        assert name in sigs, name
        assert len(sigs[name]) == len(args), (name, len(sigs[name]), len(args))
