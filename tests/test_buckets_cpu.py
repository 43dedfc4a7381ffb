"""Gradient buckets vs the backward plan (CPU dry run, no GPU): every bucket's all-reduce must be
launched after the LAST backward call that writes any parameter gradient inside it.

MXNet's kvstore pushes a parameter once its gradient is final (core/solver.py:116-121); our
rn/dist.py launches bucket b right after backward call `buckets()[b][2] - 1`. Here every bound call
of the backward plan is scanned for device pointers into the flat fp32 gradient buffer (the
buffer is only written during backward: zeroed, then produced by wgrad / BN-backward / bias /
stem-shift calls), each such pointer is mapped to its parameter, and the bucket's launch index
must exceed every such call's index -- including writers that are not the one `param_done_at`
recorded (e.g. a second call accumulating into the same gradient)."""
import bisect
import ctypes as C

import numpy as np
import pytest

from rn import graphs
from rn.executor import Executor, Plan


def _grad_writers(ex):
    """{param name: [indices of backward calls carrying a pointer into its gradient]}."""
    base = ex.grad.data_ptr()
    end = base + 4 * ex.nparam
    spans = sorted((ex.param_off[n], ex.param_off[n] + int(np.prod(ex.param_shape[n])), n) for n in ex.param_order)
    starts = [s for s, _, _ in spans]
    out = {}
    for i, (name, fn, args) in enumerate(ex._bwd):
        for a in args:
            if isinstance(a, C.c_void_p) and a.value and base <= a.value < end:
                off = (a.value - base) // 4
                j = bisect.bisect_right(starts, off) - 1
                assert j >= 0 and off < spans[j][1], (name, off)
                out.setdefault(spans[j][2], []).append(i)
    return out


CASES = {
    "resnet20": (lambda: graphs.resnet20_cifar(), (8, 3, 32, 32)),
    "resnet50": (lambda: graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16), (2, 3, 64, 64)),
    "resnext50": (lambda: graphs.resnext([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16, "float32", 32),
                  (2, 3, 64, 64)),
    "resnet_int8": (lambda: graphs.resnet_int8([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16), (2, 3, 64, 64)),
}


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
@pytest.mark.parametrize("graph", sorted(CASES))
@pytest.mark.parametrize("bucket_mb", [25.0, 1.0, 0.05])
def test_bucket_launch_after_last_writer(graph, dtype, bucket_mb):
    symf, shp = CASES[graph]
    ex = Executor(Plan(symf(), [("data", shp)], [("softmax_label", (shp[0],))], dtype=dtype), "cpu")
    ex.bucket_bytes = int(bucket_mb * (1 << 20))
    writers = _grad_writers(ex)
    # every parameter has a writer -- except fix_gamma gammas (bn_data: gradient identically zero,
    # left by the zeroing at the start of backward) -- and param_done_at is at or after the last one
    unwritten = set(ex.plan.param_names) - set(writers)
    fixed = {op.bn["gamma"] for op in ex.plan.ops if op.kind == "stem" and op.bn} | \
        {op.gamma for op in ex.plan.ops if op.kind == "bn" and op.fix_gamma}
    assert unwritten <= fixed, unwritten
    for n in unwritten:
        writers[n] = [-1]
    for n, idx in writers.items():
        assert ex.param_done_at[n] >= max(idx) + 1, (n, ex.param_done_at[n], idx)
    buckets = ex.buckets()
    if bucket_mb < 1:
        assert len(buckets) >= 4
    for s, e, launch in buckets:
        for n in ex.param_order:
            if s <= ex.param_off[n] < e:
                assert max(writers[n]) < launch, (n, max(writers[n]), launch)
        assert 0 < launch <= len(ex._bwd)
    # launches are in plan order and cover the flat buffer exactly
    assert buckets[0][0] == 0 and buckets[-1][1] == ex.nparam
    assert all(buckets[i][1] == buckets[i + 1][0] for i in range(len(buckets) - 1))
    assert all(buckets[i][2] <= buckets[i + 1][2] for i in range(len(buckets) - 1))


def test_slab_workspace_only_on_weight_gradient_calls():
    """Every call that uses the shared split-M slab workspace is a weight-gradient call (the calls
    routed to the side stream), so the slab is only ever touched by one stream."""
    symf, shp = CASES["resnet50"]
    ex = Executor(Plan(symf(), [("data", shp)], [("softmax_label", (shp[0],))], dtype="bfloat16"), "cpu")
    assert ex.wgrad_ws is not None
    ws = ex.wgrad_ws.data_ptr()
    users = [name for name, fn, args in ex._bwd + ex._fwd_train
             if any(isinstance(a, C.c_void_p) and a.value == ws for a in args)]
    assert users and all(u in Executor.WGRAD_CALLS for u in users), users


def test_trailing_bucket_is_small_and_last():
    """the parameters whose gradients the backward completes last (the stem and the
    first stage, at the flat buffer's end) form a trailing bucket of their own within
    RN_TAIL_BUCKET_MB (5 MB), so only it can be exposed after the stem's weight gradient; the other
    buckets keep ~25 MB and every bucket still launches after its last writer (test above)."""
    ex = Executor(Plan(graphs.resnet50(), [("data", (2, 3, 64, 64))], [("softmax_label", (2,))],
                       dtype="bfloat16"), "cpu")
    ex.bucket_bytes = 25 << 20
    b = ex.buckets()
    s, e, launch = b[-1]
    assert (e - s) * 4 <= 5 << 20
    names = [n for n in ex.param_order if s <= ex.param_off[n] < e]
    assert any(n.startswith("conv0") for n in names) and any(n.startswith("stage1_") for n in names)
    assert not any(n.startswith(("stage3_", "stage4_", "fc1")) for n in names)
    # the trailing bucket follows the stem's weight gradient: it launches with the backward's last calls
    assert launch >= ex.param_done_at["conv0_weight"]
    # the bucket before it is a head bucket: it ends where the trailing one starts, and it launches earlier
    assert b[-2][1] == s and b[-2][2] <= launch
    # head buckets: ~25 MB each (the last head bucket may be shorter)
    for hs, he, _ in b[:-2]:
        assert (he - hs) * 4 >= 25 << 20
    # a tail size of 0 restores the plain ~25 MB plan
    ex.tail_bucket_bytes = 0
    plain = ex.buckets()
    assert plain[-1][1] == ex.nparam and len(plain) == len(b) - 1
