"""The kvstore replacement over RCCL itself (torch.distributed backend 'nccl' = RCCL on ROCm).

The box has one GPU and RCCL refuses two ranks on one device, so the world-2 data-parallel tests
(test_dist_gpu.py) use gloo as the transport. This test runs the SAME bucketed all-reduce path on
RCCL with a world of one: the process group is initialised with backend 'nccl', the executor's
backward plan launches every bucket's all_reduce from its hook (rn/dist.py, core/solver.py:116-121
kvstore push), Module.update waits for them and runs the fused SGD. A world-1 sum is the identity, so
the gradients and the updated weights must equal those of the same step without a process group
(up to the run-to-run rounding of the fp32-atomic weight-gradient kernels: first-step gradients
Frobenius-relative 1e-4, a torn or early-read bucket is O(1)): an ordering hazard between the RCCL
stream and the compute / weight-gradient streams (a bucket reduced before its last writer, SGD
reading a bucket RCCL is still writing) shows up as a difference. It also proves RCCL initialises and runs next to librn's streams.

Every later step is checked against the SAME module recomputing that step's gradient without hooks
(same weights): comparing step 2 across two modules is not a hazard check, because this tiny-batch
ResNet-50 (8 images, 2x2 stage-4 maps: 32 values per BN channel) is chaotic under step 1's
run-to-run rounding -- ReLU decisions flip after the lr-0.1 update and step-2 gradients of two
plain runs without any process group differ O(1) (seen at 0.62 Frobenius-relative).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _step(sym, data, label, reducer_bucket_bytes=None, steps=2):
    import mxnet as mx
    from rn.dist import BucketAllReducer
    mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision="bfloat16")
    mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", label.shape)], for_training=True)
    mx.random.seed(3)
    mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
    mod.init_optimizer(kvstore="device", optimizer="sgd",
                       optimizer_params={"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9})
    ex = mod.executor
    launched = []
    if reducer_bucket_bytes is not None:
        ex.bucket_bytes = reducer_bucket_bytes
        red = BucketAllReducer(ex.grad, ex.buckets())
        orig = red.launch

        def launch(i):
            launched.append(i)
            orig(i)

        red.launch = launch
        mod._reducer = red
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    grads, plain, first_args = [], [], None
    for step in range(steps):
        mod.forward(batch, is_train=True)
        mod.backward()
        if mod._reducer is not None:
            mod._reducer.wait()
        grads.append(ex.grad.float().cpu().numpy().copy())
        if mod._reducer is not None:
            # the same step's gradient again, same weights, no hooks / collective (a world-1 sum is the
            # identity, so the buffer update() then consumes is the same gradient)
            ex.forward(is_train=True)
            ex.backward()
            plain.append(ex.grad.float().cpu().numpy().copy())
            # the update must consume the ALL-REDUCED buffer (the rerun overwrote ex.grad): put it back,
            # so the post-update weights checked below come from the hooked path
            ex.grad.copy_(torch.from_numpy(grads[-1]).to(ex.grad.device, ex.grad.dtype))
        mod.update()
        if step == 0:
            first_args = {k: v.asnumpy().copy() for k, v in mod.get_params()[0].items()}
    nb = len(ex.buckets()) if reducer_bucket_bytes else 0
    return grads, plain, first_args, launched, nb


def test_bucketed_allreduce_over_rccl_world1(gpu):
    import torch.distributed as dist
    from oracle import net as onet
    from rn import graphs
    sym = graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16)
    data, label = onet.synthetic_batch(8, (3, 64, 64), 16)
    data = data.astype(np.float32)
    ref_grads, _, ref_args, _, _ = _step(sym, data, label, steps=1)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=gpu)
    try:
        assert dist.get_backend() == "nccl"
        grads, plain, args, launched, nb = _step(sym, data, label, reducer_bucket_bytes=1 << 20, steps=2)
    finally:
        dist.destroy_process_group()
    assert nb >= 8  # 1 MB buckets over ResNet-50's 102 MB of fp32 gradients
    assert sorted(launched) == sorted(list(range(nb)) * 2)  # every bucket, once per backward
    fro = lambda a, b: float(np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-30))
    # step 1 against the module without a process group; every step against its own hook-free rerun
    assert fro(grads[0], ref_grads[0]) < 1e-4, fro(grads[0], ref_grads[0])
    for g, p in zip(grads, plain):
        assert fro(g, p) < 1e-4, fro(g, p)
    for k in ref_args:  # weights after the first SGD step (update() waited for every bucket)
        assert fro(args[k], ref_args[k]) < 1e-3, k


def _overlap_probe(main, side, cycles=200_000_000):
    """A long spin on the compute stream, then a short op on the side stream enqueued while it runs: with
    the two streams on different hardware queues the side op completes long before the spin ends; on one
    queue (HIP runs a queue's packets in order) it completes after it. Returns (spin ms, side-done ms)."""
    ev = lambda: torch.cuda.Event(enable_timing=True)
    e0, e1, s1 = ev(), ev(), ev()
    buf = torch.zeros(1024, device=main.device)
    torch.cuda.synchronize()
    e0.record(main)
    with torch.cuda.stream(main):
        torch.cuda._sleep(cycles)
    e1.record(main)
    with torch.cuda.stream(side):
        buf.add_(1.0)
    s1.record(side)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), e0.elapsed_time(s1)


def test_weight_gradient_stream_overlaps_with_rccl_hooks(gpu):
    """with an RCCL process group and the bucketed all-reduce hooks on (the product's
    data-parallel path, as bench.py RN_BENCH_ALLREDUCE=1 runs it at world 1) and the product's hardware-
    queue count (rn/__init__.py), the executor's weight-gradient stream must not share the compute
    stream's hardware queue. With HIP's 4 queues RCCL's pool streams moved it onto that queue and the
    backward's two branches ran serialised (25.8 vs 20.4 ms per step, profiles/r05/streams): a side-stream
    op enqueued behind a long compute-stream kernel then finishes only after it."""
    import torch.distributed as dist
    import mxnet as mx
    from oracle import net as onet
    from rn import dist as rdist, graphs
    from rn.dist import BucketAllReducer
    assert os.environ.get("GPU_MAX_HW_QUEUES") == "8"  # rn's import set it before this process's first HIP call
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=gpu, **rdist.nccl_pg_kwargs())
    try:
        sym = graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16)
        data, label = onet.synthetic_batch(8, (3, 64, 64), 16)
        mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision="bfloat16")
        mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", label.shape)], for_training=True)
        mx.random.seed(3)
        mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
        mod.init_optimizer(kvstore="device", optimizer="sgd", optimizer_params={"learning_rate": 0.1})
        ex = mod.executor
        ex.bucket_bytes = 1 << 20
        mod._reducer = BucketAllReducer(ex.grad, ex.buckets())
        batch = mx.io.DataBatch(data=[mx.nd.array(data.astype(np.float32))], label=[mx.nd.array(label)])
        for _ in range(2):  # RCCL has taken its streams and run its collectives beside both executor streams
            mod.forward(batch, is_train=True)
            mod.backward()
            mod.update()
        torch.cuda.synchronize()
        assert ex._side_stream is not None and ex.side_enabled
        spin, side_done = _overlap_probe(torch.cuda.current_stream(), ex._side_stream)
    finally:
        dist.destroy_process_group()
    assert spin > 5.0, spin  # the probe's compute-stream kernel really ran long
    assert side_done < 0.5 * spin, (side_done, spin)  # ... and the side stream did not wait behind it
