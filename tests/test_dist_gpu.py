"""The N > 1 data-parallel step with the HIP kernels (world_size 2 on one GPU, gloo as the transport).

MXNet's dist_sync_device semantics (core/solver.py:116-121, train.py:35): every rank's bucketed
all-reduce (launched from the backward plan, on the weight-gradient stream when it is on) must equal
the sum of the two ranks' local gradients, on every one of several repeated backward passes; the SGD
update must equal MXNet's momentum SGD (oracle.ops.sgd_mom_update) applied to that sum with
rescale_grad = 1/(batch x workers), identically on both ranks. Graphs: ResNet-20 (C1 topology),
ResNet-50 v2 and ResNeXt-50 32x4d (C3 / C4 topologies, full [3,4,6,3] units at 64x64) with small
buckets (>= 4 per step). Slice mode: context=[gpu(0), gpu(0)] under a world of 2 splits
the global batch like MXNet's Module over two devices, rescale_grad = 1/global batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPEATS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sym(graph):
    from rn import graphs
    if graph == "resnet20":
        return graphs.resnet20_cifar(), (8, 3, 32, 32), 10
    units = [3, 4, 6, 3]
    if graph == "resnet50":
        return graphs.resnet(units, 4, [64, 256, 512, 1024, 2048], 16), (4, 3, 64, 64), 16
    return graphs.resnext(units, 4, [64, 256, 512, 1024, 2048], 16, "float32", 32), (4, 3, 64, 64), 16


def _worker(rank, world, port, graph, precision, mode, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import sys
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [repo, os.path.join(repo, "resnet.mxnet_amd")]
        import torch.distributed as dist
        from rn import dist as rdist
        import mxnet as mx
        torch.cuda.set_device(0)
        sym, shp, ncls = _sym(graph)
        opt = {"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9}
        if mode == "slice":  # one global batch, rank r computes slice r (MXNet's even split)
            gshp = (2 * shp[0],) + shp[1:]
            rng = np.random.default_rng(11)
            gdata = rng.uniform(-1, 1, gshp).astype(np.float32)
            glabel = rng.integers(0, ncls, gshp[0]).astype(np.float32)
            data, label = gdata[rank * shp[0]:(rank + 1) * shp[0]], glabel[rank * shp[0]:(rank + 1) * shp[0]]
        else:
            rng = np.random.default_rng(11 + rank)
            data = rng.uniform(-1, 1, shp).astype(np.float32)
            label = rng.integers(0, ncls, shp[0]).astype(np.float32)
        batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])

        def make(kv, seed, ctxs, dshape):
            m = mx.mod.Module(sym, context=ctxs, precision=precision)
            m.bind(data_shapes=[("data", dshape)], label_shapes=[("softmax_label", (dshape[0],))], for_training=True)
            mx.random.seed(seed)
            m.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
            m.init_optimizer(kvstore=kv, optimizer="sgd", optimizer_params=opt)
            return m

        # this rank's local gradient first, before the process group exists (no exchange), from the
        # weights rank 0 will broadcast (seed 3)
        ml = make("device", 3, [mx.gpu(0)], shp)
        g_runs = []
        for _ in range(2):  # twice: the local gradient itself must repeat (no race inside the step)
            ml.forward(batch, is_train=True)
            ml.backward()
            exl = ml.executor
            g_runs.append({n: exl.get_param(n, grad=True).copy() for n in exl.plan.param_names})
        g_local = g_runs[0]
        rep = max(float(np.abs(g_runs[1][n] - g_local[n]).max()) / max(1e-6, float(np.abs(g_local[n]).max()))
                  for n in g_local)
        assert rep <= (1e-5 if precision == "float32" else 2e-2), ("local gradient does not repeat", rep)
        del ml, exl
        rdist.init_from_env("gloo")
        if mode == "slice":
            md = make("dist_sync_device", 3 + rank, [mx.gpu(0), mx.gpu(0)], gshp)
            gbatch = mx.io.DataBatch(data=[mx.nd.array(gdata)], label=[mx.nd.array(glabel)])
            assert md._slice == (rank, 2)
        else:
            md = make("dist_sync_device", 3 + rank, [mx.gpu(0)], shp)  # broadcast from rank 0 fixes it
            gbatch = batch
        rescale = md._optimizer.rescale_grad
        arg, _ = md.get_params()
        exd = md.executor
        nb = len(exd.buckets())
        sums = []
        for _ in range(REPEATS):  # same weights, same batch: the summed gradient must repeat
            md.forward(gbatch, is_train=True)
            md.backward()
            md._reducer.wait()
            sums.append({n: exd.get_param(n, grad=True).copy() for n in exd.plan.param_names})
        md.update()  # the hooks launched the last backward's buckets: no second all-reduce here
        torch.cuda.synchronize()
        arg2, _ = md.get_params()
        q.put((rank, "ok", {k: v.asnumpy() for k, v in arg.items()}, g_local, sums,
               {k: v.asnumpy() for k, v in arg2.items()}, rescale, nb))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # report instead of hanging the parent
        import traceback
        q.put((rank, "error", traceback.format_exc(), None, None, None, None, None))


def _run(graph, precision, mode, bucket_mb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    saved = {k: os.environ.get(k) for k in ("RN_BUCKET_MB", "RN_HW_QUEUES", "GPU_MAX_HW_QUEUES")}
    os.environ["RN_BUCKET_MB"] = str(bucket_mb)  # inherited by the spawned ranks
    # two ranks on one GPU: HIP's 4 hardware queues each (8 per process oversubscribe the queue slots)
    os.environ["RN_HW_QUEUES"] = "4"
    os.environ["GPU_MAX_HW_QUEUES"] = "4"
    procs = [ctx.Process(target=_worker, args=(r, 2, port, graph, precision, mode, q)) for r in range(2)]
    try:
        for p in procs:
            p.start()
    finally:  # (the spawn copied them; this process keeps its own -- later tests read them)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    res = {}
    try:
        for _ in range(2):
            r = q.get(timeout=110)
            res[r[0]] = r
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in (0, 1):
        assert res[r][1] == "ok", res[r][2]
    return res


CASES = [("resnet20", "float32", "dp"), ("resnet20", "bfloat16", "dp"), ("resnet50", "float32", "dp"),
         ("resnet50", "bfloat16", "dp"), ("resnext50", "float32", "dp"), ("resnet20", "float32", "slice")]


@pytest.mark.parametrize("graph,precision,mode", CASES)
def test_dist_step_world2(graph, precision, mode):
    from oracle import ops
    assert torch.cuda.is_available()
    res = _run(graph, precision, mode, 0.25)
    _, _, a0, gl0, sums0, w0, rs0, nb = res[0]
    _, _, a1, gl1, sums1, w1, rs1, _ = res[1]
    sym, shp, _ = _sym(graph)
    assert nb >= (4 if graph != "resnet20" else 1), nb
    for k in a0:  # initial weights broadcast from rank 0
        assert np.array_equal(a0[k], a1[k]), k
    # MXNet rescale_grad: 1/(batch x workers); slice mode: the bound batch is the global one
    assert abs(rs0 - 1.0 / (2 * shp[0])) < 1e-12 and rs0 == rs1, (rs0, rs1)
    tol = 1e-5 if precision == "float32" else 2e-2
    bad = []
    for k, (gs0, gs1) in enumerate(zip(sums0, sums1)):
        for n in gl0:
            ref = gl0[n].astype(np.float64) + gl1[n].astype(np.float64)
            scale = max(1e-6, float(np.abs(ref).max()))
            for r, gs in ((0, gs0), (1, gs1)):
                err = float(np.abs(gs[n] - ref).max()) / scale
                if not err <= tol:
                    # least-squares fit gs ~ a gl0 + b gl1 (diagnostic: a = b = 1 expected)
                    A = np.stack([gl0[n].ravel(), gl1[n].ravel()], 1).astype(np.float64)
                    coef = np.linalg.lstsq(A, gs[n].ravel().astype(np.float64), rcond=None)[0]
                    bad.append((k, n, r, round(err, 4), np.round(coef, 4).tolist()))
    assert not bad, "\n".join(map(str, bad[:20]))
    for k in w0:  # identical update on both ranks ...
        assert np.array_equal(w0[k], w1[k]), k
    # ... equal to MXNet's SGD on the summed gradient of the last backward (one all-reduce, not two)
    g = sums0[-1]
    worst = (0.0, None)
    for k in w0:
        w = a0[k].astype(np.float64).copy()
        mom = np.zeros_like(w)
        ops.sgd_mom_update(w, g[k].astype(np.float64), mom, 0.1, 1e-4 * ops.wd_mult_for(k), 0.9, rs0)
        # fp32 master arithmetic: within 1e-3 of the step size (+ fp32 rounding of the weight itself);
        # a doubled all-reduce would be off by 100 % of the step
        bound = 1e-3 * float(np.abs(w - a0[k]).max()) + 2e-7 * float(np.abs(w).max()) + 1e-30
        worst = max(worst, (float(np.abs(w0[k] - w).max()) / bound, k))
    assert worst[0] < 1.0, worst
