"""The N > 1 data-parallel step with the HIP kernels (world_size 2 on one GPU, gloo as the transport):
each rank's bucketed all-reduce (launched from the backward plan, on the weight-gradient stream) must
equal the sum of the two ranks' local gradients, and the SGD update must leave both ranks with
identical weights -- MXNet's dist_sync_device semantics (core/solver.py:116-121, train.py:35)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, precision, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import sys
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [repo, os.path.join(repo, "resnet.mxnet_amd")]
        import torch.distributed as dist
        from rn import dist as rdist
        from rn import graphs
        import mxnet as mx
        torch.cuda.set_device(0)
        sym = graphs.resnet20_cifar(10)
        shp = (8, 3, 32, 32)
        rng = np.random.default_rng(11 + rank)
        data = rng.uniform(-1, 1, shp).astype(np.float32)
        label = rng.integers(0, 10, shp[0]).astype(np.float32)
        batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
        opt = {"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9}

        def make(kv, seed):
            m = mx.mod.Module(sym, context=[mx.gpu(0)], precision=precision)
            m.bind(data_shapes=[("data", shp)], label_shapes=[("softmax_label", (shp[0],))], for_training=True)
            mx.random.seed(seed)
            m.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
            m.init_optimizer(kvstore=kv, optimizer="sgd", optimizer_params=opt)
            return m

        # this rank's local gradient first, before the process group exists (no exchange), from the
        # weights rank 0 will broadcast (seed 3)
        ml = make("device", 3)
        ml.forward(batch, is_train=True)
        ml.backward()
        exl = ml.executor
        g_local = {n: exl.get_param(n, grad=True).copy() for n in exl.plan.param_names}
        rdist.init_from_env("gloo")
        md = make("dist_sync_device", 3 + rank)  # different per rank: the broadcast from rank 0 fixes it
        arg, aux = md.get_params()
        md.forward(batch, is_train=True)
        md.backward()
        md._reducer.wait()
        exd = md.executor
        g_sum = {n: exd.get_param(n, grad=True).copy() for n in exd.plan.param_names}
        md.update()
        torch.cuda.synchronize()
        arg2, _ = md.get_params()
        q.put((rank, "ok", {k: v.asnumpy() for k, v in arg.items()}, g_local, g_sum,
               {k: v.asnumpy() for k, v in arg2.items()}))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, "error", traceback.format_exc(), None, None, None))


@pytest.mark.parametrize("precision", ["float32", "bfloat16"])
def test_dist_step_world2(precision):
    assert torch.cuda.is_available()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, precision, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r = q.get(timeout=100)
            res[r[0]] = r
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in (0, 1):
        assert res[r][1] == "ok", res[r][2]
    _, _, a0, gl0, gs0, w0 = res[0]
    _, _, a1, gl1, gs1, w1 = res[1]
    for k in a0:  # initial weights broadcast from rank 0
        assert np.array_equal(a0[k], a1[k]), k
    tol = 1e-5 if precision == "float32" else 2e-2
    bad = []
    for n in gl0:
        ref = gl0[n].astype(np.float64) + gl1[n].astype(np.float64)
        scale = max(1e-6, float(np.abs(ref).max()))
        for r, gs in ((0, gs0), (1, gs1)):
            err = float(np.abs(gs[n] - ref).max()) / scale
            if not err <= tol:
                # least-squares fit gs ~ a gl0 + b gl1 (diagnostic: a = b = 1 expected)
                A = np.stack([gl0[n].ravel(), gl1[n].ravel()], 1).astype(np.float64)
                coef = np.linalg.lstsq(A, gs[n].ravel().astype(np.float64), rcond=None)[0]
                bad.append((n, r, round(err, 4), np.round(coef, 4).tolist()))
    assert not bad, "\n".join(map(str, bad))
    for k in w0:  # identical update on both ranks
        assert np.array_equal(w0[k], w1[k]), k
