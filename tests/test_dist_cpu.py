"""Multi-process data-parallel exchange on CPU (gloo, world_size 2): bucketed all-reduce of the
flat gradient buffer launched from backward hooks, equal to the per-rank gradient sum."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "resnet.mxnet_amd")]
    from rn import dist as rdist
    import torch.distributed as dist
    rdist.init_from_env("gloo")
    n = 1000
    flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
    buckets = [(0, 300, 2), (300, 700, 5), (700, 1000, 9)]
    red = rdist.BucketAllReducer(flat, buckets)
    hooks = red.hooks()
    for i in range(1, 10):  # emulate the backward call sequence
        if i in hooks:
            hooks[i]()
    red.wait()
    expect = torch.arange(n, dtype=torch.float32) * sum(r + 1 for r in range(world))
    ok = bool(torch.equal(flat, expect))
    # MXNet kvstore semantics of the shim: rank / num_workers
    import mxnet as mx
    kv = mx.kvstore.create("dist_sync_device")
    kv2 = mx.kvstore.create("device")
    q.put((rank, ok, kv.rank, kv.num_workers, kv2.num_workers))
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_allreduce_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort()
    assert all(r[1] for r in res), res
    assert [r[2] for r in res] == [0, 1]
    assert all(r[3] == 2 and r[4] == 1 for r in res)
