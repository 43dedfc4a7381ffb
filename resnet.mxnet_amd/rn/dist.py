"""Data-parallel gradient exchange: bucketed all-reduce over the flat fp32 gradient buffer.

Replaces MXNet kvstore push/pull (core/solver.py:121, train.py:35). One process per GPU;
backend 'nccl' is RCCL over xGMI on MI355X ('gloo' on CPU for tests). Buckets are contiguous
slices of the gradient buffer (parameters stored in reverse forward order), launched from the
backward plan right after the last kernel writing into them, so RCCL runs on its own stream
while the remaining backward kernels execute.
"""
import os


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*)."""
    import torch
    import torch.distributed as dist
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 or dist.is_initialized():
        return dist.is_initialized()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend, rank=int(os.environ["RANK"]), world_size=ws, **kw)
    return True


class BucketAllReducer:
    """Launch all-reduce(sum) of each bucket [start, end) of `flat` once backward reaches its index."""

    def __init__(self, flat, buckets, group=None):
        self.flat = flat
        self.buckets = list(buckets)  # [(start, end, launch_after_call_index)]
        self.group = group
        self.works = []
        self.launched_step = False  # set by Module.backward once the hooks launched every bucket

    def hooks(self):
        h = {}
        for i, (s, e, idx) in enumerate(self.buckets):
            h.setdefault(idx, []).append(i)

        def make(ids):
            return lambda: [self.launch(i) for i in ids]

        return {idx: make(ids) for idx, ids in h.items()}

    def launch(self, i):
        import torch.distributed as dist
        s, e, _ = self.buckets[i]
        self.works.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def launch_all(self):
        for i in range(len(self.buckets)):
            self.launch(i)

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []
