"""mx.kvstore: the gradient exchange, re-designed as RCCL all-reduce over xGMI.

MXNet's kvstore ('local' / 'device', train.py:35) reduced gradients across the GPUs of one
process and broadcast the updated weights (core/solver.py:121 -> Module.update). Here each GPU
is its own process (torchrun); the KVStore wraps torch.distributed (backend 'nccl' = RCCL on
ROCm, 'gloo' on CPU) and the Module all-reduces bucketed fp32 gradients during backward, then
runs the identical SGD step on every rank -- mathematically push(sum)+update+pull.
"""
import os

from .base import MXNetError


class KVStore:
    def __init__(self, kv_type="local"):
        self.type = kv_type
        self._dist = None

    @property
    def _world(self):
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                return dist.get_world_size(), dist.get_rank()
        except ImportError:
            pass
        return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))

    @property
    def rank(self):
        return self._world[1]

    @property
    def num_workers(self):
        # MXNet: local/device stores are one worker; dist_* stores count machines/processes.
        return self._world[0] if self.type.startswith("dist") else 1

    @property
    def world_size(self):
        return self._world[0]

    def barrier(self):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.barrier()

    def set_optimizer(self, optimizer):
        self._optimizer = optimizer

    def init(self, key, value):
        pass

    def push(self, key, value, priority=0):
        raise MXNetError("explicit push/pull is not used on the MI355X path; Module.update all-reduces gradients")

    pull = push


def create(name="local"):
    if not isinstance(name, str):
        raise MXNetError("name must be a string")
    if name not in ("local", "device", "local_allreduce_cpu", "local_allreduce_device", "nccl", "dist_sync",
                    "dist_device_sync", "dist_sync_device", "dist_async"):
        raise MXNetError("unknown kvstore type %s" % name)
    return KVStore(name)
