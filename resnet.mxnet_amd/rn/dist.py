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
        kw.update(nccl_pg_kwargs())
    dist.init_process_group(backend=backend, rank=int(os.environ["RANK"]), world_size=ws, **kw)
    return True


def nccl_pg_kwargs():
    """RN_NCCL_HIPRIO=1: RCCL's streams from torch's high-priority pool (ProcessGroupNCCL.Options
    is_high_priority_stream), i.e. hardware queues apart from the normal-priority compute and weight-gradient
    streams (A/B knob)."""
    if os.environ.get("RN_NCCL_HIPRIO", "0") != "1":
        return {}
    import torch.distributed as dist
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return {"pg_options": opts}


class BucketAllReducer:
    """Launch all-reduce(sum) of each bucket [start, end) of `flat` once backward reaches its index."""

    def __init__(self, flat, buckets, group=None):
        self.flat = flat
        self.buckets = list(buckets)  # [(start, end, launch_after_call_index)]
        self.group = group
        self.works = []
        self.launched_step = False  # set by Module.backward once the hooks launched every bucket
        # overlap evidence (bench.py, N > 1): HIP events per step at the backward's start, at each
        # bucket's launch, at the end of the backward (the stream that waits for the buckets) and after
        # each bucket's wait; off by default
        self.timing = False
        self.records = []
        self._cur = None

    def begin_step(self):
        """Module.backward calls this before the backward's first kernel is enqueued."""
        if self.timing:
            self._cur = {"start": self._event(), "launch": {}, "done": []}

    @staticmethod
    def _event():
        import torch
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

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
        if self._cur is not None:
            self._cur["launch"][i] = self._event()
        self.works.append(dist.all_reduce(self.flat[s:e], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def launch_all(self):
        for i in range(len(self.buckets)):
            self.launch(i)

    def wait(self):
        cur = self._cur if self.works else None
        if cur is not None:
            cur["bwd_end"] = self._event()  # every backward kernel is enqueued before this point
        for w in self.works:
            w.wait()
            if cur is not None:
                cur["done"].append(self._event())  # = max(end of the backward, this bucket's completion)
        self.works = []
        if cur is not None:
            self.records.append(cur)
            self._cur = None

    def timing_summary(self, world):
        """Overlap of the bucket all-reduces with the backward over the recorded steps (call after a
        device synchronize): exposed_ms = end of the backward -> last bucket done (the communication
        the backward did not hide), the last step's per-bucket launch offsets from its backward's start
        (compare with backward_ms_last, that step's backward; the steps vary), and the
        algorithmic bus bandwidth 2(n-1)/n x bytes over the window first launch -> last done (a
        lower bound: the window includes waiting for gradients)."""
        if not self.records:
            return None
        nbytes = sum((e - s) * self.flat.element_size() for s, e, _ in self.buckets)
        exp, win, bwd, offs = [], [], [], []
        for r in self.records:
            if not r["done"] or not r["launch"]:
                continue
            st = r["start"]
            bwd_ms = st.elapsed_time(r["bwd_end"])
            last = st.elapsed_time(r["done"][-1])
            first = min(st.elapsed_time(ev) for ev in r["launch"].values())
            exp.append(max(0.0, last - bwd_ms))
            win.append(max(1e-6, last - first))
            bwd.append(bwd_ms)
            offs.append([round(st.elapsed_time(r["launch"][i]), 3) for i in sorted(r["launch"])])
        if not exp:
            return None
        mean = lambda v: sum(v) / len(v)  # noqa: E731
        return {"steps_timed": len(exp), "exposed_ms": round(mean(exp), 3), "exposed_ms_max": round(max(exp), 3),
                "backward_ms": round(mean(bwd), 3), "comm_window_ms": round(mean(win), 3),
                "bucket_launch_offsets_ms": offs[-1], "backward_ms_last": round(bwd[-1], 3),
                "bus_gbs": round(2.0 * (world - 1) / world * nbytes / (mean(win) * 1e-3) / 1e9, 2),
                "bytes_per_step": int(nbytes)}
