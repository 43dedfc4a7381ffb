"""One Python process driving several devices: the reference's own launch.

`python train.py` (script/train.sh:3) builds devs = [mx.gpu(i) for i in config.gpu_list]
(train.py:34) and hands the whole list to ONE Module (core/solver.py:58-61). MXNet then ran every
device from that process, split each batch evenly over them, kept BatchNorm statistics per device,
summed the gradients through the kvstore and applied one update (core/solver.py:115-121).

MI355X design: the Module spawns one worker process per device at bind time (spawn start method:
fresh interpreters that inherit nothing of the caller's HIP state). The workers form a
torch.distributed group -- backend nccl (= RCCL over xGMI) when the devices are distinct, gloo when
a device repeats (two contexts on one GPU: a rehearsal on a one-GPU box) -- and each runs the
one-device slice path of module.py: rank r binds slice r of the global batch, per-slice BatchNorm
statistics, bucketed all-reduce launched during backward, the identical fused SGD. The parent keeps
MXNet's host-side objects -- the optimizer with its learning-rate schedule, the metrics, the
iterators, the checkpoint callbacks -- and ships each worker its slice of every batch through
shared host memory (two buffer sets, alternating per step).

This is the same arithmetic as one process per GPU under torchrun (the launch bench.py uses); it
exists so that the reference's single-process entry point runs unchanged.
"""
import atexit
import os
import socket
import time
import traceback

import numpy as np

from ..base import MXNetError


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def dry_run():
    """RN_DRY_RUN=1: executors are built on the CPU without launching kernels (CPU tests of the
    host plumbing; no numbers are produced)."""
    return os.environ.get("RN_DRY_RUN", "0") == "1"


# ----------------------------------------------------------------------------- worker side
class _Worker:
    def __init__(self, rank, device_ids, sym_json, names, precision):
        import mxnet as mx
        self.rank = rank
        sym = mx.sym.load_json(sym_json)
        ctxs = [mx.gpu(i) for i in device_ids]
        self.mod = mx.mod.Module(sym, data_names=names[0], label_names=names[1], context=ctxs, precision=precision)
        self.bufs = None
        self.pending_copy = None

    def bind(self, data_shapes, label_shapes, for_training, bufs):
        self.mod.bind(data_shapes=data_shapes, label_shapes=label_shapes, for_training=for_training)
        if self.mod._slice != (self.rank, len(self.mod._context)):
            raise MXNetError("worker %d bound slice %s" % (self.rank, self.mod._slice))
        self.bufs = bufs  # [(data, label)] x 2 shared host tensors holding this rank's slice
        return {"slice": self.mod._slice, "data_shape": self.mod.executor.plan.data_tensor.shape}

    def init_params(self, arg, aux):
        self.mod.init_params(arg_params=arg, aux_params=aux, allow_missing=False, force_init=True)

    def init_optimizer(self, kv_type):
        # the parent owns the optimizer and its schedule; here only the exchange (bucketed all-reduce)
        self.mod.init_optimizer(kvstore=kv_type, optimizer="sgd", optimizer_params={"learning_rate": 0.0},
                                force_init=True)
        return self.mod._optimizer.rescale_grad

    def forward(self, slot, is_train):
        import torch
        ex = self.mod.executor
        if self.pending_copy is not None:
            # the parent rewrites a buffer set two steps after handing it over: the copy out of it
            # (issued in the step before last) has finished before this step is acknowledged
            self.pending_copy.synchronize()
        data, label = self.bufs[slot]
        ex.set_input(data, label)
        if not ex.dry_run:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self.pending_copy = ev
        if is_train:
            ex.stats.zero_()
        ex.forward(is_train)

    def backward(self):
        self.mod.backward()

    def update(self, lr, wd, momentum, rescale, clip):
        self.mod._update_with(lr, wd, momentum, rescale, clip)

    def stats(self):
        return self.mod.executor.stats.detach().cpu().numpy().copy()

    def outputs(self):
        return [o.asnumpy().copy() for o in self.mod.get_outputs()]

    def get_params(self):
        arg, aux = self.mod.get_params()  # collective: aux averaged over the ranks
        return {k: v.asnumpy() for k, v in arg.items()}, {k: v.asnumpy() for k, v in aux.items()}

    def set_params(self, arg, aux):
        self.mod.set_params(arg, aux)

    def grads(self):
        if self.mod._reducer is not None:  # the summed gradient (update() waits again: no-op)
            self.mod._reducer.wait()
        ex = self.mod.executor
        return {n: ex.get_param(n, grad=True) for n in ex.plan.param_names}

    def env(self, name):
        """The worker's own environment value (tests: the hardware-queue count rn/__init__ chose)."""
        return os.environ.get(name)

    def input_slice(self):
        ex = self.mod.executor
        return ex._in_bufs[ex._in_idx].detach().cpu().numpy().copy()


def _worker_main(rank, world, port, device_ids, sym_json, names, precision, backend, env, conn):
    try:
        os.environ.update(env)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank))
        import torch
        from rn import dist as rdist
        if not dry_run():
            torch.cuda.set_device(device_ids[rank])
        rdist.init_from_env(backend)
        w = _Worker(rank, device_ids, sym_json, names, precision)
        conn.send(("ok", None))
    except Exception:
        conn.send(("error", traceback.format_exc()))
        return
    while True:
        try:
            cmd, args = conn.recv()
        except EOFError:
            break
        if cmd == "close":
            conn.send(("ok", None))
            break
        try:
            # fault injection for the failure-path tests: RN_FAULT_INJECT="<command>:<rank>"
            if os.environ.get("RN_FAULT_INJECT") == "%s:%d" % (cmd, rank):
                raise RuntimeError("injected fault in %s on worker %d" % (cmd, rank))
            conn.send(("ok", getattr(w, cmd)(*args)))
        except Exception:
            conn.send(("error", traceback.format_exc()))
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:
        pass


# ----------------------------------------------------------------------------- parent side
class DeviceGroup:
    """The worker processes of one multi-device Module."""

    def __init__(self, symbol, contexts, names, precision):
        import torch.multiprocessing as mp
        ids = [c.device_id for c in contexts]
        shared = len(set(ids)) < len(ids)
        backend = os.environ.get("RN_DIST_BACKEND") or ("gloo" if dry_run() or shared else "nccl")
        ctx = mp.get_context("spawn")
        port = _free_port()
        env = {k: v for k, v in os.environ.items() if k.startswith(("RN_", "HSA_", "HIP_", "NCCL_", "RCCL_"))}
        # A spawned worker imports rn (rn/__init__.py sets GPU_MAX_HW_QUEUES) while unpickling its target,
        # before _worker_main applies `env`: what it must see then is set in os.environ around p.start()
        # (spawn copies the parent's environment at that moment). Ranks sharing one GPU keep HIP's 4
        # hardware queues -- 8 per process oversubscribe the queue slots there (rn/__init__.py) -- and the
        # parent's own GPU_MAX_HW_QUEUES (raised to 8 by its `import rn`) must not leak into them.
        # (explicit for distinct devices too: the worker may import rn only after it has set WORLD_SIZE, and
        # a gloo backend over distinct GPUs is not a shared GPU)
        start_env = ({"RN_HW_QUEUES": "4", "GPU_MAX_HW_QUEUES": "4"} if shared
                     else {"RN_HW_QUEUES": os.environ.get("RN_HW_QUEUES", "8")})
        env.update(RN_HW_QUEUES=start_env["RN_HW_QUEUES"])
        saved = {k: os.environ.get(k) for k in start_env}
        self.conns, self.procs = [], []
        try:
            os.environ.update(start_env)
            for r in range(len(ids)):
                a, b = ctx.Pipe()
                p = ctx.Process(target=_worker_main, args=(r, len(ids), port, ids, symbol.tojson(), names, precision,
                                                           backend, env, b), daemon=True)
                p.start()
                self.conns.append(a)
                self.procs.append(p)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        self.backend = backend
        self._collect()  # every worker initialised its process group
        atexit.register(self.close)

    def _collect(self, timeout=None):
        """Every worker's reply to the last command, in rank order. Replies are taken in whatever
        order they arrive: the first error (or a worker that dies, or no reply within `timeout`
        seconds: RN_WORKER_TIMEOUT, default 1800) ends the wait at once and kills every worker --
        its peers may be blocked in a collective it will never join, so they are not asked to close."""
        from multiprocessing.connection import wait
        if timeout is None:
            timeout = float(os.environ.get("RN_WORKER_TIMEOUT", "1800"))
        deadline = time.monotonic() + timeout
        out = [None] * len(self.conns)
        pending = dict(enumerate(self.conns))
        errs = []
        while pending and not errs:
            left = deadline - time.monotonic()
            if left <= 0:
                errs.append("no reply from worker(s) %s within %.0f s" % (sorted(pending), timeout))
                break
            sentinels = {self.procs[r].sentinel: r for r in pending}
            ready = wait(list(pending.values()) + list(sentinels), timeout=min(left, 5.0))
            for r, c in list(pending.items()):
                if c.poll():
                    try:
                        status, val = c.recv()
                    except (EOFError, OSError):
                        errs.append("worker %d exited (code %s)" % (r, self.procs[r].exitcode))
                        del pending[r]
                        continue
                    del pending[r]
                    out[r] = val
                    if status != "ok":
                        errs.append("worker %d:\n%s" % (r, val))
                elif self.procs[r].sentinel in ready:
                    self.procs[r].join(timeout=1)
                    errs.append("worker %d exited (code %s) without replying" % (r, self.procs[r].exitcode))
                    del pending[r]
        if errs:
            self.kill()
            raise MXNetError("\n".join(errs))
        return out

    def kill(self):
        """Stop every worker without asking (used after a failure)."""
        for p in self.procs:
            if p.is_alive():
                p.kill()
        for p in self.procs:
            p.join(timeout=10)
        for c in self.conns:
            try:
                c.close()
            except OSError:
                pass
        self.conns, self.procs = [], []

    def call(self, cmd, *args, per_rank=None):
        """Run `cmd` on every worker (per_rank: one argument tuple per worker); results by rank."""
        if not self.conns:
            raise MXNetError("the device workers are gone (an earlier command failed)")
        for r, c in enumerate(self.conns):
            try:
                c.send((cmd, per_rank[r] if per_rank is not None else args))
            except OSError:
                self.procs[r].join(timeout=1)
                code = self.procs[r].exitcode
                self.kill()
                raise MXNetError("worker %d exited (code %s)" % (r, code))
        return self._collect()

    def close(self):
        for c, p in zip(self.conns, self.procs):
            try:
                if p.is_alive():
                    c.send(("close", ()))
                    c.recv()
            except (OSError, EOFError):
                pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        self.conns, self.procs = [], []


def make_module_class(Module):
    """The multi-device Module: a subclass of module.Module that Module.__new__ returns when one
    process is given several contexts outside a torchrun launch."""
    from .. import ndarray as nd
    from .. import optimizer as opt
    from .. import kvstore as kvs
    from ..initializer import InitDesc, Uniform
    from ..io import DataDesc

    class MultiDeviceModule(Module):
        def __init__(self, *a, **kw):
            super().__init__(*a, **kw)
            self._group = None
            self._slot = 0
            self._outputs_cache = None

        @property
        def executor(self):
            return None

        @property
        def output_shapes(self):
            _, outs, _ = self._symbol.infer_shape(**dict(self._data_shapes + self._label_shapes))
            return list(zip(self.output_names, outs))

        def _known(self):
            return set(dict(self._data_shapes + self._label_shapes))

        def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
                 shared_module=None, grad_req="write"):
            if self.binded and not force_rebind:
                self.logger.warning("Already bound, ignoring bind()")
                return
            if inputs_need_grad:
                raise MXNetError("inputs_need_grad is not supported")
            import torch
            for c in self._context:
                if c.device_type != "gpu":
                    raise MXNetError("the MI355X runtime executes on mx.gpu() contexts only (got %s)" % (c,))
            ds = [(d.name, tuple(d.shape)) if isinstance(d, DataDesc) else (d[0], tuple(d[1])) for d in data_shapes]
            ls = [(d.name, tuple(d.shape)) if isinstance(d, DataDesc) else (d[0], tuple(d[1]))
                  for d in (label_shapes or [])]
            self._data_shapes, self._label_shapes = ds, ls
            n = len(self._context)
            self._total_batch = ds[0][1][0]
            if self._total_batch % n:
                raise MXNetError("batch %d is not divisible over %d devices" % (self._total_batch, n))
            self._per = self._total_batch // n
            self.for_training = for_training
            self._group = DeviceGroup(self._symbol, self._context, (self._data_names, self._label_names),
                                      self.precision)
            # two sets of shared host buffers per worker (data slice, label slice), alternating per step
            dnum = self._per * int(np.prod(ds[0][1][1:]))
            self._bufs = [[(torch.zeros(dnum, dtype=torch.float32).share_memory_(),
                            torch.zeros(self._per, dtype=torch.float32).share_memory_()) for _ in range(2)]
                          for _ in range(n)]
            info = self._group.call("bind", per_rank=[(ds, ls, for_training, self._bufs[r]) for r in range(n)])
            for r, i in enumerate(info):
                if i["slice"] != (r, n) or i["data_shape"][0] != self._per:
                    raise MXNetError("worker %d bound %s" % (r, i))
            self.binded = True

        def init_params(self, initializer=None, arg_params=None, aux_params=None, allow_missing=False,
                        force_init=False, allow_extra=False):
            if self.params_initialized and not force_init:
                return
            assert self.binded, "call bind before initializing the parameters"
            initializer = initializer if initializer is not None else Uniform(0.01)
            args, _, auxs = self._symbol.infer_shape(**dict(self._data_shapes + self._label_shapes))
            shapes = dict(zip(self._symbol.list_arguments(), args))
            ashapes = dict(zip(self._symbol.list_auxiliary_states(), auxs))
            known = self._known()

            def fill(names, given, shape_of):
                out = {}
                for name in names:
                    if given is not None and name in given:
                        v = given[name]
                        out[name] = np.asarray(v.asnumpy() if hasattr(v, "asnumpy") else v, dtype=np.float32)
                    else:
                        if given is not None and not allow_missing:
                            raise MXNetError("%s is not presented" % name)
                        arr = nd.zeros(shape_of[name])
                        initializer(InitDesc(name), arr)
                        out[name] = arr.asnumpy()
                return out
            arg = fill([a for a in self._symbol.list_arguments() if a not in known], arg_params, shapes)
            aux = fill(self._symbol.list_auxiliary_states(), aux_params, ashapes)
            self._group.call("init_params", arg, aux)
            self.params_initialized = True

        def get_params(self):
            arg, aux = self._group.call("get_params")[0]
            return {k: nd.NDArray(v) for k, v in arg.items()}, {k: nd.NDArray(v) for k, v in aux.items()}

        def set_params(self, arg_params, aux_params, allow_missing=False, force_init=True, allow_extra=False):
            cv = lambda d: {k: np.asarray(v.asnumpy() if hasattr(v, "asnumpy") else v, np.float32)
                            for k, v in d.items()}
            self._group.call("set_params", cv(arg_params), cv(aux_params))
            self.params_initialized = True

        def init_optimizer(self, kvstore="local", optimizer="sgd", optimizer_params=(("learning_rate", 0.01),),
                           force_init=False):
            if self.optimizer_initialized and not force_init:
                return
            kv = kvstore if isinstance(kvstore, kvs.KVStore) else (kvs.create(kvstore) if kvstore else None)
            self._kv = kv
            params = dict(optimizer_params)
            # one MXNet worker drives every device: rescale = 1 / global batch (x machines for dist_*)
            workers = kv.num_workers if (kv is not None and kv.type.startswith("dist") and "_sync" in kv.type) else 1
            params.setdefault("rescale_grad", 1.0 / (self._total_batch * max(1, workers)))
            known = self._known()
            idx2name = dict(enumerate(a for a in self._symbol.list_arguments() if a not in known))
            self._optimizer = opt.create(optimizer, param_idx2name=idx2name, **params)
            if kv is not None:
                kv.set_optimizer(self._optimizer)
            self._group.call("init_optimizer", "dist_sync_device")
            self.optimizer_initialized = True

        def forward(self, data_batch, is_train=None):
            import torch
            if is_train is None:
                is_train = self.for_training
            data = data_batch.data[0]
            data = data.asnumpy() if hasattr(data, "asnumpy") else np.asarray(data)
            if data.shape[0] != self._total_batch:
                raise MXNetError("batch size %d differs from the bound %d" % (data.shape[0], self._total_batch))
            label = None
            if data_batch.label and self._label_names:
                lab = data_batch.label[0]
                label = lab.asnumpy() if hasattr(lab, "asnumpy") else np.asarray(lab)
            slot = self._slot
            self._slot ^= 1
            p = self._per
            for r in range(len(self._context)):
                d, l_ = self._bufs[r][slot]
                d.copy_(torch.from_numpy(np.ascontiguousarray(data[r * p:(r + 1) * p], dtype=np.float32)).reshape(-1))
                if label is not None:
                    l_.copy_(torch.from_numpy(np.ascontiguousarray(label[r * p:(r + 1) * p], dtype=np.float32)))
            self._outputs_cache = None
            self._group.call("forward", slot, bool(is_train))

        def backward(self, out_grads=None):
            if out_grads is not None:
                raise MXNetError("head gradients are not supported (SoftmaxOutput is a loss head)")
            self._group.call("backward")

        def update(self):
            o = self._optimizer
            lr = o.step_lr()
            clip = o.clip_gradient if o.clip_gradient is not None else -1.0
            self._group.call("update", float(lr), float(o.wd), float(getattr(o, "momentum", 0.0)),
                             float(o.rescale_grad), float(clip))

        def get_outputs(self, merge_multi_context=True):
            if self._outputs_cache is None:
                outs = self._group.call("outputs")
                self._outputs_cache = [np.concatenate([o[i] for o in outs], axis=0) for i in range(len(outs[0]))]
            return [nd.NDArray(o) for o in self._outputs_cache]

        def update_metric(self, eval_metric, labels, pre_sliced=False):
            if getattr(eval_metric, "_dev_slot", None) is not None:
                import torch
                st = np.sum(self._group.call("stats"), axis=0)
                eval_metric.update_device(torch.from_numpy(st.astype(np.float32)), self._total_batch)
                return
            eval_metric.update([l.asnumpy() if hasattr(l, "asnumpy") else np.asarray(l) for l in labels],
                               self.get_outputs())

        def _slice_rows(self, arr):
            return arr  # the parent always holds the whole batch

        # hooks for tests and diagnostics
        def worker_grads(self):
            return self._group.call("grads")

        def worker_inputs(self):
            return self._group.call("input_slice")

        def close(self):
            if self._group is not None:
                self._group.close()
                self._group = None

    return MultiDeviceModule
