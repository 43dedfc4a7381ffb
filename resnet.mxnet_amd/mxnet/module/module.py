"""mx.mod.Module on the MI355X runtime (the object core/solver.py:58-82,115-139,170-171 drives).

bind -> rn.executor.Plan + Executor (static plan of librn calls on one GPU)
init_params / set_params / get_params -> flat fp32 master buffer (MXNet OIHW layout at the API)
init_optimizer -> SGD hyper-parameters, rescale_grad = 1/batch (x workers for dist_* stores)
forward / backward / update -> librn kernels; gradients all-reduced over RCCL in buckets while
backward runs (one process per GPU), then the fused SGD kernel on every rank.

Multi-device contexts: MXNet splits the batch evenly over `context` (core/solver.py:58-61,
train.py:34). Here each device is its own process:
  * under torchrun with world size == len(context), rank r computes slice r of every batch
    (per-slice BN statistics, summed gradients -- the same semantics);
  * one process given several contexts (the reference's own `python train.py`, script/train.sh:3)
    gets a MultiDeviceModule (module/multidev.py) that spawns one worker per device at bind and runs
    that same slice path in them, the optimizer, metrics and schedule staying in the caller.
RN_DRY_RUN=1 binds the call plan on the CPU without launching anything (host-plumbing tests).
"""
import logging
import os
import time

import numpy as np

from ..base import MXNetError
from ..context import Context, cpu
from .. import ndarray as nd
from .. import metric as metric_mod
from .. import optimizer as opt
from .. import kvstore as kvs
from ..initializer import InitDesc, Uniform
from ..io import DataDesc


def _as_list(x):
    return x if isinstance(x, (list, tuple)) else [x]


def _dist():
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist
    except ImportError:
        pass
    return None


_MultiDeviceModule = None


class BatchEndParam:
    def __init__(self, epoch, nbatch, eval_metric, locals=None):
        self.epoch, self.nbatch, self.eval_metric, self.locals = epoch, nbatch, eval_metric, locals


def _torchrun_world():
    """World size of an enclosing torchrun / torch.distributed launch (1 outside one)."""
    d = _dist()
    if d is not None:
        return d.get_world_size()
    return int(os.environ.get("WORLD_SIZE", "1"))


class Module:
    def __new__(cls, symbol=None, data_names=("data",), label_names=("softmax_label",), logger=logging, context=None,
                *args, **kwargs):
        # several contexts in one process outside a torchrun launch: the reference's own
        # `python train.py` with gpu_list (train.py:34, core/solver.py:58-61) -> one worker per device
        if cls is Module and context is not None and len(_as_list(context)) > 1 and _torchrun_world() == 1:
            from .multidev import make_module_class
            global _MultiDeviceModule
            if _MultiDeviceModule is None:
                _MultiDeviceModule = make_module_class(Module)
            return super().__new__(_MultiDeviceModule)
        return super().__new__(cls)

    def __init__(self, symbol, data_names=("data",), label_names=("softmax_label",), logger=logging, context=None,
                 work_load_list=None, fixed_param_names=None, state_names=None, group2ctxs=None,
                 compression_params=None, precision=None):
        self._symbol = symbol
        self._data_names = list(data_names or [])
        self._label_names = list(label_names or [])
        self.logger = logger
        self._context = _as_list(context if context is not None else cpu())
        self._fixed = set(fixed_param_names or [])
        self.precision = precision or os.environ.get("RN_PRECISION", "bfloat16")
        self.binded = self.params_initialized = self.optimizer_initialized = False
        self.for_training = False
        self._exec = None
        self._optimizer = None
        self._reducer = None
        self._kv = None
        self._slice = None

    # ------------------------------------------------------------------ properties
    @property
    def symbol(self):
        return self._symbol

    @property
    def data_names(self):
        return self._data_names

    @property
    def label_names(self):
        return self._label_names

    @property
    def output_names(self):
        return self._symbol.list_outputs()

    @property
    def data_shapes(self):
        return self._data_shapes

    @property
    def label_shapes(self):
        return self._label_shapes

    @property
    def output_shapes(self):
        return [(n, t.shape) for n, t in zip(self.output_names, self._exec.plan.outputs)]

    @property
    def executor(self):
        return self._exec

    # ------------------------------------------------------------------ bind
    def bind(self, data_shapes, label_shapes=None, for_training=True, inputs_need_grad=False, force_rebind=False,
             shared_module=None, grad_req="write"):
        if self.binded and not force_rebind:
            self.logger.warning("Already bound, ignoring bind()")
            return
        if inputs_need_grad:
            raise MXNetError("inputs_need_grad is not supported")
        from rn.executor import Plan, Executor
        dshapes = [(d.name, tuple(d.shape)) if isinstance(d, DataDesc) else (d[0], tuple(d[1])) for d in data_shapes]
        lshapes = [(d.name, tuple(d.shape)) if isinstance(d, DataDesc) else (d[0], tuple(d[1]))
                   for d in (label_shapes or [])]
        self._data_shapes, self._label_shapes = dshapes, lshapes
        self.for_training = for_training
        ctxs = self._context or [cpu()]  # MXNet's default context
        kinds = {c.device_type if isinstance(c, Context) else None for c in ctxs}
        if kinds == {"cpu"}:
            # mx.cpu(): the host device (BASELINE C1, rn/cpu_executor.py); one context
            if len(ctxs) != 1:
                raise MXNetError("Module: one mx.cpu() context per process (got %s)" % (ctxs,))
            return self._bind_cpu(dshapes, lshapes, for_training)
        if kinds != {"gpu"}:
            raise MXNetError("Module: contexts must all be mx.gpu() (MI355X) or one mx.cpu(); got %s" % (ctxs,))
        d = _dist()
        world = d.get_world_size() if d else 1
        local_rank = int(os.environ.get("LOCAL_RANK", d.get_rank() if d else 0))
        if len(ctxs) > 1 and world == len(ctxs):
            self._slice = (local_rank, len(ctxs))
            ctx = ctxs[local_rank]
        elif len(ctxs) > 1:
            # (one process with several contexts outside torchrun is the MultiDeviceModule)
            raise MXNetError("Module: %d contexts under a distributed launch of %d processes; MXNet's per-device "
                             "split needs one process per context (world size == len(context))" % (len(ctxs), world))
        else:
            self._slice = None
            ctx = ctxs[0]
        self._ctx = ctx
        self._total_batch = dshapes[0][1][0]
        nsl = self._slice[1] if self._slice else 1
        if self._total_batch % nsl:
            raise MXNetError("batch %d is not divisible over %d devices" % (self._total_batch, nsl))
        per = lambda shp: (shp[0] // nsl,) + tuple(shp[1:])
        pd = [(n, per(s)) for n, s in dshapes]
        pl = [(n, per(s)) for n, s in lshapes]
        from .multidev import dry_run
        plan = Plan(self._symbol, pd, pl, dtype=self.precision, for_training=for_training)
        if dry_run():  # RN_DRY_RUN=1: the call plan on the CPU, nothing launched (host-plumbing tests)
            self._exec = Executor(plan, "cpu")
        else:
            import torch
            torch.cuda.set_device(ctx.device_id)
            self._exec = Executor(plan, ctx.torch_device())
        self.binded = True

    def _bind_cpu(self, dshapes, lshapes, for_training):
        from rn.executor import Plan
        from rn.cpu_executor import CPUExecutor
        self._slice = None
        self._ctx = self._context[0] if self._context else cpu()
        self._total_batch = dshapes[0][1][0]
        plan = Plan(self._symbol, dshapes, lshapes, dtype="float32", for_training=for_training)
        self._exec = CPUExecutor(plan)
        self.binded = True

    # ------------------------------------------------------------------ params
    def init_params(self, initializer=None, arg_params=None, aux_params=None, allow_missing=False, force_init=False,
                    allow_extra=False):
        if self.params_initialized and not force_init:
            return
        assert self.binded, "call bind before initializing the parameters"
        initializer = initializer if initializer is not None else Uniform(0.01)
        ex = self._exec
        plan = ex.plan
        for name in plan.param_names:
            shp = ex.param_shape[name]
            if arg_params is not None and name in arg_params:
                v = arg_params[name]
                v = v.asnumpy() if hasattr(v, "asnumpy") else np.asarray(v)
            else:
                if arg_params is not None and not allow_missing:
                    raise MXNetError("%s is not presented" % name)
                arr = nd.zeros(shp)
                initializer(InitDesc(name), arr)
                v = arr.asnumpy()
            ex.set_param(name, v)
        for name in plan.aux_names:
            shp = ex.aux_off[name][1]
            if aux_params is not None and name in aux_params:
                v = aux_params[name]
                v = v.asnumpy() if hasattr(v, "asnumpy") else np.asarray(v)
            else:
                if aux_params is not None and not allow_missing:
                    raise MXNetError("%s is not presented" % name)
                arr = nd.zeros(shp)
                initializer(InitDesc(name), arr)
                v = arr.asnumpy()
            ex.set_aux(name, v)
        d = _dist()
        if d is not None and d.get_world_size() > 1:
            # identical replicas (MXNet initialises once on CPU and copies to every device)
            d.broadcast(ex.master, src=0)
            d.broadcast(ex.aux, src=0)
        ex.repack_weights()
        self.params_initialized = True

    def get_params(self):
        ex = self._exec
        arg = {n: nd.NDArray(ex.get_param(n)) for n in ex.plan.param_names}
        d = _dist()
        if self._slice is not None and d is not None:
            # MXNet averages aux states over devices (core/solver.py:170-171 get_params)
            import torch
            buf = ex.aux.clone()
            d.all_reduce(buf)
            buf /= d.get_world_size()
            aux = {}
            for n in ex.plan.aux_names:
                o, shp = ex.aux_off[n]
                aux[n] = nd.NDArray(buf[o:o + int(np.prod(shp))].cpu().numpy().reshape(shp).copy())
        else:
            aux = {n: nd.NDArray(ex.get_aux(n)) for n in ex.plan.aux_names}
        return arg, aux

    def set_params(self, arg_params, aux_params, allow_missing=False, force_init=True, allow_extra=False):
        self.init_params(initializer=None, arg_params=arg_params, aux_params=aux_params, allow_missing=allow_missing,
                         force_init=force_init, allow_extra=allow_extra)

    def save_params(self, fname):
        arg, aux = self.get_params()
        d = {("arg:%s" % k): v for k, v in arg.items()}
        d.update({("aux:%s" % k): v for k, v in aux.items()})
        nd.save(fname, d)

    def load_params(self, fname):
        save_dict = nd.load(fname)
        arg, aux = {}, {}
        for k, v in save_dict.items():
            tp, name = k.split(":", 1)
            (arg if tp == "arg" else aux)[name] = v
        self.set_params(arg, aux)

    def save_checkpoint(self, prefix, epoch, save_optimizer_states=False):
        from ..model import save_checkpoint
        arg, aux = self.get_params()
        save_checkpoint(prefix, epoch, self._symbol, arg, aux)

    @staticmethod
    def load(prefix, epoch, load_optimizer_states=False, **kwargs):
        from ..model import load_checkpoint
        sym, args, auxs = load_checkpoint(prefix, epoch)
        mod = Module(symbol=sym, **kwargs)
        mod._arg_params, mod._aux_params = args, auxs
        return mod

    # ------------------------------------------------------------------ optimizer
    def init_optimizer(self, kvstore="local", optimizer="sgd", optimizer_params=(("learning_rate", 0.01),),
                       force_init=False):
        if self.optimizer_initialized and not force_init:
            return
        kv = kvstore if isinstance(kvstore, kvs.KVStore) else (kvs.create(kvstore) if kvstore else None)
        self._kv = kv
        params = dict(optimizer_params)
        batch = self._total_batch
        if kv is not None and kv.type.startswith("dist") and "_sync" in kv.type:
            # MXNet: rescale = 1 / (batch x MXNet workers). In slice mode the bound batch is already the
            # global one (each rank runs one device's slice of it, as MXNet's one worker drives all of
            # len(context) devices), so only the processes beyond one per context count as workers.
            workers = kv.num_workers // len(self._context) if self._slice is not None else kv.num_workers
            batch *= max(1, workers)
        params.setdefault("rescale_grad", 1.0 / batch)
        idx2name = {i: n for i, n in enumerate(self._exec.plan.param_names)}
        self._optimizer = opt.create(optimizer, param_idx2name=idx2name, **params)
        if kv is not None:
            kv.set_optimizer(self._optimizer)
        d = _dist()
        if d is not None and d.get_world_size() > 1:
            from rn.dist import BucketAllReducer
            self._reducer = BucketAllReducer(self._exec.grad, self._exec.buckets())
        self.optimizer_initialized = True

    # ------------------------------------------------------------------ step
    def _slice_rows(self, arr):
        if self._slice is None:
            return arr
        r, n = self._slice
        per = arr.shape[0] // n
        return arr[r * per:(r + 1) * per]

    def forward(self, data_batch, is_train=None):
        if is_train is None:
            is_train = self.for_training
        ex = self._exec
        if data_batch is None:
            # extension: inputs already resident on the device (set by a previous forward)
            if is_train:
                ex.stats.zero_()
            ex.forward(is_train)
            return
        data = data_batch.data[0]
        label = data_batch.label[0] if (data_batch.label and self._label_names) else None
        dsrc = data._torch() if isinstance(data, nd.NDArray) else data
        lsrc = None
        if label is not None:
            lsrc = label._torch() if isinstance(label, nd.NDArray) else label
        if dsrc.shape[0] != self._total_batch:
            raise MXNetError("batch size %d differs from the bound %d" % (dsrc.shape[0], self._total_batch))
        ex.set_input(self._slice_rows(dsrc), None if lsrc is None else self._slice_rows(lsrc))
        if is_train:
            ex.stats.zero_()
        ex.forward(is_train)

    def backward(self, out_grads=None):
        if out_grads is not None:
            raise MXNetError("head gradients are not supported (SoftmaxOutput is a loss head)")
        ex = self._exec
        if self._reducer is not None:
            self._reducer.begin_step()
        ex.backward(hooks=self._reducer.hooks() if self._reducer else None)
        if self._reducer is not None:
            self._reducer.launched_step = True  # every bucket was launched by its backward hook

    def update(self):
        o = self._optimizer
        lr = o.step_lr()
        clip = o.clip_gradient if o.clip_gradient is not None else -1.0
        self._update_with(lr, o.wd, getattr(o, "momentum", 0.0), o.rescale_grad, clip)

    def _update_with(self, lr, wd, momentum, rescale_grad, clip):
        """kvstore push(sum) + SGD + pull: the summed gradient, then the fused update on this device."""
        ex = self._exec
        if self._reducer is not None:
            # exactly one all-reduce per backward: launched by the hooks (or here, when backward ran
            # without them), waited for here even if the caller already waited
            if not self._reducer.launched_step:
                self._reducer.launch_all()
            self._reducer.wait()
            self._reducer.launched_step = False
        ex.sgd_update(lr, wd, momentum, rescale_grad, clip)

    def get_outputs(self, merge_multi_context=True):
        return [nd.NDArray(self._exec.output(i), self._ctx) for i in range(len(self._exec.plan.outputs))]

    def update_metric(self, eval_metric, labels, pre_sliced=False):
        ex = self._exec
        n = ex.plan.outputs[0].n
        if getattr(eval_metric, "_dev_slot", None) is not None:
            eval_metric.update_device(ex.stats.clone(), n)
            return
        labels = [self._slice_rows(l.asnumpy() if hasattr(l, "asnumpy") else np.asarray(l)) for l in labels]
        eval_metric.update(labels, self.get_outputs())

    # ------------------------------------------------------------------ eval / fit
    def score(self, eval_data, eval_metric, num_batch=None, batch_end_callback=None, score_end_callback=None,
              reset=True, epoch=0):
        if reset:
            eval_data.reset()
        if not isinstance(eval_metric, metric_mod.EvalMetric):
            eval_metric = metric_mod.create(eval_metric)
        eval_metric.reset()
        for nbatch, batch in enumerate(eval_data):
            if num_batch is not None and nbatch == num_batch:
                break
            self.forward(batch, is_train=False)
            labels = [self._slice_rows(l.asnumpy()) for l in batch.label]
            eval_metric.update(labels, self.get_outputs())
            for cb in _as_list(batch_end_callback or []):
                cb(BatchEndParam(epoch, nbatch, eval_metric, locals()))
        return eval_metric.get_name_value()

    def predict(self, eval_data, num_batch=None, reset=True):
        if reset:
            eval_data.reset()
        outs = []
        for nbatch, batch in enumerate(eval_data):
            if num_batch is not None and nbatch == num_batch:
                break
            self.forward(batch, is_train=False)
            outs.append(self.get_outputs()[0].asnumpy().copy())
        return nd.NDArray(np.concatenate(outs))

    def fit(self, train_data, eval_data=None, eval_metric="acc", epoch_end_callback=None, batch_end_callback=None,
            kvstore="local", optimizer="sgd", optimizer_params=(("learning_rate", 0.01),), initializer=Uniform(0.01),
            arg_params=None, aux_params=None, allow_missing=False, force_init=False, begin_epoch=0, num_epoch=None,
            **kwargs):
        self.bind(train_data.provide_data, train_data.provide_label, for_training=True)
        self.init_params(initializer, arg_params, aux_params, allow_missing, force_init)
        self.init_optimizer(kvstore, optimizer, optimizer_params)
        if not isinstance(eval_metric, metric_mod.EvalMetric):
            eval_metric = metric_mod.create(eval_metric)
        for epoch in range(begin_epoch, num_epoch):
            tic = time.time()
            eval_metric.reset()
            for nbatch, batch in enumerate(train_data):
                self.forward(batch, is_train=True)
                self.backward()
                self.update()
                self.update_metric(eval_metric, batch.label)
                for cb in _as_list(batch_end_callback or []):
                    cb(BatchEndParam(epoch, nbatch, eval_metric, locals()))
            for name, val in eval_metric.get_name_value():
                self.logger.info("Epoch[%d] Train-%s=%f", epoch, name, val)
            self.logger.info("Epoch[%d] Time cost=%.3f", epoch, time.time() - tic)
            arg, aux = self.get_params()
            self.set_params(arg, aux)
            for cb in _as_list(epoch_end_callback or []):
                cb(epoch, self._symbol, arg, aux)
            if eval_data is not None:
                for name, val in self.score(eval_data, eval_metric, epoch=epoch):
                    self.logger.info("Epoch[%d] Validation-%s=%f", epoch, name, val)
            train_data.reset()


BaseModule = Module
