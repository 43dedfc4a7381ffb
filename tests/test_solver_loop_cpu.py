"""The reference's training driver through the drop-in `mxnet` package (CPU, RN_DRY_RUN=1: the call
plan is bound on the CPU and nothing is launched; the numerics of the same step are the GPU tests').

Restates, as user code over the shim, what the reference's driver does around the hot path:
  * train.py:158-194 -- the learning-rate schedule choice (WarmupMultiFactorScheduler, a user
    subclass of mx.lr_scheduler.LRScheduler, core/scheduler.py:9-55; multi_factor_scheduler,
    core/scheduler.py:5-7; PolyScheduler with linear warm-up, train.py:164-166) and the optimizer
    parameters;
  * core/solver.py:65-212 -- Solver.fit: bind, init_params(Xavier, train.py:221), init_optimizer,
    metric.create, per batch forward(is_train=True) / backward / update / update_metric, a
    BatchEndParam namedtuple (core/callback.py:5-19) with kvstore.rank to the Speedometer
    (train.py:219), per epoch get_params / set_params and do_checkpoint (train.py:218), train_data.reset;
  * data/imagenet.py:9-41 -- SyntheticDataIter over mx.io.DataIter with cpu_pinned NDArrays;
  * config/edict_config.py -- the EasyDict configuration the driver reads.
The learning rate handed to the fused SGD kernel at every update is checked against the oracle's
restatement of the same schedulers (oracle/ops.py)."""
import logging
import math
import os
from collections import namedtuple

import numpy as np
import pytest

import mxnet as mx
from mxnet.lr_scheduler import LRScheduler
from oracle import ops
from rn import graphs
from rn.executor import Executor


@pytest.fixture
def dry(monkeypatch):
    monkeypatch.setenv("RN_DRY_RUN", "1")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    calls = []
    orig = Executor.sgd_update

    def spy(self, lr, wd, momentum, rescale_grad, clip=-1.0):
        calls.append((lr, wd, momentum, rescale_grad, clip))
        return orig(self, lr, wd, momentum, rescale_grad, clip)

    monkeypatch.setattr(Executor, "sgd_update", spy)
    return calls


class WarmupMultiFactorScheduler(LRScheduler):
    """User code as the reference writes it (core/scheduler.py:9-55): subclasses the shim's base."""

    def __init__(self, base_lr, step, factor=1, warmup=False, warmup_type="constant", warmup_lr=0, warmup_step=0):
        super(WarmupMultiFactorScheduler, self).__init__()
        assert isinstance(step, list) and len(step) >= 1
        self.base_lr = base_lr
        self.step, self.cur_step_ind, self.factor, self.count = step, 0, factor, 0
        self.warmup, self.warmup_type, self.warmup_lr, self.warmup_step = warmup, warmup_type, warmup_lr, warmup_step

    def __call__(self, num_update):
        if self.warmup and num_update <= self.warmup_step:
            if self.warmup_type == "constant":
                return self.warmup_lr
            return (self.base_lr - self.warmup_lr) / self.warmup_step * num_update + self.warmup_lr
        while self.cur_step_ind <= len(self.step) - 1:
            if num_update > self.step[self.cur_step_ind]:
                self.count = self.step[self.cur_step_ind]
                self.cur_step_ind += 1
                self.base_lr *= self.factor
            else:
                return self.base_lr
        return self.base_lr


def multi_factor_scheduler(begin_epoch, epoch_size, step, factor=0.1):
    step_ = [epoch_size * (x - begin_epoch) for x in step if x - begin_epoch > 0]
    return mx.lr_scheduler.MultiFactorScheduler(step=step_, factor=factor) if len(step_) else None


class SyntheticDataIter(mx.io.DataIter):
    """data/imagenet.py:9-41 over the shim."""

    def __init__(self, num_classes, data_shape, max_iter, dtype):
        self.batch_size = data_shape[0]
        self.cur_iter, self.max_iter, self.dtype = 0, max_iter, dtype
        label = np.random.randint(0, num_classes, [self.batch_size])
        data = np.random.uniform(-1, 1, data_shape)
        self.data = mx.nd.array(data, dtype=self.dtype, ctx=mx.Context("cpu_pinned", 0))
        self.label = mx.nd.array(label, dtype=self.dtype, ctx=mx.Context("cpu_pinned", 0))

    def __iter__(self):
        return self

    @property
    def provide_data(self):
        return [mx.io.DataDesc("data", self.data.shape, self.dtype)]

    @property
    def provide_label(self):
        return [mx.io.DataDesc("softmax_label", (self.batch_size,), self.dtype)]

    def next(self):
        self.cur_iter += 1
        if self.cur_iter <= self.max_iter:
            return mx.io.DataBatch(data=(self.data,), label=(self.label,), pad=0, index=None,
                                   provide_data=self.provide_data, provide_label=self.provide_label)
        raise StopIteration

    def __next__(self):
        return self.next()

    def reset(self):
        self.cur_iter = 0


BatchEndParam = namedtuple("BatchEndParams", ["epoch", "nbatch", "eval_metric", "locals", "rank", "total_iter",
                                              "cur_data_time", "avg_data_time", "cur_batch_time", "avg_batch_time",
                                              "cur_kvstore_sync_time", "avg_kvstore_sync_time",
                                              "cur_iter_total_time", "avg_iter_total_time"])


def solver_fit(module, data_shapes, label_shapes, train_data, eval_metric, epoch_end_callback, batch_end_callback,
               initializer, optimizer, optimizer_params, begin_epoch, num_epoch, kvstore):
    """core/solver.py:65-212 (no eval data), the per-batch and per-epoch call sequence."""
    module.bind(data_shapes=data_shapes, label_shapes=label_shapes, for_training=True)
    module.init_params(initializer=initializer, arg_params=None, aux_params=None, allow_missing=False)
    module.init_optimizer(kvstore=kvstore, optimizer=optimizer, optimizer_params=optimizer_params)
    if not isinstance(eval_metric, mx.metric.EvalMetric):
        eval_metric = mx.metric.create(eval_metric)
    temp_count = 0
    seen = []
    for epoch in range(begin_epoch, num_epoch):
        eval_metric.reset()
        nbatch = 0
        data_iter = iter(train_data)
        end_of_batch = False
        next_data_batch = next(data_iter)
        while not end_of_batch:
            data_batch = next_data_batch
            module.forward(data_batch, is_train=True)
            module.backward()
            module.update()
            try:
                next_data_batch = next(data_iter)
            except StopIteration:
                end_of_batch = True
            module.update_metric(eval_metric, data_batch.label)
            p = BatchEndParam(epoch=epoch, nbatch=nbatch, eval_metric=eval_metric, locals=locals(),
                              rank=kvstore.rank, total_iter=temp_count, cur_data_time=0.0, avg_data_time=0.0,
                              cur_batch_time=0.0, avg_batch_time=0.0, cur_kvstore_sync_time=0.0,
                              avg_kvstore_sync_time=0.0, cur_iter_total_time=0.0, avg_iter_total_time=0.0)
            for cb in batch_end_callback:
                cb(p)
            seen.append((epoch, nbatch, temp_count))
            nbatch += 1
            temp_count += 1
        arg_params, aux_params = module.get_params()
        module.set_params(arg_params, aux_params)
        if epoch_end_callback is not None and kvstore.rank == 0:
            epoch_end_callback(epoch, module.symbol, arg_params, aux_params)
        train_data.reset()
    return eval_metric, seen


def test_solver_fit_sequence_and_lr_schedule(dry, tmp_path, caplog):
    batch, epoch_size, num_epoch = 8, 3, 3
    lr, wd, momentum = 0.4, 1e-4, 0.9
    # train.py:156-162: warm-up (lr > 0.1), lr steps in epochs -> iterations
    lr_step, warm_epoch, warmup_lr = [2], 1, 0.1
    lr_iters = [int(e * epoch_size) for e in lr_step]
    sched = WarmupMultiFactorScheduler(base_lr=lr, step=lr_iters, factor=0.1, warmup=True, warmup_type="gradual",
                                       warmup_lr=warmup_lr, warmup_step=int(warm_epoch * epoch_size))
    optimizer_params = {"learning_rate": lr, "wd": wd, "lr_scheduler": sched, "multi_precision": True,
                        "momentum": momentum}
    kv = mx.kvstore.create("device")
    mod = mx.mod.Module(graphs.resnet20_cifar(), data_names=("data",), label_names=("softmax_label",),
                        logger=logging, context=[mx.gpu(0)])
    train = SyntheticDataIter(10, (batch, 3, 32, 32), epoch_size, np.float32)
    speedo = mx.callback.Speedometer(batch, 2)
    prefix = str(tmp_path / "resnet20")
    caplog.set_level(logging.INFO)
    metric, seen = solver_fit(mod, [("data", (batch, 3, 32, 32))], [("softmax_label", (batch,))], train,
                              ["acc", mx.metric.create("top_k_accuracy", top_k=5)], mx.callback.do_checkpoint(prefix),
                              [speedo], mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2), "sgd",
                              optimizer_params, 0, num_epoch, kv)
    # every batch of every epoch ran forward/backward/update/update_metric, epochs reset the iterator
    assert seen == [(e, b, e * epoch_size + b) for e in range(num_epoch) for b in range(epoch_size)]
    # the per-update learning rate given to the SGD kernel = the oracle scheduler at num_update 1, 2, ...
    ref = ops.WarmupMultiFactorScheduler(lr, lr_iters, 0.1, True, "gradual", warmup_lr, warm_epoch * epoch_size)
    assert len(dry) == num_epoch * epoch_size
    for k, (lr_k, wd_k, mom_k, rescale_k, clip_k) in enumerate(dry):
        assert abs(lr_k - ref(k + 1)) < 1e-12, (k, lr_k, ref(k + 1))
        assert wd_k == wd and mom_k == momentum and clip_k == -1.0
        assert abs(rescale_k - 1.0 / batch) < 1e-15  # MXNet rescale_grad = 1 / batch for a local store
    assert abs(dry[-1][0] - lr * 0.1) < 1e-12  # past the step at iteration 6
    # metrics named as MXNet names them; Speedometer logged every 2 batches after its first call
    assert [n for n, _ in metric.get_name_value()] == ["accuracy", "top_k_accuracy_5"]
    assert any("Speed:" in r.getMessage() for r in caplog.records)
    # do_checkpoint each epoch: prefix-symbol.json + prefix-%04d.params, loadable as MXNet's
    for e in range(1, num_epoch + 1):
        assert os.path.exists("%s-%04d.params" % (prefix, e))
    assert os.path.exists(prefix + "-symbol.json")
    sym, arg, aux = mx.model.load_checkpoint(prefix, num_epoch)
    a2, x2 = mod.get_params()
    assert set(arg) == set(a2) and set(aux) == set(x2)
    for k in arg:
        np.testing.assert_array_equal(arg[k].asnumpy(), a2[k].asnumpy())


def test_train_py_scheduler_choices():
    """train.py:158-181: multi_factor_scheduler on epoch boundaries, PolyScheduler with warm-up."""
    epoch_size, begin_epoch = 10, 1
    s = multi_factor_scheduler(begin_epoch, epoch_size, [3, 5], factor=0.1)
    assert s.step == [20, 40]
    o = mx.optimizer.create("sgd", learning_rate=0.2, lr_scheduler=s, momentum=0.9)
    lrs = [o.step_lr() for _ in range(45)]
    ref = ops.MultiFactorScheduler([20, 40], 0.1, base_lr=0.2)
    for k, v in enumerate(lrs):
        assert abs(v - ref(k + 1)) < 1e-15, (k, v)
    assert multi_factor_scheduler(9, epoch_size, [3, 5]) is None
    # PolyScheduler(max_update, base_lr, pwr=2, final_lr=0, warmup_steps, warmup_begin_lr=0, 'linear')
    total, warm, base = 100, 10, 0.5
    p = mx.lr_scheduler.PolyScheduler(total, base_lr=base, pwr=2, final_lr=0, warmup_steps=warm,
                                      warmup_begin_lr=0, warmup_mode="linear")
    for n in range(0, total + 5):
        if n < warm:
            want = base * n / warm
        elif n <= total:
            want = base * (1 - (n - warm) / (total - warm)) ** 2
        else:
            want = 0.0
        assert abs(p(n) - want) < 1e-12, (n, p(n), want)
    f = mx.lr_scheduler.FactorScheduler(step=5, factor=0.5, base_lr=1.0)
    assert [f(n) for n in (1, 5, 6, 10, 11)] == [1.0, 1.0, 0.5, 0.5, 0.25]
    c = mx.lr_scheduler.CosineScheduler(20, base_lr=1.0, final_lr=0.0)
    assert abs(c(10) - 0.5) < 1e-12 and abs(c(20)) < 1e-12
    # the reference's warm-up subclass validates nothing itself beyond asserts; the base class the
    # user subclasses must accept the no-argument super().__init__() call (core/scheduler.py:11)
    assert isinstance(WarmupMultiFactorScheduler(0.1, [5]), LRScheduler)
    assert abs(WarmupMultiFactorScheduler(0.1, [5], warmup=True, warmup_lr=0.05, warmup_step=2)(1) - 0.05) < 1e-15


def test_xavier_and_default_initialisation(dry):
    """mx.init.Xavier(rnd_type='gaussian', factor_type='in', magnitude=2) (train.py:221): weights
    N(0, sqrt(magnitude / fan_in)) with fan_in = in_channels x kernel area; MXNet's name rules:
    *_bias / *_beta / moving_mean -> 0, *_gamma / moving_var -> 1."""
    sym = graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 1000)
    mod = mx.mod.Module(sym, context=[mx.gpu(0)])
    mod.bind(data_shapes=[("data", (2, 3, 64, 64))], label_shapes=[("softmax_label", (2,))])
    mx.random.seed(7)
    mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
    arg, aux = mod.get_params()
    nweights = 0
    for n, v in arg.items():
        a = v.asnumpy().astype(np.float64)
        if n.endswith("_weight"):
            fan_in = int(np.prod(a.shape[1:]))
            sigma = math.sqrt(2.0 / fan_in)
            assert abs(a.mean()) < 6 * sigma / math.sqrt(a.size), n
            assert abs(a.std() / sigma - 1) < max(0.02, 6 / math.sqrt(2 * a.size)), (n, a.std(), sigma)
            nweights += 1
        elif n.endswith("_gamma"):
            assert np.all(a == 1.0), n
        elif n.endswith("_beta") or n.endswith("_bias"):
            assert np.all(a == 0.0), n
        else:
            raise AssertionError("unexpected parameter %s" % n)
    assert nweights == 54  # conv0 + 16 units x 3 convs + 4 shortcuts + fc1
    for n, v in aux.items():
        a = v.asnumpy()
        assert np.all(a == (1.0 if n.endswith("moving_var") else 0.0)), n
    # MXNet's defaults (uniform, 'avg', magnitude 3): U(-s, s), s = sqrt(magnitude / ((fan_in + fan_out) / 2)),
    # fan_in = 64 x 3 x 3, fan_out = 256 x 3 x 3
    arr = mx.nd.zeros((256, 64, 3, 3))
    mx.init.Xavier(rnd_type="uniform", factor_type="avg", magnitude=3)(mx.init.InitDesc("c_weight"), arr)
    a = arr.asnumpy()
    s = math.sqrt(3.0 / ((64 * 9 + 256 * 9) / 2.0))
    assert a.max() <= s and a.min() >= -s and abs(a.std() - s / math.sqrt(3)) < 0.02 * s


def test_edict_config_as_the_driver_reads_it():
    """config/edict_config.py builds an EasyDict by attribute assignment (nested dicts included) and
    train.py reads it back by attribute; the shim's easydict behaves like easydict 1.x."""
    from easydict import EasyDict as edict
    config = edict()
    config.gpu_list = [0, 1, 2, 3]
    config.dataset = "imagenet"
    config.depth = 50
    config.batch_per_gpu = 128
    config.batch_size = config.batch_per_gpu * len(config.gpu_list)
    config.lr = 0.1 * config.batch_per_gpu * len(config.gpu_list) / 256
    config.units_dict = {"18": [2, 2, 2, 2], "50": [3, 4, 6, 3]}
    config.units = config.units_dict[str(config.depth)]
    config.quantize_setting = {"weight": {"quantize_op_name": "Quantization_int8", "attrs": {"nbits": "3"}},
                               "act": {"quantize_op_name": "Quantization_int8", "attrs": {"nbits": "4"}}}
    config.image_shape = [3, 224, 224]
    assert config.batch_size == 512 and config.units == [3, 4, 6, 3] and abs(config.lr - 0.2) < 1e-15
    # nested dicts become attribute-accessible, item and attribute access agree
    assert config.quantize_setting.weight.attrs.nbits == "3"
    assert config["quantize_setting"]["act"]["attrs"]["nbits"] == config.quantize_setting.act.attrs.nbits
    assert tuple([config.batch_size] + config.image_shape) == (512, 3, 224, 224)  # train.py:74
    assert "lr" in config and getattr(config, "warmup", None) is None
    config.update({"warmup": True})
    assert config.warmup is True and config["warmup"] is True
