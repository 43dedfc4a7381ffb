"""One process, two contexts (the reference's `python train.py` with gpu_list, script/train.sh:3,
train.py:34, core/solver.py:58-61) on the CPU: RN_DRY_RUN=1 builds every worker's call plan without
launching kernels, so this checks the host plumbing -- two worker processes each bound to its slice
of the global batch, the batch split MXNet's way, parameters identical on both, the learning-rate
schedule and rescale_grad owned by the caller, gradient buckets all-reduced over gloo."""
import numpy as np
import pytest

import mxnet as mx
from rn import graphs


@pytest.fixture
def dry(monkeypatch):
    monkeypatch.setenv("RN_DRY_RUN", "1")
    monkeypatch.delenv("WORLD_SIZE", raising=False)


def test_two_contexts_split_the_batch(dry):
    sym = graphs.resnet20_cifar()
    mod = mx.mod.Module(sym, context=[mx.gpu(0), mx.gpu(1)])
    assert type(mod).__name__ == "MultiDeviceModule"
    try:
        mod.bind(data_shapes=[("data", (8, 3, 32, 32))], label_shapes=[("softmax_label", (8,))])
        assert mod._group.backend == "gloo"
        mx.random.seed(1)
        mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
        sched = mx.lr_scheduler.MultiFactorScheduler(step=[2], factor=0.1)
        mod.init_optimizer(kvstore="device", optimizer="sgd",
                           optimizer_params={"learning_rate": 0.1, "momentum": 0.9, "wd": 1e-4, "lr_scheduler": sched})
        assert abs(mod._optimizer.rescale_grad - 1.0 / 8) < 1e-15  # one MXNet worker, global batch 8
        rng = np.random.default_rng(0)
        data = rng.uniform(-1, 1, (8, 3, 32, 32)).astype(np.float32)
        label = rng.integers(0, 10, 8).astype(np.float32)
        batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
        lrs = []
        for step in range(3):
            mod.forward(batch, is_train=True)
            ins = mod.worker_inputs()  # each worker's device input buffer holds its slice
            for r in range(2):
                np.testing.assert_array_equal(ins[r].reshape(4, 3, 32, 32), data[4 * r:4 * r + 4])
            mod.backward()
            lrs.append(mod._optimizer.lr_scheduler(mod._optimizer.num_update + 1))
            mod.update()
        assert lrs == [0.1, 0.1, pytest.approx(0.01)]
        arg, aux = mod.get_params()
        assert len(arg) == 65 and "stage1_unit1_conv1_weight" in arg
        # parameters set through the group come back unchanged (OIHW at the API)
        arg2 = {k: mx.nd.array(v.asnumpy() * 0 + 0.5) for k, v in arg.items()}
        mod.set_params(arg2, aux)
        back, _ = mod.get_params()
        assert all(np.all(v.asnumpy() == 0.5) for v in back.values())
        m = mx.metric.create("acc")
        mod.update_metric(m, batch.label)
        assert mod.output_shapes[0][1] == (8, 10)
    finally:
        mod.close()


def test_worker_failure_in_a_collective_raises_instead_of_hanging(dry, monkeypatch):
    """worker 1 raises inside get_params (the aux all-reduce of core/solver.py:170) while
    worker 0 blocks in that collective; the parent must report the error promptly and kill both."""
    import time
    monkeypatch.setenv("RN_FAULT_INJECT", "get_params:1")
    mod = mx.mod.Module(graphs.resnet20_cifar(), context=[mx.gpu(0), mx.gpu(1)])
    try:
        mod.bind(data_shapes=[("data", (4, 3, 32, 32))], label_shapes=[("softmax_label", (4,))])
        mx.random.seed(1)
        mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
        procs = list(mod._group.procs)
        t0 = time.monotonic()
        with pytest.raises(mx.MXNetError, match="injected fault in get_params on worker 1"):
            mod.get_params()
        assert time.monotonic() - t0 < 60
        assert not any(p.is_alive() for p in procs)  # worker 0 was stuck in the all-reduce: killed
    finally:
        mod.close()


def test_worker_death_is_reported(dry):
    mod = mx.mod.Module(graphs.resnet20_cifar(), context=[mx.gpu(0), mx.gpu(1)])
    try:
        mod.bind(data_shapes=[("data", (4, 3, 32, 32))], label_shapes=[("softmax_label", (4,))])
        mod._group.procs[0].kill()
        with pytest.raises(mx.MXNetError, match="worker 0 exited"):
            mod._group.call("stats")
    finally:
        mod.close()


def test_multi_context_under_mismatched_launch_raises(dry, monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "3")
    mod = mx.mod.Module(graphs.resnet20_cifar(), context=[mx.gpu(0), mx.gpu(1)])
    assert type(mod).__name__ == "Module"
    with pytest.raises(mx.MXNetError):
        mod.bind(data_shapes=[("data", (8, 3, 32, 32))], label_shapes=[("softmax_label", (8,))])
