"""One process, two contexts on the GPU (the reference's `python train.py` with gpu_list:
script/train.sh:3, train.py:34, core/solver.py:58-61). Both contexts are gpu(0) on this one-GPU box,
so the two spawned workers exchange over gloo (RCCL refuses a repeated device); the arithmetic is
the RCCL path's. MXNet semantics checked: worker r runs slice r of the global batch with its own BN
statistics, the all-reduced gradient equals the sum of two single-device modules run on the slices,
and the update equals MXNet's SGD on that sum with rescale_grad = 1/global batch."""
import numpy as np
import pytest

import mxnet as mx
from oracle import ops
from rn import graphs

pytestmark = pytest.mark.gpu


def test_two_contexts_one_process(gpu):
    sym = graphs.resnet20_cifar()
    rng = np.random.default_rng(5)
    data = rng.uniform(-1, 1, (8, 3, 32, 32)).astype(np.float32)
    label = rng.integers(0, 10, 8).astype(np.float32)
    opt = {"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9}
    mx.random.seed(4)
    mod = mx.mod.Module(sym, context=[mx.gpu(0), mx.gpu(0)], precision="float32")
    assert type(mod).__name__ == "MultiDeviceModule"
    try:
        mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", (8,))])
        mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
        mod.init_optimizer(kvstore="device", optimizer="sgd", optimizer_params=opt)
        arg0, aux0 = mod.get_params()
        arg0 = {k: v.asnumpy() for k, v in arg0.items()}
        aux0 = {k: v.asnumpy() for k, v in aux0.items()}
        mod.forward(mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)]), is_train=True)
        mod.backward()
        gs = mod.worker_grads()
        mod.update()
        arg1, _ = mod.get_params()
    finally:
        mod.close()
    ref = {}
    for r in range(2):  # the two slices, each on its own single-device module
        m = mx.mod.Module(sym, context=[mx.gpu(0)], precision="float32")
        m.bind(data_shapes=[("data", (4, 3, 32, 32))], label_shapes=[("softmax_label", (4,))])
        m.init_params(arg_params=arg0, aux_params=aux0)
        m.forward(mx.io.DataBatch(data=[mx.nd.array(data[4 * r:4 * r + 4])],
                                  label=[mx.nd.array(label[4 * r:4 * r + 4])]), is_train=True)
        m.backward()
        for n in m.executor.plan.param_names:
            ref[n] = ref.get(n, 0) + m.executor.get_param(n, grad=True).astype(np.float64)
    for n, g in ref.items():
        scale = max(1e-6, float(np.abs(g).max()))
        for r in range(2):
            assert float(np.abs(gs[r][n] - g).max()) / scale < 1e-5, (n, r)
    for k, w0 in arg0.items():
        w = w0.astype(np.float64).copy()
        ops.sgd_mom_update(w, ref[k], np.zeros_like(w), 0.1, 1e-4 * ops.wd_mult_for(k), 0.9, 1.0 / 8)
        bound = 1e-3 * float(np.abs(w - w0).max()) + 2e-7 * float(np.abs(w).max()) + 1e-30
        assert float(np.abs(arg1[k].asnumpy() - w).max()) <= bound, k
