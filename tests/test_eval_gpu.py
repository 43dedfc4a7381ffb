"""Eval path: Module.score / predict with moving BatchNorm statistics
(core/solver.py:176-210, the reference's per-epoch validation) against the oracle's inference
forward, and a checkpoint written by one Module and loaded by another (train.py:90-95) giving the
same predictions on the GPU."""
import numpy as np
import pytest

import mxnet as mx
from oracle import net as onet
from rn import graphs

pytestmark = pytest.mark.gpu


def _setup(batch=16, nbatch=3):
    g = onet.resnet20_cifar()
    args, aux = onet.init_params(g)
    rng = np.random.default_rng(11)
    aux = {k: (np.abs(v + rng.standard_normal(v.shape) * 0.2) if k.endswith("_var") else
               v + rng.standard_normal(v.shape) * 0.2) for k, v in aux.items()}
    data = rng.uniform(-1, 1, (batch * nbatch, 3, 32, 32))
    label = rng.integers(0, 10, batch * nbatch).astype(np.float64)
    return g, args, aux, data, label


def _oracle_topk(g, args, aux, data, label, batch):
    probs = []
    for i in range(0, data.shape[0], batch):
        p, _ = onet.forward(g, args, dict(aux), data[i:i + batch], label[i:i + batch], is_train=False)
        probs.append(p)
    p = np.concatenate(probs)
    order = np.argsort(p, axis=1)
    top1 = float(np.mean(order[:, -1] == label))
    top5 = float(np.mean([label[i] in order[i, -5:] for i in range(len(label))]))
    return p, top1, top5


def _module(sym, args, aux, batch):
    mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision="float32")
    mod.bind(data_shapes=[("data", (batch, 3, 32, 32))], label_shapes=[("softmax_label", (batch,))],
             for_training=False)
    mod.init_params(arg_params={k: v.astype(np.float32) for k, v in args.items()},
                    aux_params={k: v.astype(np.float32) for k, v in aux.items()})
    return mod


def test_score_and_predict_match_oracle(gpu):
    batch = 16
    g, args, aux, data, label = _setup(batch)
    sym = graphs.resnet_cifar10([3, 3, 3], 3, [16, 16, 32, 64], 10)
    mod = _module(sym, args, aux, batch)
    it = mx.io.NDArrayIter(data, label, batch_size=batch)
    res = dict(mod.score(it, mx.metric.create(["acc", mx.metric.TopKAccuracy(top_k=5)])))
    p_ref, top1, top5 = _oracle_topk(g, args, aux, data, label, batch)
    assert abs(res["accuracy"] - top1) < 1e-9 and abs(res["top_k_accuracy_5"] - top5) < 1e-9, (res, top1, top5)
    p = mod.predict(it).asnumpy()
    assert np.abs(p - p_ref).max() / np.abs(p_ref).max() < 2e-5


def test_checkpoint_reload_predicts_the_same(gpu, tmp_path):
    batch = 16
    g, args, aux, data, label = _setup(batch, nbatch=2)
    sym = graphs.resnet_cifar10([3, 3, 3], 3, [16, 16, 32, 64], 10)
    mod = _module(sym, args, aux, batch)
    it = mx.io.NDArrayIter(data, label, batch_size=batch)
    p0 = mod.predict(it).asnumpy()
    prefix = str(tmp_path / "r20")
    mod.save_checkpoint(prefix, 3)
    sym2, args2, aux2 = mx.model.load_checkpoint(prefix, 3)
    mod2 = mx.mod.Module(sym2, context=[mx.gpu(0)], precision="float32")
    mod2.bind(data_shapes=[("data", (batch, 3, 32, 32))], label_shapes=[("softmax_label", (batch,))],
              for_training=False)
    mod2.set_params(args2, aux2)
    np.testing.assert_array_equal(mod2.predict(it).asnumpy(), p0)
