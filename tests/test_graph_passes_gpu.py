"""The reference's graph passes (core/graph_optimize.py via tests/graph_passes.py) on the GPU vs the
oracle.

* fix_bn (config.fix_bn, train.py:106-109; test.py:45-48): every BatchNorm normalises with its moving
  statistics, which stay constant; one training step of ResNet-50 v2 (full [3,4,6,3] units, 64x64,
  batch 4, fp32) with non-trivial moving statistics vs oracle.net.fix_bn. ReLU decisions replayed
  (test_step_gpu.py explains why); gradients max(1e-4, 4x numpy-fp32 error), probabilities 1e-4,
  moving statistics bit-unchanged.
* merge_bn (test.py inference): the folded graph's inference probabilities vs the oracle's inference
  on the ORIGINAL graph and parameters (an algebraic identity): 1e-4; FeedForward.score (test.py:64-71)
  equals the oracle's top-1 accuracy. One training step through the folded graph vs the fix_bn oracle
  of the original parameters also checks the per-channel affine's backward (gamma' / beta' gradients
  follow by the chain rule: dgamma' = dgamma*sqrt(v+eps) + mean*dbeta, dbeta' = dbeta).
* attach_quantize_node (config.quantize_flag, train.py:111-120) with the reference's default settings
  (3-bit weights, 4-bit activations, conv0 and fc1 skipped, edict_config.py:159-195): one QAT step vs
  oracle.net.attach_quant with the device's fake-quantized tensors and ReLU decisions replayed
  (test_resnet_int8_fp32_small explains why).
"""
import numpy as np
import pytest

import mxnet as mx
from graph_passes import attach_quantize_node, fix_bn, merge_bn, shape_dict
from oracle import net as onet
from step_util import max_rel, module_step, oracle_state, replayed_parity

pytestmark = pytest.mark.gpu

CFG = ([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16)


def _assert_replayed(errs):
    bad = {n: v for n, v in errs.items() if v[0] > v[2]}
    assert not bad, sorted(bad.items(), key=lambda kv: -kv[1][0])[:5]


def _stats(aux, seed=5):
    """Non-trivial moving statistics (a fresh graph's are 0 / 1)."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, v in aux.items():
        out[k] = rng.uniform(0.5, 2.0, v.shape) if k.endswith("moving_var") else rng.standard_normal(v.shape) * 0.3
    return out


def _graphs():
    from rn import graphs
    return graphs.resnet(*CFG)


def test_fix_bn_step_fp32(gpu):
    g = onet.fix_bn(onet.resnet(*CFG))
    args, aux = oracle_state(g)
    aux = _stats(aux)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    res = module_step(fix_bn(_graphs()), args, aux, data, label, "float32")
    errs, ref = replayed_parity(res, g, args, aux, data, label)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    _assert_replayed(errs)
    for k, v in aux.items():  # use_global_stats: the moving statistics are constants
        np.testing.assert_array_equal(res["aux"][k], v.astype(np.float32), err_msg=k)


def _nd(d):
    return {k: mx.nd.array(np.asarray(v, np.float32)) for k, v in d.items()}


def test_merge_bn_inference_and_score(gpu):
    g = onet.resnet(*CFG)
    args, aux = oracle_state(g)
    aux = _stats(aux)
    data, label = onet.synthetic_batch(8, (3, 64, 64), 16)
    ref, _ = onet.forward(g, args, {k: v.copy() for k, v in aux.items()}, data, label, is_train=False)
    merged, margs, mauxs = merge_bn(fix_bn(_graphs()), _nd(args), _nd(aux))
    it = mx.io.NDArrayIter(data.astype(np.float32), label.astype(np.float32), batch_size=8,
                           label_name="softmax_label")
    mod = mx.mod.Module(merged, context=[mx.gpu(0)], precision="float32")
    mod.bind(it.provide_data, it.provide_label, for_training=False)
    mod.init_params(arg_params=margs, aux_params=mauxs, allow_extra=True)
    prob = mod.predict(it).asnumpy()
    assert sum(1 for op in mod.executor.plan.ops if op.kind == "affine") == 33
    assert max_rel(prob, ref) < 1e-4, max_rel(prob, ref)
    model = mx.model.FeedForward(merged, mx.gpu(0), arg_params=margs, aux_params=mauxs)
    acc = model.score(it)
    top1 = float(np.mean(np.argmax(ref, axis=1) == label))
    assert abs(acc - top1) < 1e-9, (acc, top1)


def test_merge_bn_training_step_fp32(gpu):
    """Backward through BroadcastScale + broadcast_add (+ReLU): the folded graph trains like the fixed
    one (data gradients and every unfolded parameter's gradient identical up to rounding)."""
    g = onet.fix_bn(onet.resnet(*CFG))
    args, aux = oracle_state(g)
    aux = _stats(aux)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    merged, margs, mauxs = merge_bn(fix_bn(_graphs()), _nd(args), _nd(aux))
    res = module_step(merged, {k: v.asnumpy() for k, v in margs.items()},
                      {k: v.asnumpy() for k, v in mauxs.items()}, data, label, "float32")
    errs, ref = replayed_parity(res, g, args, aux, data, label)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    rg = ref["grads"][0]
    gg = res["grads"][0]
    bad = []
    for name, (e, e32, tol) in errs.items():
        if name not in gg:
            continue
        if gg[name].ndim == 4 and (name.endswith("_gamma") or name.endswith("_beta")):
            continue  # folded scale / bias, shaped (1,C,1,1): checked below
        if e > tol:
            bad.append((name, e, tol))
    assert not bad, bad[:5]
    # folded BNs: y = conv*gamma' + beta' with gamma' = gamma/s, beta' = beta - gamma*mean/s,
    # s = sqrt(var+eps): dgamma' = sum(dz*conv) = dgamma*s + mean*dbeta, dbeta' = dbeta
    for name, v in gg.items():
        if v.ndim != 4 or not name.endswith("_gamma"):
            continue
        bn = name[:-len("_gamma")]
        s = np.sqrt(aux[bn + "_moving_var"] + 1e-5)
        want = rg[name] * s + aux[bn + "_moving_mean"] * rg[bn + "_beta"]
        e = np.linalg.norm(v.ravel() - want) / np.linalg.norm(want)
        tol = errs[name][2]
        assert e <= max(tol, 1e-4), (name, e, tol)
        eb = np.linalg.norm(gg[bn + "_beta"].ravel() - rg[bn + "_beta"]) / np.linalg.norm(rg[bn + "_beta"])
        assert eb <= max(errs[bn + "_beta"][2], 1e-4), (bn, eb)


def test_attach_quantize_node_step_fp32(gpu):
    from test_graph_passes_cpu import QSET
    g = onet.attach_quant(onet.resnet(*CFG), skip={"conv": 1, "fc": 1}, wbits=3, abits=4)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    sym = _graphs()
    q = attach_quantize_node(sym, shape_dict(sym, data.shape, label.shape), QSET["weight"], QSET["act"],
                             ("Convolution", "FullyConnected", "Deconvolution"), {"Convolution": 1, "FullyConnected": 1})
    res = module_step(q, args, aux, data, label, "float32")
    qv = res["quant_values"][0]
    assert len(qv) == 52 + 48
    errs, ref = replayed_parity(res, g, args, aux, data, label, quant_values=qv)
    assert max_rel(res["prob"][0], ref["prob"][0]) < 1e-4
    _assert_replayed(errs)
    st = res["mod"].get_params()[1]
    for k, v in st.items():
        if k.endswith("_minmax") and k in ref["quant_state"]:
            assert abs(v.asnumpy().item() - ref["quant_state"][k]) <= 1e-6 * ref["quant_state"][k], k
