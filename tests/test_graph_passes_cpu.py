"""The reference's graph passes (core/graph_optimize.py) on the shim, CPU side: graph structure,
folded parameters and the bound call plan (RN_DRY_RUN=1: nothing launched). The numerics of the same
graphs are tests/test_graph_passes_gpu.py's; the oracle restatements of the passes
(oracle.net.fix_bn / attach_quant) are pinned here against the graphs they must equal."""
import json

import numpy as np
import pytest

import mxnet as mx
from graph_passes import attach_quantize_node, fix_bn, merge_bn, shape_dict
from oracle import net as onet
from oracle import ops
from rn import graphs

R50_SMALL = dict(units=[3, 4, 6, 3], num_stage=4, filter_list=[64, 256, 512, 1024, 2048], num_classes=16)
QSET = {  # edict_config.py:159-186 (the reference's default quantize_setting)
    "weight": {"quantize_op_name": "Quantization_int8", "init_value": 0,
               "attrs": {"nbits": "3", "quant_mode": "minmax", "is_weight": "True", "is_weight_perchannel": "False",
                         "delay_quant": "0", "ema_decay": "0.99", "grad_mode": "ste", "fix_act_scale": "False"}},
    "act": {"quantize_op_name": "Quantization_int8", "init_value": 0,
            "attrs": {"nbits": "4", "quant_mode": "minmax", "is_weight": "False", "is_weight_perchannel": "False",
                      "delay_quant": "0", "ema_decay": "0.99", "grad_mode": "ste", "fix_act_scale": "False"}},
}


@pytest.fixture
def dry(monkeypatch):
    monkeypatch.setenv("RN_DRY_RUN", "1")
    monkeypatch.delenv("WORLD_SIZE", raising=False)


def _nodes(sym):
    return json.loads(sym.tojson())["nodes"]


def _bind(sym, shape=(2, 3, 64, 64), for_training=True, precision="float32"):
    mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision=precision)
    mod.bind(data_shapes=[("data", shape)], label_shapes=[("softmax_label", (shape[0],))], for_training=for_training)
    return mod


def _call_names(calls):
    return [c[0] for c in calls]


def test_fix_bn_graph_and_plan(dry):
    sym = fix_bn(graphs.resnet(**R50_SMALL))
    bns = [n for n in _nodes(sym) if n["op"] == "BatchNorm"]
    assert len(bns) == 51 and all(n["attrs"]["use_global_stats"] == "True" for n in bns)
    ex = _bind(sym).executor
    assert all(op.use_global_stats for op in ex.plan.ops if op.kind == "bn")
    names = _call_names(ex._bwd)
    nbn = sum(1 for op in ex.plan.ops if op.kind == "bn")
    # every BN backward is the global-statistics one; no batch-statistics reduction fused into a dgrad
    assert names.count("rn_bn_bwd_global") == nbn
    assert "rn_bn_bwd_part" not in names and "rn_conv_bwd_data_bnred" not in names
    assert "rn_bn_fwd_train_part" not in _call_names(ex._fwd_train)
    # the unfixed graph keeps batch statistics
    ex0 = _bind(graphs.resnet(**R50_SMALL)).executor
    assert "rn_bn_bwd_global" not in _call_names(ex0._bwd)


def _random_params(sym, shape, seed=0):
    arg_shapes, _, aux_shapes = sym.infer_shape(data=shape, softmax_label=(shape[0],))
    rng = np.random.default_rng(seed)
    args = {n: mx.nd.array(rng.standard_normal(s).astype(np.float32) * 0.1)
            for n, s in zip(sym.list_arguments(), arg_shapes) if n not in ("data", "softmax_label")}
    auxs = {}
    for n, s in zip(sym.list_auxiliary_states(), aux_shapes):
        v = rng.uniform(0.5, 2.0, s) if n.endswith("moving_var") else rng.standard_normal(s) * 0.2
        auxs[n] = mx.nd.array(v.astype(np.float32))
    return args, auxs


def test_merge_bn_folds_conv_batchnorms(dry):
    shape = (2, 3, 64, 64)
    sym = fix_bn(graphs.resnet(**R50_SMALL))
    args, auxs = _random_params(sym, shape)
    ref_args = {k: v.asnumpy().copy() for k, v in args.items()}
    ref_aux = {k: v.asnumpy().copy() for k, v in auxs.items()}
    merged, margs, mauxs = merge_bn(sym, args, auxs)
    nodes = _nodes(merged)
    # bn0 (after conv0) and every unit's bn2 / bn3 (after conv1 / conv2) fold; bn_data, the units'
    # bn1 (after the residual sum) and the final bn1 stay BatchNorm
    scales = [n for n in nodes if n["op"] == "_contrib_BroadcastScale"]
    assert len(scales) == 1 + 2 * 16
    assert sum(1 for n in nodes if n["op"] == "BatchNorm") == 51 - 33
    for n in scales:
        bn = nodes[n["inputs"][1][0]]["name"][:-len("_gamma")]  # the scaler Variable <bn>_gamma
        g, b = margs[bn + "_gamma"].asnumpy(), margs[bn + "_beta"].asnumpy()
        assert g.shape == b.shape == (1, ref_args[bn + "_gamma"].shape[0], 1, 1)
        inv = 1.0 / np.sqrt(ref_aux[bn + "_moving_var"].astype(np.float64) + 1e-5)
        np.testing.assert_allclose(g.ravel(), ref_args[bn + "_gamma"] * inv, rtol=1e-6)
        np.testing.assert_allclose(b.ravel(), ref_args[bn + "_beta"] - ref_args[bn + "_gamma"] *
                                   ref_aux[bn + "_moving_mean"] * inv, rtol=1e-5, atol=1e-6)
        assert np.all(mauxs[bn + "_moving_mean"].asnumpy() == 0) and np.all(mauxs[bn + "_moving_var"].asnumpy() == 1)
    # the plan: one per-channel affine (+ the following ReLU) per folded BN, inference and training
    for training in (False, True):
        ex = _bind(merged, shape, for_training=training).executor
        aff = [op for op in ex.plan.ops if op.kind == "affine"]
        assert len(aff) == 33 and all(op.relu and op.gamma and op.beta for op in aff)
        assert sum(1 for op in ex.plan.ops if op.kind == "bn") == 17  # + bn_data, folded into the stem
        assert _call_names(ex._fwd_infer).count("rn_bn_apply") == 33
        if training:
            assert _call_names(ex._bwd).count("rn_bn_bwd_global") == 50  # 17 fixed BNs + 33 affines


def test_feedforward_score_plumbing(dry):
    """test.py:64-71: mx.model.FeedForward(symbol, ctx, arg_params, aux_params).score(iterator)."""
    shape = (4, 3, 32, 32)
    sym = graphs.resnet(**R50_SMALL)
    args, auxs = _random_params(sym, shape)
    merged, margs, mauxs = merge_bn(fix_bn(sym), args, auxs)
    it = mx.io.NDArrayIter(np.zeros(shape, np.float32), np.zeros((4,), np.float32), batch_size=4,
                           label_name="softmax_label")
    model = mx.model.FeedForward(merged, mx.gpu(0), arg_params=margs, aux_params=mauxs)
    acc = model.score(it)
    assert 0.0 <= acc <= 1.0


def test_attach_quantize_node_graph_and_plan(dry):
    shape = (2, 3, 64, 64)
    sym = graphs.resnet(**R50_SMALL)
    q = attach_quantize_node(sym, shape_dict(sym, shape, (2,)), QSET["weight"], QSET["act"],
                             ("Convolution", "FullyConnected", "Deconvolution"), {"Convolution": 1, "FullyConnected": 1})
    nodes = _nodes(q)
    quants = [n for n in nodes if n["op"] == "_contrib_Quantization_int8"]
    w = [n for n in quants if n["attrs"]["is_weight"] == "True"]
    a = [n for n in quants if n["attrs"]["is_weight"] == "False"]
    # conv0 and fc1 skipped; 52 conv weights; per unit one node for act1 (conv1 + shortcut share it),
    # act2, act3: 48 activation nodes
    assert len(w) == 52 and len(a) == 48
    assert {n["name"] for n in a} == {"stage%d_unit%d_relu%d" % (i, j, k) for i, u in zip(range(1, 5), (3, 4, 6, 3))
                                      for j in range(1, u + 1) for k in (1, 2, 3)}
    assert all(n["attrs"]["nbits"] == "3" for n in w) and all(n["attrs"]["nbits"] == "4" for n in a)
    ex = _bind(q, shape).executor
    qops = [op for op in ex.plan.ops if op.kind == "quant"]
    assert len(qops) == 48 and all(op.q["nbits"] == 4 for op in qops)
    convs = [op for op in ex.plan.ops if op.kind == "conv"]
    assert len(convs) == 52 and all(op.qweight is not None and op.qweight["nbits"] == 3 for op in convs)
    stem = [op for op in ex.plan.ops if op.kind == "stem"]
    assert len(stem) == 1 and stem[0].qweight is None and stem[0].quant is None
    # minmax states are aux states of the new graph
    assert sum(1 for n in q.list_auxiliary_states() if n.endswith("_minmax")) == 100


def test_int8_forward_plan(dry, monkeypatch):
    """Quantized convs whose data quantizer is a separate op run the int8 MFMA forward (rn_conv_fwd_i8)
    fed by the quantizer's codes (rn_quant_int8_fwd_codes); the stem (quantizer folded into its
    im2col) and fc1 stay on the fake-quant path; RN_INT8_MFMA=0 turns it off."""
    shape = (2, 3, 64, 64)
    # npair: BNs whose output two quantizers read (resnet_int8's first units: conv1 and the shortcut
    # each quantize act1; attach_quantize_node shares one quantizer per tensor)
    for sym, nconv, npair in ((graphs.resnet_int8(*R50_SMALL.values()), 52, 4),
                       (attach_quantize_node(graphs.resnet(**R50_SMALL), shape_dict(graphs.resnet(**R50_SMALL), shape,
                                                                                     (2,)),
                                             QSET["weight"], QSET["act"], ("Convolution", "FullyConnected"),
                                             {"Convolution": 1, "FullyConnected": 1}), 52, 0)):
        for prec in ("float32", "bfloat16"):
            ex = _bind(sym, shape, precision=prec).executor
            convs = [op for op in ex.plan.ops if op.kind == "conv"]
            assert len(convs) == nconv and all(op.int8 for op in convs)
            names = _call_names(ex._fwd_train)
            # (rn_conv_fwd_i8_mm: + the per-block extremes of y the quantizers of bn(y) take their max from)
            nmm = names.count("rn_conv_fwd_i8_mm")
            assert names.count("rn_conv_fwd_i8") + nmm == nconv and (nmm > 0) == (prec == "bfloat16")
            assert all(op.mm_src is not None for op in ex.plan.ops if op.kind == "bn" and op.apply_in_quant
                       and op.part_src is not None and prec == "bfloat16")
            # only the stem and fc1 keep a fake-quant / float forward
            assert sum(1 for nm in names if nm.startswith("rn_conv_fwd") and not nm.startswith("rn_conv_fwd_i8")) <= 2
            assert _call_names(ex._fwd_infer).count("rn_conv_fwd_i8") == nconv  # (inference: no statistics)
            qops = [op for op in ex.plan.ops if op.kind == "quant"]
            # every conv's data quantizer emits codes (fc1's, in resnet_int8, does not)
            nbn, nbn2 = names.count("rn_quant_int8_fwd_codes_bn"), names.count("rn_quant_int8_fwd_codes_bn2")
            assert names.count("rn_quant_int8_fwd_codes") + nbn + 2 * nbn2 == sum(op.emit_codes for op in qops) \
                >= len(qops) - 1
            # quantizers of a BN+ReLU output nothing else reads apply that BN on load (one call for the
            # two quantizers of a stage's first unit); the BN output is not written
            assert nbn + nbn2 == sum(op.bn_src is not None for op in qops) > 0
            assert nbn2 == sum(op.bn_peer is not None for op in qops) == npair
            assert all(op.bn_src.apply_in_quant and op.bn_src.y is op.x for op in qops if op.bn_src is not None)
            # (no value expansion in the plan: round 4's opt-in deferred values were removed in round 5)
            assert "rn_quant_int8_expand" not in _call_names(ex._bwd)
            # every weight quantizer (+ the int8 convs' codes and data-gradient copies) in one batched call
            packs = _call_names(ex.packs)
            assert packs[0] == "rn_weight_quant_pack" and "rn_conv_weight_pack_i8" not in packs
            assert len(ex._wq_ops) >= nconv and sum(op.int8 for op in ex._wq_ops if op.kind == "conv") == nconv
    ex = _bind(graphs.resnet_int8(*R50_SMALL.values()), shape).executor
    assert "rn_quant_int8_expand" not in _call_names(ex._bwd)
    # default (bf16): the quantizers whose convs' weight gradients take codes (all but stage 1's act2, whose
    # conv2 runs the image-band kernel) write codes only (rn_conv_bwd_filter_i8, on the side stream)
    ex = _bind(graphs.resnet_int8(*R50_SMALL.values()), shape, precision="bfloat16").executor
    cw = [op for op in ex.plan.ops if op.kind == "quant" and op.codes_wgrad]
    bn = _call_names(ex._bwd)
    assert len(cw) == 49 and bn.count("rn_conv_bwd_filter_i8") == 49
    assert all(op.qsrc.codes_wgrad == (not (op.name.startswith("stage1") and op.name.endswith("conv2")))
               for op in ex.plan.ops if op.kind == "conv")
    assert "rn_conv_bwd_filter_i8" in ex.WGRAD_CALLS  # (routed to the side stream by name, _route_wgrads)
    # the stage-first units' act1 quantizer pairs: both clips folded into their BN's backward (rn_bn_desc.clip /
    # clip2 / dy2; the opt-in fold into the later data gradient, RN_QUANT_PAIR_FUSION, was removed in round 6)
    ex0 = _bind(graphs.resnet_int8(*R50_SMALL.values()), shape, precision="bfloat16").executor
    assert "rn_conv_bwd_data_bnred_clip2" not in _call_names(ex0._bwd)
    pairs = [op for op in ex0.plan.ops if op.kind == "bn" and op.qpair]
    assert len(pairs) == 4 and all(op.desc.dy2 for op in pairs)
    monkeypatch.setenv("RN_QUANT_CODES_WGRAD", "0")
    ex = _bind(graphs.resnet_int8(*R50_SMALL.values()), shape, precision="bfloat16").executor
    assert not any(op.codes_wgrad for op in ex.plan.ops if op.kind == "quant")
    assert "rn_conv_bwd_filter_i8" not in _call_names(ex._bwd)
    monkeypatch.delenv("RN_QUANT_CODES_WGRAD")
    monkeypatch.setenv("RN_INT8_MFMA", "0")
    ex = _bind(graphs.resnet_int8(*R50_SMALL.values()), shape).executor
    assert "rn_conv_fwd_i8" not in _call_names(ex._fwd_train)


# ----------------------------------------------------------------------------- oracle restatements
def test_oracle_attach_quant_equals_resnet_int8():
    """attach_quant with nothing skipped (8 bits) computes what resnet_int8's graph computes (same
    topology, a fake-quant node on every conv / fc input and weight)."""
    g_att = onet.attach_quant(onet.resnet([1, 1, 1, 1], 4, [8, 16, 16, 32, 32], 5))
    g_int8 = onet.resnet_int8([1, 1, 1, 1], 4, [8, 16, 16, 32, 32], 5)
    assert g_att.params == g_int8.params
    args, aux = onet.init_params(g_att)
    data, label = onet.synthetic_batch(2, (3, 32, 32), 5)
    p1, s1 = onet.forward(g_att, args, {k: v.copy() for k, v in aux.items()}, data, label, True, {}, True)
    p2, s2 = onet.forward(g_int8, args, {k: v.copy() for k, v in aux.items()}, data, label, True, {}, True)
    np.testing.assert_array_equal(p1, p2)
    g1 = onet.backward(g_att, args, s1)
    g2 = onet.backward(g_int8, args, s2)
    for k in g1:
        np.testing.assert_allclose(g1[k], g2[k], rtol=1e-12, atol=1e-14)


def test_oracle_bn_global_against_torch():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(3)
    x = rng.standard_normal((3, 5, 4, 4))
    dy = rng.standard_normal(x.shape)
    gamma, beta = rng.standard_normal(5), rng.standard_normal(5)
    mm, mv = rng.standard_normal(5) * 0.3, rng.uniform(0.5, 2, 5)
    for fix_gamma in (False, True):
        y, cache = ops.bn_global_fwd(x, gamma, beta, mm, mv, 1e-5, fix_gamma)
        dx, dg, db = ops.bn_global_bwd(dy, cache, fix_gamma)
        tx = torch.tensor(x, requires_grad=True)
        tg = torch.tensor(np.ones(5) if fix_gamma else gamma, requires_grad=True)
        tb = torch.tensor(beta, requires_grad=True)
        ty = torch.nn.functional.batch_norm(tx, torch.tensor(mm), torch.tensor(mv), tg, tb, training=False, eps=1e-5)
        ty.backward(torch.tensor(dy))
        np.testing.assert_allclose(y, ty.detach().numpy(), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(dx, tx.grad.numpy(), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(db, tb.grad.numpy(), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(dg, np.zeros(5) if fix_gamma else tg.grad.numpy(), rtol=1e-12, atol=1e-12)


def test_oracle_fix_bn_keeps_moving_stats():
    g = onet.fix_bn(onet.resnet20_cifar())
    args, aux = onet.init_params(g)
    aux = {k: v + 0.1 for k, v in aux.items()}
    before = {k: v.copy() for k, v in aux.items()}
    data, label = onet.synthetic_batch(2, (3, 32, 32), 10)
    onet.forward(g, args, aux, data, label, True)
    for k in aux:
        np.testing.assert_array_equal(aux[k], before[k])


def test_grouped_repacks_batched(dry, monkeypatch):
    """ResNeXt's grouped weights are repacked after every update (the SGD kernel writes only dense
    copies): one rn_conv_weight_pack_multi for all 16 grouped layers; RN_GPACK_BATCH=0 = one
    rn_conv_weight_pack each."""
    sym = graphs.resnext([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16, "float32", 32)
    ex = _bind(sym, precision="bfloat16").executor
    names = _call_names(ex.unfused_packs)  # + the stem's 4-channel copy (rn_stem_weight_pack_p4)
    assert names == ["rn_stem_weight_pack_p4", "rn_conv_weight_pack_multi"]
    descs = ex.unfused_packs[1][2][0]
    assert len(descs) == 16 and all(d.groups == 32 for d in descs)
    monkeypatch.setenv("RN_GPACK_BATCH", "0")
    ex0 = _bind(sym, precision="bfloat16").executor
    assert _call_names(ex0.unfused_packs) == ["rn_stem_weight_pack_p4"] + ["rn_conv_weight_pack"] * 16


def test_stem_backward_chunked(dry, monkeypatch):
    """The NHWC4 stem's BN backward: rn_bn_bwd reduces + finalizes only, then per image chunk the
    rows of dx (rn_bn_bwd_apply_rows) and that chunk's weight gradient (side stream), the chunks
    tiling the batch; RN_STEM_CHUNKS=1 = the single apply + wgrad."""
    sym = graphs.resnet(**R50_SMALL)
    ex = _bind(sym, shape=(8, 3, 64, 64), precision="bfloat16").executor
    names = _call_names(ex._bwd)
    i = names.index("rn_bn_bwd_apply_rows")
    # bn0's reduction done by the max-pool backward (rn_pool_bwd_bnred): finalize only, then the rows
    assert names[i - 1] == "rn_bn_bwd_finalize" and "rn_pool_bwd_bnred" in names[:i]
    monkeypatch.setenv("RN_BN_BWD_FUSION", "0")
    names0 = _call_names(_bind(sym, shape=(8, 3, 64, 64), precision="bfloat16").executor._bwd)
    i0 = names0.index("rn_bn_bwd_apply_rows")
    assert names0[i0 - 1] == "rn_bn_bwd" and "rn_pool_bwd_bnred" not in names0
    monkeypatch.delenv("RN_BN_BWD_FUSION")
    assert names[i:i + 8] == ["rn_bn_bwd_apply_rows", "rn_stem_conv_wgrad_p4"] * 4
    rows = [ex._bwd[i + 2 * j][2][8:10] for j in range(4)]
    m = ex._bwd[i - 1][2][0]._obj.m
    assert [r[0] for r in rows] == [j * m // 4 for j in range(4)] and all(r[1] == m // 4 for r in rows)
    assert sum(ex._bwd[i + 2 * j + 1][2][0]._obj.n for j in range(4)) == 8
    monkeypatch.setenv("RN_STEM_CHUNKS", "1")
    names1 = _call_names(_bind(sym, shape=(8, 3, 64, 64), precision="bfloat16").executor._bwd)
    assert "rn_bn_bwd_apply_rows" not in names1 and names1.count("rn_stem_conv_wgrad_p4") == 1


def test_int8_stem_backward_chunked(dry, monkeypatch):
    """The int8 stem (NHWC-8 image with the clip masks): the same per-chunk BN apply rows, each chunk's
    weight gradient over the real + mask channels (rn_stem_clip_wgrad_chunk: the first zeroes the
    extended gradient, the last adds the real part into dW), then the clip's dbeta after the shift grad."""
    sym = graphs.resnet_int8(*R50_SMALL.values())
    ex = _bind(sym, shape=(8, 3, 64, 64), precision="bfloat16").executor
    names = _call_names(ex._bwd)
    i = names.index("rn_bn_bwd_apply_rows")
    assert names[i:i + 8] == ["rn_bn_bwd_apply_rows", "rn_stem_clip_wgrad_chunk"] * 4
    flags = [tuple(ex._bwd[i + 2 * j + 1][2][7:9]) for j in range(4)]
    assert flags == [(1, 0), (0, 0), (0, 0), (0, 1)]
    assert sum(ex._bwd[i + 2 * j + 1][2][0]._obj.n for j in range(4)) == 8
    assert names.index("rn_stem_shift_grad") < names.index("rn_stem_clip_dbeta")
    assert "rn_stem_clip_wgrad" not in names
    monkeypatch.setenv("RN_STEM_CHUNKS", "1")
    names1 = _call_names(_bind(sym, shape=(8, 3, 64, 64), precision="bfloat16").executor._bwd)
    assert "rn_stem_clip_wgrad_chunk" not in names1 and names1.count("rn_stem_clip_wgrad") == 1
