"""CPU tests of the mx.sym IR, the graph builders, lowering (Plan) and a dry-run executor build."""
import json

import numpy as np
import pytest

import mxnet as mx
from rn import graphs
from rn.executor import Executor, Plan, PlanError


def _nparams(sym, shape):
    args = sym.list_arguments()
    a, o, x = sym.infer_shape(data=shape, softmax_label=(shape[0],))
    sizes = {n: int(np.prod(s)) for n, s in zip(args, a) if n not in ("data", "softmax_label")}
    return len(sizes), sum(sizes.values()), o


def test_param_counts_match_survey():
    # SURVEY.md 8a rows A4-A6
    assert _nparams(graphs.resnet50(), (2, 3, 224, 224))[:2] == (157, 25549486)
    assert _nparams(graphs.resnext50_32x4d(), (2, 3, 224, 224))[:2] == (161, 25028904)
    assert _nparams(graphs.resnet20_cifar(), (2, 3, 32, 32))[:2] == (65, 272474)
    assert len(graphs.resnet50().list_auxiliary_states()) == 102


def test_names_and_order_match_oracle():
    from oracle import net as onet
    sym = graphs.resnet50()
    args = [n for n in sym.list_arguments() if n not in ("data", "softmax_label")]
    assert args == list(onet.resnet50_imagenet().params)
    sym = graphs.resnet20_cifar()
    args = [n for n in sym.list_arguments() if n not in ("data", "softmax_label")]
    assert args == list(onet.resnet20_cifar().params)


def test_infer_shape_and_internals():
    sym = graphs.resnet50()
    internals = sym.get_internals()
    _, outs, _ = internals.infer_shape(data=(2, 3, 224, 224), softmax_label=(2,))
    shapes = dict(zip(internals.list_outputs(), outs))
    assert shapes["conv0_output"] == (2, 64, 112, 112)
    # auto-named like MXNet's NameManager (global counter): pooling<i>
    assert any(k.startswith("pooling") and v == (2, 64, 56, 56) for k, v in shapes.items())
    assert shapes["stage4_unit3_conv3_output"] == (2, 2048, 7, 7)
    assert shapes["fc1_output"] == (2, 1000)


def test_json_roundtrip():
    sym = graphs.resnet20_cifar()
    js = sym.tojson()
    d = json.loads(js)
    assert d["nodes"][d["heads"][0][0]]["op"] == "SoftmaxOutput"
    sym2 = mx.sym.load_json(js)
    assert sym2.list_arguments() == sym.list_arguments()
    assert sym2.list_auxiliary_states() == sym.list_auxiliary_states()
    a1 = sym.infer_shape(data=(4, 3, 32, 32), softmax_label=(4,))
    a2 = sym2.infer_shape(data=(4, 3, 32, 32), softmax_label=(4,))
    assert a1 == a2


def test_auto_names_and_attrs():
    x = mx.sym.Variable("data")
    c = mx.sym.Convolution(data=x, num_filter=8, kernel=(3, 3), pad=(1, 1), no_bias=True, name="c1")
    assert c.list_arguments() == ["data", "c1_weight"]
    b = mx.sym.BatchNorm(data=c, fix_gamma=False, name="b1")
    assert b.list_auxiliary_states() == ["b1_moving_mean", "b1_moving_var"]
    s = c + b
    s._set_attr(mirror_stage="True")
    assert s.attr("mirror_stage") == "True"
    q = mx.sym.contrib.Quantization_int8(data=x, name="q", is_weight=False)
    assert q.list_auxiliary_states() == ["q_minmax"]


def test_plan_fusion_and_flops():
    p = Plan(graphs.resnet50(), [("data", (256, 3, 224, 224))], [("softmax_label", (256,))])
    assert p.summary() == {"stem": 1, "bn": 50, "pool": 2, "conv": 52, "fc": 1, "softmax": 1}
    # 16 residual adds are all fused into conv epilogues
    assert sum(1 for op in p.ops if op.kind == "conv" and op.res is not None) == 16
    # 6,220.6 GFLOP per 256-image step
    assert abs(p.train_flops() / 1e9 - 6220.6) < 0.1
    p20 = Plan(graphs.resnet20_cifar(), [("data", (128, 3, 32, 32))], [("softmax_label", (128,))])
    assert abs(p20.train_flops() / 1e9 - 31.2) < 0.05


def test_plan_resnext_grouped():
    p = Plan(graphs.resnext50_32x4d(), [("data", (256, 3, 224, 224))], [("softmax_label", (256,))])
    assert sum(1 for op in p.ops if op.kind == "conv" and op.groups == 32) == 16
    # 6,437.6 GFLOP per 256-image step
    assert abs(p.train_flops() / 1e9 - 6437.6) < 0.1
    ex = Executor(Plan(graphs.resnext50_32x4d(), [("data", (2, 3, 64, 64))], [("softmax_label", (2,))]), "cpu")
    names = [c[0] for c in ex._bwd]
    # 52 conv + fc1 weight gradients, and the stem's (the padded-NHWC4 kernel in bf16)
    assert sum(n.startswith("rn_conv_bwd_filter") or n == "rn_stem_conv_wgrad_p4" for n in names) == 54


def test_plan_rejects_unsupported():
    x = mx.sym.Variable("data")
    c = mx.sym.Convolution(data=x, num_filter=8, kernel=(3, 3), dilate=(2, 2), no_bias=True, name="c")
    sym = mx.sym.SoftmaxOutput(data=mx.sym.FullyConnected(data=c, num_hidden=4, name="fc"), name="softmax")
    with pytest.raises(PlanError):
        Plan(sym, [("data", (2, 8, 16, 16))], [("softmax_label", (2,))])


@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_executor_dry_run(dtype):
    sym = graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], 16)
    p = Plan(sym, [("data", (2, 3, 64, 64))], [("softmax_label", (2,))], dtype=dtype)
    ex = Executor(p, "cpu")
    names = [c[0] for c in ex._bwd]
    # the stem's weight gradient runs on the padded-NHWC4 kernel in bf16
    assert sum(n.startswith("rn_conv_bwd_filter") for n in names) == (54 if dtype == "float32" else 53)
    assert names.count("rn_stem_conv_wgrad_p4") == (0 if dtype == "float32" else 1)
    assert sum(n.startswith("rn_conv_bwd_data") for n in names) == 53
    # BN-backward reductions fused where the dgrad runs the 256-row tile (bf16 only)
    # (the 224-row tiles' dgrads)
    assert names.count("rn_conv_bwd_data_bnred") == (0 if dtype == "float32" else 41)
    assert names.count("rn_stem_shift_grad") == 1
    # every parameter's gradient has a producing call, buckets cover the flat buffer in order
    assert set(ex.param_done_at) == set(p.param_names)
    b = ex.buckets()
    assert b[0][0] == 0 and b[-1][1] == ex.nparam
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    assert all(b[i][2] <= b[i + 1][2] for i in range(len(b) - 1))
    # parameter I/O round trip (OIHW <-> KRSC)
    w = np.random.default_rng(0).standard_normal((64, 256, 1, 1)).astype(np.float32)
    ex.set_param("stage2_unit1_conv1_weight", np.random.default_rng(1).standard_normal((128, 256, 1, 1)))
    w3 = np.random.default_rng(2).standard_normal((128, 128, 3, 3)).astype(np.float32)
    ex.set_param("stage2_unit1_conv2_weight", w3)
    np.testing.assert_array_equal(ex.get_param("stage2_unit1_conv2_weight"), w3)


def test_plan_int8_quantization(monkeypatch):
    """resnet_int8 (symbol/resnet_int8.py): 108 Quantization_int8 nodes -> 54 weight
    quantizations folded into the weight packs, 53 activation quant ops, 1 folded into the stem."""
    sym = graphs.resnet50_int8()
    aux = sym.list_auxiliary_states()
    assert len(aux) == 210 and sum(a.endswith("_minmax") for a in aux) == 108
    p = Plan(sym, [("data", (256, 3, 224, 224))], [("softmax_label", (256,))])
    assert p.summary() == {"stem": 1, "bn": 50, "pool": 2, "quant": 53, "conv": 52, "fc": 1, "softmax": 1}
    assert sum(1 for op in p.ops if getattr(op, "qweight", None)) == 54
    assert [op for op in p.ops if op.kind == "stem"][0].quant["minmax"] == "conv0_data_minmax"
    assert abs(p.train_flops() / 1e9 - 6220.6) < 0.1
    ex = Executor(Plan(graphs.resnet_int8([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16),
                       [("data", (2, 3, 64, 64))], [("softmax_label", (2,))]), "cpu")
    names = [c[0] for c in ex._bwd]
    # 16 of the 17 activation quantizers read a BN+ReLU output only quantizers read -- one (8 BNs) or
    # two (the 4 units' act1: conv1 and the shortcut): their straight-through backwards fold into that
    # BN's backward (rn_bn_desc.clip, + clip2 / dy2); fc1's stays. RN_QUANT_BWD_FOLD=0 keeps all 17
    assert names.count("rn_quant_int8_bwd") == 1 and names.count("rn_stem_quant_clip_grad") == 0
    # the stem input quantizer's clip gradient rides in the stem's weight gradient (bf16): the masks
    # first (side stream), the mask channels' weight gradient, its dot product after the shift gradient
    assert names[0] == "rn_stem_clip_mask" and names.count("rn_stem_clip_wgrad") == 1
    assert names.index("rn_stem_shift_grad") < names.index("rn_stem_clip_dbeta")
    monkeypatch.setenv("RN_STEM_CLIP_MASK", "0")
    n0 = [c[0] for c in Executor(Plan(graphs.resnet_int8([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16),
                                      [("data", (2, 3, 64, 64))], [("softmax_label", (2,))]), "cpu")._bwd]
    assert n0.count("rn_stem_quant_clip_grad") == 1 and "rn_stem_clip_mask" not in n0
    monkeypatch.delenv("RN_STEM_CLIP_MASK")
    assert sum(1 for op in ex.plan.ops if op.kind == "bn" and op.desc.clip) == 12
    assert sum(1 for op in ex.plan.ops if op.kind == "bn" and op.desc.dy2 and op.desc.clip2) == 4
    monkeypatch.setenv("RN_QUANT_BWD_FOLD", "0")
    ex = Executor(Plan(graphs.resnet_int8([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16),
                       [("data", (2, 3, 64, 64))], [("softmax_label", (2,))]), "cpu")
    assert [c[0] for c in ex._bwd].count("rn_quant_int8_bwd") == 17
    packs = [c[0] for c in ex.packs]
    # (one batched rn_weight_quant_pack by default; RN_WQUANT_BATCH=0: per weight, counted here)
    assert packs == ["rn_weight_quant_pack"] + packs[1:] and "rn_quant_int8_fwd" not in packs
    monkeypatch.setenv("RN_WQUANT_BATCH", "0")
    ex = Executor(Plan(graphs.resnet_int8([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16),
                       [("data", (2, 3, 64, 64))], [("softmax_label", (2,))]), "cpu")
    packs = [c[0] for c in ex.packs]
    # the 16 non-stem convs' weight quantizers also keep the unit of their int8 codes (int8 forward)
    assert packs.count("rn_quant_int8_fwd") + packs.count("rn_quant_int8_fwd_codes") == 18
    assert packs.count("rn_conv_weight_pack_i8") == 16


def test_plan_bn_apply_fusion_opt_in(monkeypatch):
    """RN_BN_APPLY_FUSION=1: BN+ReLU outputs read only by 1x1 convs or poolings are applied on load."""
    monkeypatch.setenv("RN_BN_APPLY_FUSION", "1")
    p = Plan(graphs.resnet50(), [("data", (2, 3, 224, 224))], [("softmax_label", (2,))])
    fused = [op for op in p.ops if op.kind == "bn" and op.apply_fused]
    # bn1 of every unit (-> conv1, and sc in unit 1) and bn3 (-> conv3), bn0 (-> the stem's max pool) and
    # the final bn1 (-> the global pool); not bn2 (3x3)
    assert len(fused) == 34
    assert all(getattr(op, "xf", None) is not None for op in p.ops if op.kind == "conv" and op.kernel == (1, 1))
    assert all(op.xf is not None and op.xf.apply_fused for op in p.ops if op.kind == "pool")
    monkeypatch.setenv("RN_POOL_XF", "0")
    p = Plan(graphs.resnet50(), [("data", (2, 3, 224, 224))], [("softmax_label", (2,))])
    assert sum(1 for op in p.ops if op.kind == "bn" and op.apply_fused) == 32
    assert all(op.xf is None for op in p.ops if op.kind == "pool")
    monkeypatch.delenv("RN_POOL_XF")
    monkeypatch.setenv("RN_BN_APPLY_FUSION", "0")
    p = Plan(graphs.resnet50(), [("data", (2, 3, 224, 224))], [("softmax_label", (2,))])
    assert not any(op.apply_fused for op in p.ops if op.kind == "bn")


def test_plan_bn_bwd_fusion_default(monkeypatch):
    """RN_BN_BWD_FUSION: the BN backward reduction rides in the dgrad epilogue that completes the
    BN's output gradient -- by default (1) where that dgrad runs the 256-row tile (41 of 50 here),
    with 2 on every eligible dgrad (48: bn0 and the final bn1 get theirs from pooling), 0 never; bn0's
    rides in the stem max-pool's backward (rn_pool_bwd_bnred) unless 0."""
    def counts():
        ex = Executor(Plan(graphs.resnet50(), [("data", (2, 3, 64, 64))], [("softmax_label", (2,))]), "cpu")
        names = [c[0] for c in ex._bwd]
        return names.count("rn_conv_bwd_data_bnred"), names.count("rn_bn_bwd_part"), names.count("rn_bn_bwd")
    monkeypatch.delenv("RN_BN_BWD_FUSION", raising=False)
    assert counts() == (41, 42, 8)
    monkeypatch.setenv("RN_BN_BWD_FUSION", "2")
    assert counts() == (48, 49, 1)
    monkeypatch.setenv("RN_BN_BWD_FUSION", "0")
    assert counts() == (0, 0, 50)


def _live_tensors(ex):
    """Every torch tensor the executor (or its plan's ops) keeps a reference to."""
    import torch
    seen, out = set(), []

    def walk(o, depth=0):
        if depth > 4 or id(o) in seen:
            return
        seen.add(id(o))
        if isinstance(o, torch.Tensor):
            out.append(o)
        elif isinstance(o, dict):
            for v in o.values():
                walk(v, depth + 1)
        elif isinstance(o, (list, tuple)):
            for v in o:
                walk(v, depth + 1)
    for v in vars(ex).values():
        walk(v)
    for op in ex.plan.ops:
        for v in vars(op).values():
            walk(v)
    return out


@pytest.mark.parametrize("graph", ["resnet20", "resnext", "resnet_int8"])
def test_bound_pointers_are_owned(graph):
    """Every device pointer a bound call carries lies inside a tensor the executor keeps alive
    (a dropped temporary is recycled by the caching allocator while the plan still writes it)."""
    import ctypes as C
    sym, shp = {
        "resnet20": (graphs.resnet20_cifar(), (4, 3, 32, 32)),
        "resnext": (graphs.resnext([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16, "float32", 32), (2, 3, 64, 64)),
        "resnet_int8": (graphs.resnet_int8([1, 1, 1, 1], 4, [64, 256, 512, 1024, 2048], 16), (2, 3, 64, 64)),
    }[graph]
    ex = Executor(Plan(sym, [("data", shp)], [("softmax_label", (shp[0],))]), "cpu")
    spans = sorted((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for t in _live_tensors(ex))
    starts = [s for s, _ in spans]
    import bisect
    lists = [ex._fwd_train, ex._fwd_infer, ex._bwd, ex.wpack_calls, getattr(ex, "unfused_packs", [])]
    n = 0
    for lst in lists:
        for name, fn, args in lst:
            for a in args:
                if isinstance(a, C.c_void_p) and a.value and a is not ex._spv:
                    i = bisect.bisect_right(starts, a.value) - 1
                    assert i >= 0 and a.value < spans[i][1], (name, hex(a.value))
                    n += 1
    assert n > 100


def test_plan_bn_epilogue_stats_every_conv(monkeypatch):
    """RN_BN_EPILOGUE_STATS=2 (statistics in every producing conv's epilogue) binds: producers that are
    not convolutions (the stem, pooling, residual adds) keep the separate statistics pass."""
    monkeypatch.setenv("RN_BN_EPILOGUE_STATS", "2")
    ex = Executor(Plan(graphs.resnet50(), [("data", (2, 3, 64, 64))], [("softmax_label", (2,))]), "cpu")
    names = [c[0] for c in ex._fwd_train]
    assert names.count("rn_bn_fwd_train_part") > 0 and names.count("rn_bn_fwd_train") > 0


def test_bench_family_names():
    """bench.py names the conv kernel family of each call from the library's own tile choice: the
    ResNet-50 bench step uses the 224-row 256 / 128-column families and the 256x64 tile."""
    import bench
    ex = Executor(Plan(graphs.resnet50(), [("data", (256, 3, 224, 224))], [("softmax_label", (256,))]), "cpu")
    fams = {bench.family_of(ex, n, a) for n, f, a in ex._fwd_train + ex._bwd} - {None}
    assert "igemm_big_kernel<224x256>" in fams and "igemm_big_kernel<224x128>" in fams
    assert all(not f.startswith("igemm_big_kernel<448") for f in fams), fams
