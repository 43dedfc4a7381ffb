"""bf16 whole-step parity of the headline bench configuration (BASELINE C2: ResNet-50 v2 bf16).

The bench runs the executor's default knobs, and so does this test (no RN_* overrides): weight
gradients on a side stream, the step on a high-priority stream, persistent 224-row conv tiles,
BatchNorm statistics / BN-backward reductions in the conv epilogues, the NHWC4 stem, split-M slab
weight gradients. `tiles="wide"` additionally forces the 256-column tiles (rn_set_tuning 4 = 2) and
an 8-workgroup persistent grid (rn_set_tuning 10 = 8), so that at this small batch every eligible
layer runs the 224x256 tile family the 256-image bench uses, with its BN epilogues, and walks
several tiles per workgroup; `tiles="w4"` forces the 4-wave one-buffer 224x128 tile (rn_set_tuning
11 = 2) on every 1x1 pad-0 layer, which the bench's stage-1/2 layers run.

Reference: the numpy oracle in fp64 (symbol/resnet.py:77-121 restated) and its bf16-storage
emulation (oracle.net.forward storage='bf16': weights and every stored activation rounded to
bf16, fp64 arithmetic). A deep random-init ResNet at small spatial size is chaotic under rounding
(DESIGN.md 4): unreplayed, bf16 storage alone leaves gradients at cosine ~0.26 to fp64, and the
device must be no more chaotic than that. With the device's ReLU decisions replayed in both oracle
runs the gradients are well conditioned: over all 157 tensors (step_util.grad_summary) the
device's distance to fp64 must stay within 4x the bf16 emulation's own distance (with absolute
floors), probabilities and loss likewise, updated weights within the gradient bar.

Full size: one 224x224 / 256-image step checked through size-independent properties -- finite
outputs, BatchNorm moving statistics of channel subsets against a host recompute from the device's
own BN input tensors, and a loss that decreases over 3 SGD steps on the fixed batch.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import net as onet
from step_util import ce_loss, fro_rel, grad_summary, max_rel, module_step, oracle_state, oracle_step

pytestmark = pytest.mark.gpu


def _r50(ncls=16):
    from rn import graphs
    return graphs.resnet([3, 4, 6, 3], 4, [64, 256, 512, 1024, 2048], ncls)


def _prio_stream():
    lo, hi = torch.cuda.Stream.priority_range()
    return torch.cuda.Stream(priority=min(lo, hi))


@pytest.mark.parametrize("tiles", ["auto", "wide", "w4"])
def test_resnet50_bf16_step_gradients(gpu, tiles):
    from rn import lib as L
    lib = L.load()
    if tiles == "wide":
        L.check(lib.rn_set_tuning(4, 2), "tune")
        L.check(lib.rn_set_tuning(10, 8), "tune")
    if tiles == "w4":  # every 1x1 pad-0 layer on the 4-wave one-buffer tile, persistent over 16 workgroups
        L.check(lib.rn_set_tuning(11, 2), "tune")
        L.check(lib.rn_set_tuning(10, 8), "tune")
    try:
        g = onet.resnet50_imagenet(num_classes=16)
        args, aux = oracle_state(g)
        data, label = onet.synthetic_batch(2, (3, 112, 112), 16)
        with torch.cuda.stream(_prio_stream()):
            res = module_step(_r50(), args, aux, data, label, "bfloat16")
        torch.cuda.synchronize()
    finally:
        L.check(lib.rn_set_tuning(4, 0), "tune")
        L.check(lib.rn_set_tuning(10, 512), "tune")
        L.check(lib.rn_set_tuning(11, 0), "tune")
    masks = res["relu_masks"][0]
    # (1) unreplayed: at 2 images of 112x112 a random-init ResNet-50 is chaotic under ANY rounding
    # (thousands of ReLU decisions flip; measured: the bf16 emulation's own gradients have cosine
    # ~0.26 to fp64). The device must be exactly as chaotic as bf16 storage is, no more.
    ref = oracle_step(g, args, aux, data, label)
    emu = oracle_step(g, args, aux, data, label, storage="bf16")
    raw_dev = grad_summary(res["grads"][0], ref["grads"][0])
    raw_emu = grad_summary(emu["grads"][0], ref["grads"][0])
    # (2) replayed: the same ReLU decisions in all three (the device's, step_util.gpu_relu_masks),
    # then the gradients are well conditioned and the device must match the fp64 oracle within a
    # small factor of what bf16 storage alone costs
    ref_m = oracle_step(g, args, aux, data, label, relu_masks=masks)
    emu_m = oracle_step(g, args, aux, data, label, storage="bf16", relu_masks=masks)
    s_dev = grad_summary(res["grads"][0], ref_m["grads"][0])
    s_emu = grad_summary(emu_m["grads"][0], ref_m["grads"][0])
    p_dev = max_rel(res["prob"][0], ref_m["prob"][0])
    p_emu = max_rel(emu_m["prob"][0], ref_m["prob"][0])
    print("unreplayed  device vs fp64:", raw_dev, " bf16 emulation vs fp64:", raw_emu)
    print("replayed    device vs fp64:", s_dev, "prob", p_dev, " bf16 emulation vs fp64:", s_emu, "prob", p_emu)
    # measured (r02): even replayed, bf16 storage moves this ill-conditioned network's gradients by
    # ~46 % per tensor (BN backward over 32 elements per channel at stage 4 cancels heavily): both
    # bars say "the device is as accurate as ideal bf16 storage", not an absolute accuracy
    assert raw_dev["median"] < 1.5 * raw_emu["median"] + 0.1, (raw_dev, raw_emu)
    assert 1 - s_dev["cos"] < 1.5 * (1 - s_emu["cos"]) + 0.01, (s_dev, s_emu)
    for k in ("fro", "median", "p95"):
        assert s_dev[k] < 1.5 * s_emu[k] + 0.02, (k, s_dev, s_emu)
    assert p_dev < 2 * p_emu + 0.02, (p_dev, p_emu)


def test_resnet50_bf16_full_size_gradients(gpu):
    """The exact bench configuration -- 256 images at 224x224, no tuning override -- against the
    torch-CPU fp32 restatement of the same step (oracle/torch_cpu.py, itself pinned to the numpy
    oracle) and its bf16-storage emulation. At this Xavier init the network is chaotic under ANY
    bf16 rounding (the emulation's own forward error grows ~1.17x per
    BatchNorm+ReLU layer, 0.2 % at the stem to 25 % at stage 4; measured r03, profiles/r03/
    bf16_full_size_gradients.log: emulation vs fp32 cosine 0.297, device vs fp32 cosine 0.298), so
    end to end the bar is relative: the device no further from fp32 than ideal bf16 storage (+10 %).
    The absolute per-layer bars are test_resnet50_bf16_full_size_layerwise below."""
    from oracle import torch_cpu
    g = onet.resnet50_imagenet()
    args, aux = onet.init_params(g, dtype=np.float32)
    data, label = onet.synthetic_batch(256, (3, 224, 224), 1000, dtype=np.float32)
    from rn import graphs
    with torch.cuda.stream(_prio_stream()):
        res = module_step(graphs.resnet50(), args, aux, data, label, "bfloat16")
    torch.cuda.synchronize()
    del res["mod"]
    torch.cuda.empty_cache()
    grads, prob = torch_cpu.TorchStep(g, args, aux).grads(data, label)
    egrads, eprob = torch_cpu.TorchStep(g, args, aux, storage="bf16").grads(data, label)
    s = grad_summary(res["grads"][0], grads)
    se = grad_summary(egrads, grads)
    sde = grad_summary(res["grads"][0], egrads)
    p, pe = max_rel(res["prob"][0], prob), max_rel(eprob, prob)
    print("bench config vs torch-CPU fp32:", s, "prob", p)
    print("torch-CPU bf16-storage emulation vs fp32:", se, "prob", pe)
    print("bench config vs the bf16-storage emulation:", sde, "prob", max_rel(res["prob"][0], eprob))
    assert 1 - s["cos"] < 1.1 * (1 - se["cos"]) + 0.01, (s, se)
    for k in ("fro", "median", "p95"):
        assert s[k] < 1.1 * se[k] + 0.01, (k, s, se)
    assert p < 1.25 * pe + 0.01, (p, pe)
    assert abs(ce_loss(res["prob"][0], label) - ce_loss(prob, label)) < 0.01 * ce_loss(prob, label)


def _layerwise(sym, n, image, precision, tune=None, warm=0):
    """One training step (forward + backward, serialised on one stream) with every kernel checked
    against its fp32 torch restatement from the device's own inputs (tests/layerwise.py). warm: full
    steps (forward, backward, SGD update + the weight repacks after it) run before the checked one, so
    the checked forward reads weights the post-update packs wrote and quantizer states that follow
    the EMA."""
    import json
    import os
    import mxnet as mx
    from layerwise import Checker
    from rn import lib as L
    lib = L.load()
    for k, v in (tune or {}).items():
        L.check(lib.rn_set_tuning(k, v), "tune")
    try:
        rng = np.random.default_rng(0)
        data = rng.uniform(-1, 1, (n, 3, image, image)).astype(np.float32)
        label = np.random.default_rng(1).integers(0, 1000, n).astype(np.float32)
        mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision=precision)
        mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", (n,))])
        mx.random.seed(2)
        mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
        mod.init_optimizer(kvstore="device", optimizer="sgd",
                           optimizer_params={"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9})
        ex = mod.executor
        ex.side_enabled = False  # the checks read buffers between calls: one stream, in plan order
        batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
        for _ in range(warm):
            mod.forward(batch, is_train=True)
            mod.backward()
            mod.update()
        torch.cuda.synchronize()
        prev_aux = {nm: ex.aview(nm).clone() for nm in ex.aux_off if nm.endswith("minmax")}
        first = bool(ex._qfirst.value)
        mod.forward(batch, is_train=True)
        torch.cuda.synchronize()
        ck = Checker(ex, prev_aux=prev_aux, first_batch=first)
        with torch.no_grad():
            ck.check_forward()
            ex.backward(hooks=ck.backward_hooks())
        torch.cuda.synchronize()
    finally:
        for k in (tune or {}):
            L.check(lib.rn_set_tuning(k, 512 if k == 10 else 0), "tune")
    tab = ck.table()
    for kind, e in sorted(tab.items()):
        print("%-16s %4d checked, worst: %s" % (kind, e["n"], ", ".join(
            "%s %.2e (%s)" % (k, v[0], v[1]) for k, v in sorted(e.items()) if k != "n")))
    print("backward calls checked:", ck.covered, "not checked:", ck.skipped)
    out = os.environ.get("RN_LAYERWISE_OUT")
    if out:
        with open(out, "w") as f:
            json.dump({"config": [n, image, precision], "records": ck.rec, "covered": ck.covered,
                       "skipped": ck.skipped}, f)
    return ck


def test_resnet50_bf16_full_size_layerwise(gpu):
    """The bench configuration (ResNet-50 v2, 256 x 224 x 224, bf16, default knobs) with ABSOLUTE
    bars per kernel: every one of the step's 53 convolutions forward / data gradient / weight gradient,
    51 BatchNorms forward (statistics, coefficients, stored outputs) and backward (dx, dgamma, dbeta),
    the stem's bn_data transform, pooling, FullyConnected, SoftmaxOutput and the gradient fan-in adds,
    each recomputed in fp32 from the device's own inputs: bf16 outputs within one bf16 rounding (Frobenius
    4e-3, max 8e-3 of the tensor's max), fp32 weight gradients within 2e-6 of the magnitude sum of their
    terms per element (layerwise.WGRAD_BAR), BatchNorm statistics within 1e-5. Every call of the backward
    plan is checked. Measured numbers: profiles/r03/layerwise_bf16.log."""
    from rn import graphs
    ck = _layerwise(graphs.resnet50(), 256, 224, "bfloat16")
    assert not ck.skipped, ck.skipped
    kinds = {r[0] for r in ck.rec}
    assert {"conv_fwd", "dgrad", "dgrad_bnred", "wgrad", "bn_fwd", "bn_bwd_dx", "bn_bwd_params", "stem_prepare",
            "pool_fwd", "pool_bwd", "fc_fwd", "softmax", "softmax_grad", "bn_apply", "fc_bias_grad", "stem_dbeta"} <= kinds, kinds
    assert sum(1 for r in ck.rec if r[0] == "wgrad") == 54  # 53 convs + fc1
    assert sum(1 for r in ck.rec if r[0] == "conv_fwd") == 53
    bad = ck.failures()
    assert not bad, bad[:10]


def test_resnext50_bf16_full_size_layerwise(gpu):
    """BASELINE C4 at its bench configuration (ResNeXt-50 32x4d, 256 x 224 x 224, bf16, default knobs),
    with the same absolute per-kernel bars as C2, after one full step (so the grouped weights' compute
    copies are the ones rn_conv_weight_pack_multi rewrites after an update): every grouped 3x3
    convolution (the direct v_dot2 kernels at 4 channels per group and at 8 per group with stride 2,
    the block-diagonal MFMA tiles elsewhere) forward / data gradient / weight gradient against the
    bf16-rounded master per group, the post-activation unit tail (rn_bn_apply_add) and its backward
    (rn_relu_bwd_bnred, then rn_bn_bwd_part), every dense layer and BatchNorm as in C2
    (symbol/resnext.py:17-47)."""
    _c4_layerwise(256, 224)


def _c4_layerwise(n, image):
    from rn import graphs
    ck = _layerwise(graphs.resnext50_32x4d(), n, image, "bfloat16", warm=1)
    assert not ck.skipped, ck.skipped
    kinds = {r[0] for r in ck.rec}
    # (the grouped data gradients carry their BN-backward reduction: direct kernel or block-diagonal tile)
    # (every unit tail's backward in rn_relu_bwd_bnred)
    assert {"conv_fwd", "conv_fwd_grouped", "dgrad_bnred_grouped", "wgrad_grouped", "wgrad", "bn_apply_add",
            "relu_bwd_bnred", "bn_fwd", "bn_bwd_dx", "bn_bwd_params", "weight_copy"} <= kinds, kinds
    assert sum(1 for r in ck.rec if r[0] == "relu_bwd_bnred") == 16
    assert sum(1 for r in ck.rec if r[0] == "conv_fwd_grouped") == 16
    assert sum(1 for r in ck.rec if r[0] in ("dgrad_grouped", "dgrad_bnred_grouped")) == 16
    assert sum(1 for r in ck.rec if r[0] in ("wgrad", "wgrad_grouped")) == 54  # 53 convs + fc1
    assert sum(1 for r in ck.rec if r[0] == "bn_apply_add") == 16
    bad = ck.failures()
    assert not bad, bad[:10]


def test_resnet50_int8_full_size_layerwise(gpu):
    """BASELINE C5 at its bench configuration (symbol/resnet_int8.py, 256 x 224 x 224, int8 forward /
    bf16 backward, default knobs), after one full step (the batched weight quantizer's repack after an
    update, quantizer EMA states): every activation quantizer -- BatchNorm+ReLU applied on load, the
    pairs, the block-extreme max from rn_conv_fwd_i8_mm -- bit for bit (state, unit, int8 codes,
    fake-quantized values); every weight quantizer bit for bit (threshold, unit, codes, fake-quantized
    fp32 and bf16 CRSK copies); every int8 convolution against the exact fp64 sum of the device's codes
    times its units (BF16 bar); the folded straight-through clips in the BatchNorm backwards
    (rn_conv_bwd_data_bnred_clip, rn_bn_desc.clip / clip2 / dy2), the FullyConnected input's STE and
    the stem's clip gradient (symbol/int8_api.py:120-171, clip_grad_quantization_int8.py:37-67)."""
    _c5_layerwise(256, 224)


def _c5_layerwise(n, image):
    from rn import graphs
    ck = _layerwise(graphs.resnet50_int8(), n, image, "bfloat16", warm=1)
    assert not ck.skipped, ck.skipped
    kinds = {r[0] for r in ck.rec}
    assert {"conv_fwd_i8", "quant", "weight_quant", "dgrad_bnred", "bn_bwd_dx", "bn_bwd_params", "wgrad",
            "quant_bwd", "stem_dbeta", "fc_fwd"} <= kinds, kinds
    n_i8 = sum(1 for r in ck.rec if r[0] == "conv_fwd_i8")
    assert n_i8 == 52, n_i8
    assert sum(1 for r in ck.rec if r[0] == "weight_quant") == 54  # 53 convs + fc1
    assert sum(1 for r in ck.rec if r[0] == "quant") == 54  # 52 int8 inputs + conv0's + fc1's
    assert sum(1 for r in ck.rec if r[0] == "quant_expand") == 0
    # (default: the quantizers but stage 1's act2 write codes only and their weight gradients multiply
    # the codes, rn_conv_bwd_filter_i8)
    n_cw = sum(1 for op in ck.ex.plan.ops if op.kind == "quant" and op.codes_wgrad)
    assert n_cw == 49, n_cw
    assert ck.covered.get("rn_conv_bwd_filter_i8", 0) == 49  # one per quantizer
    assert sum(1 for r in ck.rec if r[0] == "wgrad") == 54
    bad = ck.failures()
    assert not bad, bad[:10]
    return ck


def test_resnext50_bf16_layerwise_small(gpu):
    """The C4 per-kernel checks at 8 images of 64x64 (a fast first gate before the full size)."""
    _c4_layerwise(8, 64)


def test_resnet50_int8_layerwise_small(gpu):
    """The C5 per-kernel checks at 8 images of 64x64 (a fast first gate before the full size)."""
    _c5_layerwise(8, 64)


def test_resnet50_fp32_layerwise(gpu):
    """The same per-kernel checks on the fp32 parity path (exact fp32 MFMA), small batch: validates
    the checker itself at fp32 bars and covers the fp32 kernels layer by layer."""
    from rn import graphs
    ck = _layerwise(graphs.resnet50(), 4, 64, "float32")
    assert not ck.skipped, ck.skipped
    bad = ck.failures()
    assert not bad, bad[:10]


def test_resnet50_bf16_full_size_properties(gpu):
    import mxnet as mx
    from rn import graphs
    sym = graphs.resnet50()
    n = 256
    rng = np.random.default_rng(0)
    data = rng.uniform(-1, 1, (n, 3, 224, 224)).astype(np.float32)
    label = np.random.default_rng(1).integers(0, 1000, n).astype(np.float32)
    mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision="bfloat16")
    mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", (n,))])
    mx.random.seed(2)
    mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
    mod.init_optimizer(kvstore="device", optimizer="sgd",
                       optimizer_params={"learning_rate": 0.05, "wd": 1e-4, "momentum": 0.9})
    ex = mod.executor
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    check = ["bn0", "stage1_unit1_bn2", "stage1_unit2_bn1", "stage2_unit1_bn3", "stage3_unit4_bn2", "bn1"]
    bn_ops = {op.name: op for op in ex.plan.ops if op.kind == "bn"}
    losses = []
    stream = _prio_stream()
    for step in range(3):
        with torch.cuda.stream(stream):
            mod.forward(batch, is_train=True)
        torch.cuda.synchronize()
        prob = mod.get_outputs()[0].asnumpy()
        assert np.isfinite(prob).all()
        losses.append(ce_loss(prob, label))
        if step == 0:
            # moving stats after one step from (0, 1): 0.1 * batch mean, 0.9 + 0.1 * biased batch var,
            # recomputed here from the device's own (stored, bf16) BN input
            for name in check:
                op = bn_ops[name]
                x = op.x
                xs = ex.act(x).view(x.rows, x.cp)[:, :8].float().cpu().numpy().astype(np.float64)
                mean, var = xs.mean(0), xs.var(0)
                mm = ex.get_aux(op.mean)[:8]
                mv = ex.get_aux(op.var)[:8]
                sd = np.sqrt(var) + 1e-6
                assert np.all(np.abs(mm - 0.1 * mean) <= 1e-4 * 0.1 * sd + 1e-7), (name, mm, 0.1 * mean)
                assert np.allclose(mv, 0.9 + 0.1 * var, rtol=1e-4, atol=1e-6), (name, mv, 0.9 + 0.1 * var)
        with torch.cuda.stream(stream):
            mod.backward()
            mod.update()
        torch.cuda.synchronize()
    for nm in ("conv0_weight", "stage2_unit1_conv2_weight", "fc1_weight", "bn1_gamma"):
        assert np.isfinite(ex.get_param(nm)).all(), nm
    assert losses[2] < losses[0], losses
