"""Lower an mx.sym graph onto librn and run training steps on one MI355X.

This replaces what MXNet's Module/executor did under core/solver.py (bind :75,
forward :115, backward :116, update :121): shape inference, buffer allocation, op dispatch,
gradient fan-in accumulation (req='add') and the optimizer step -- all as a static plan of
C-ABI calls on one HIP stream.

Planning (`Plan`) is pure Python and runs without a GPU (it is what the CPU tests check).
`Executor` allocates device memory through PyTorch (plumbing only) and turns the plan into
lists of bound C calls. Every compute op is a librn kernel; there is no fallback path.

Layout: activations NHWC, channel stride padded to a multiple of 8, dtype bf16 (default) or
fp32 (`dtype='float32'`, exact-fp32 MFMA path used for parity). Parameters live in ONE flat
fp32 master buffer (conv / FC weights in KRSC), ordered in reverse forward order so that
gradient buckets complete front-to-back during backward (RCCL bucketing, rn/dist.py).
"""
import math
import os

import numpy as np

from . import lib as L

F32, BF16 = L.RN_F32, L.RN_BF16


def _pad8(c):
    return (c + 7) // 8 * 8


def _parse(v, default=None):
    from mxnet.symbol import _parse as p  # the shim's attr parser
    return p(v) if v is not None else default


def _tup(v, n=2):
    from mxnet.symbol import _tup as t
    return t(v, n)


class PlanError(RuntimeError):
    pass


# ============================================================================= plan (CPU)
class TensorSpec:
    """An activation tensor: logical NCHW (or (N,F)) shape -> NHWC buffer with padded C."""

    def __init__(self, name, shape, dtype, needs_grad=True, kind="act"):
        self.name = name
        self.shape = tuple(shape)
        if len(shape) == 4:
            self.n, self.c, self.h, self.w = shape
        elif len(shape) == 2:
            self.n, self.c = shape
            self.h = self.w = 1
        else:
            raise PlanError("unsupported activation rank for %s: %s" % (name, shape))
        self.cp = _pad8(self.c)
        self.dtype = dtype
        self.needs_grad = needs_grad
        self.kind = kind  # act | logits | prob | data_nchw | label

    @property
    def rows(self):
        return self.n * self.h * self.w

    @property
    def numel(self):
        if self.kind in ("data_nchw", "prob", "label"):
            return int(np.prod(self.shape))
        return self.rows * self.cp


class PlanOp:
    def __init__(self, kind, name, **kw):
        self.kind = kind
        self.name = name
        self.__dict__.update(kw)

    def __repr__(self):
        return "<%s %s>" % (self.kind, self.name)


class Plan:
    """Fused op list for a symbol at fixed input shapes."""

    def __init__(self, symbol, data_shapes, label_shapes=(), dtype="bfloat16", for_training=True):
        self.symbol = symbol
        self.dtype = BF16 if dtype in ("bfloat16", "bf16", BF16) else F32
        self.for_training = for_training
        self.data_names = [n for n, _ in data_shapes]
        self.label_names = [n for n, _ in label_shapes]
        known = dict(list(data_shapes) + list(label_shapes))
        self.input_shapes = known
        self.topo = symbol._topo()
        self._infer(known)
        self.arg_names = symbol.list_arguments()
        self.aux_names = symbol.list_auxiliary_states()
        self.param_names = [n for n in self.arg_names if n not in known]
        self.tensors = {}
        self.alias = {}
        self.ops = []
        self.qweight = {}  # id(weight Quantization_int8 node) -> quant info
        self._lower()

    # --- shapes of every node output
    def _infer(self, known):
        from mxnet.symbol import _infer_node, _parse as parse
        shapes = {}
        for n in self.topo:
            if n.op == "null":
                if n.name in known:
                    shapes[(id(n), 0)] = tuple(known[n.name])
                elif "__shape__" in n.attrs:
                    shapes[(id(n), 0)] = tuple(parse(n.attrs["__shape__"]))
        for n in self.topo:
            if n.op != "null":
                _infer_node(n, shapes, False)
        self.shapes = shapes

    def shape_of(self, node, idx=0):
        return self.shapes[(id(node), idx)]

    def param_shape(self, name):
        for n in self.topo:
            if n.op == "null" and n.name == name:
                return self.shapes[(id(n), 0)]
        raise KeyError(name)

    # --- helpers
    def _consumers(self):
        cons = {}
        for n in self.topo:
            for (i, _) in n.inputs:
                cons.setdefault(id(i), []).append(n)
        for n, _ in self.symbol._outputs:
            cons.setdefault(id(n), []).append(None)  # graph output
        return cons

    def tensor(self, node):
        key = id(node)
        while key in self.alias:
            key = self.alias[key]
        return self.tensors[key]

    def _new_tensor(self, node, shape, dtype=None, kind="act", needs_grad=True):
        t = TensorSpec(node.name, shape, self.dtype if dtype is None else dtype, needs_grad, kind)
        self.tensors[id(node)] = t
        return t

    def _var_input(self, node):
        """Follow identity/Cast/Flatten aliases back; return (node, is_variable)."""
        while node.op in ("identity", "Cast", "Flatten"):
            node = node.inputs[0][0]
        return node

    @staticmethod
    def _is_quant(node):
        return node is not None and node.op == "_contrib_Quantization_int8"

    def _quant_info(self, n):
        """Quantization_int8 attrs (int8_api.py:133-136; semantics clip_grad_quantization_int8.py)."""
        if _parse(n.attrs.get("quant_mode", "minmax")) != "minmax":
            raise PlanError("%s: quant_mode other than 'minmax' not supported" % n.name)
        if int(_parse(n.attrs.get("delay_quant", 0))):
            raise PlanError("%s: delay_quant > 0 not supported" % n.name)
        if _parse(n.attrs.get("is_weight_perchannel", False)):
            raise PlanError("%s: per-channel weight quantization not supported" % n.name)
        return dict(name=n.name, minmax=n.inputs[1][0].name, ema=float(_parse(n.attrs.get("ema_decay", 0.99))),
                    nbits=int(_parse(n.attrs.get("nbits", 8))),
                    is_weight=bool(_parse(n.attrs.get("is_weight", False))))

    def _stem_quant(self, node, cons):
        """A data Quantization_int8 whose only consumer is the stem conv (folded into its im2col)."""
        cl = cons.get(id(node), [])
        return self._is_quant(node) and len(cl) == 1 and cl[0] is not None and cl[0].op == "Convolution" and \
            self._is_stem(cl[0])

    # --- lowering
    def _lower(self):
        cons = self._consumers()
        topo = self.topo
        done = set()
        order = {id(n): i for i, n in enumerate(topo)}
        data_vars = set(self.data_names)
        # data / label inputs
        for n in topo:
            if n.op == "null" and n.name in data_vars:
                shp = self.shape_of(n)
                t = TensorSpec(n.name, shp, F32, needs_grad=False, kind="data_nchw")
                self.tensors[id(n)] = t
                self.data_tensor = t
            elif n.op == "null" and n.name in self.label_names:
                self.tensors[id(n)] = TensorSpec(n.name, (self.shape_of(n)[0], 1), F32, False, "label")
        # pre-pass: fused residual adds (conv output consumed only by an add)
        fused_add_into = {}  # id(conv node) -> (add node, other input node)
        fused_add_relu = {}  # id(add node) -> relu node
        for n in topo:
            if n.op in ("_Plus", "elemwise_add", "ElementWiseSum") and len(n.inputs) == 2:
                a, b = n.inputs[0][0], n.inputs[1][0]
                cands = [x for x in (a, b) if x.op == "Convolution" and len(cons.get(id(x), [])) == 1
                         and id(x) not in fused_add_into and not self._is_stem(x)]
                if cands:
                    conv = max(cands, key=lambda x: order[id(x)])
                    other = b if conv is a else a
                    if order[id(other)] < order[id(conv)] or other.op == "null":
                        fused_add_into[id(conv)] = (n, other)
                        continue
                cl = cons.get(id(n), [])
                if len(cl) == 1 and cl[0] is not None and cl[0].op == "Activation" and \
                        _parse(cl[0].attrs.get("act_type")) == "relu":
                    fused_add_relu[id(n)] = cl[0]
        for n in topo:
            if n.op == "null" or id(n) in done:
                continue
            op = n.op
            if op in ("identity", "Flatten", "Cast"):
                # Cast is a no-op under the runtime precision policy (bf16 / fp32 compute)
                src = n.inputs[0][0]
                if op == "Flatten":
                    st = self.tensor(src)
                    if st.kind == "act" and (st.h != 1 or st.w != 1):
                        raise PlanError("Flatten of a spatial map (%s) is not supported" % n.name)
                self.alias[id(n)] = id(src) if id(src) not in self.alias else self.alias[id(src)]
                done.add(id(n))
            elif op == "Convolution":
                self._lower_conv(n, cons, fused_add_into.get(id(n)))
                done.add(id(n))
                if id(n) in fused_add_into:
                    addn = fused_add_into[id(n)][0]
                    self.alias[id(addn)] = id(n)
                    done.add(id(addn))
            elif op == "BatchNorm":
                cl = cons.get(id(n), [])
                relu_node = None
                if len(cl) == 1 and cl[0] is not None and cl[0].op == "Activation" and \
                        _parse(cl[0].attrs.get("act_type")) == "relu":
                    relu_node = cl[0]
                src = self._var_input(n.inputs[0][0])
                stem_consumers = [c for c in cl if c is not None and
                                  ((c.op == "Convolution" and self._is_stem(c)) or self._stem_quant(c, cons))]
                if src.op == "null" and src.name in data_vars and stem_consumers and len(cl) == 1:
                    done.add(id(n))  # folded into the stem conv (bn_data)
                    continue
                self._lower_bn(n, relu_node)
                self.ops[-1].relu_name = relu_node.name if relu_node is not None else None
                done.add(id(n))
                if relu_node is not None:
                    self.alias[id(relu_node)] = id(n)
                    done.add(id(relu_node))
            elif op == "_contrib_Quantization_int8":
                q = self._quant_info(n)
                src = n.inputs[0][0]
                if q["is_weight"]:
                    if src.op != "null":
                        raise PlanError("%s: weight quantization of a computed tensor" % n.name)
                    q["param"] = src.name
                    self.qweight[id(n)] = q
                elif not self._stem_quant(n, cons):  # (the stem's is folded into its im2col)
                    x = self.tensor(src)
                    if x.kind != "act":
                        raise PlanError("%s: data quantization of a non-activation tensor" % n.name)
                    y = self._new_tensor(n, x.shape)
                    self.ops.append(PlanOp("quant", n.name, x=x, y=y, q=q))
                done.add(id(n))
            elif op == "Activation":
                act = _parse(n.attrs.get("act_type"))
                if act != "relu":
                    raise PlanError("Activation %s is not supported" % act)
                x = self.tensor(n.inputs[0][0])
                y = self._new_tensor(n, self.shape_of(n))
                self.ops.append(PlanOp("relu", n.name, x=x, y=y, relu_name=n.name))
                done.add(id(n))
            elif op in ("_Plus", "elemwise_add", "ElementWiseSum"):
                if len(n.inputs) != 2:
                    raise PlanError("ElementWiseSum with %d inputs not supported" % len(n.inputs))
                a = self.tensor(n.inputs[0][0])
                b = self.tensor(n.inputs[1][0])
                relu_node = fused_add_relu.get(id(n))
                y = self._new_tensor(n, self.shape_of(n))
                self.ops.append(PlanOp("add", n.name, a=a, b=b, y=y, relu=relu_node is not None,
                                       relu_name=relu_node.name if relu_node is not None else None))
                done.add(id(n))
                if relu_node is not None:
                    self.alias[id(relu_node)] = id(n)
                    done.add(id(relu_node))
            elif op in ("_contrib_BroadcastScale", "broadcast_add"):
                self._lower_affine(n, cons, done)
            elif op == "Pooling":
                self._lower_pool(n)
                done.add(id(n))
            elif op == "FullyConnected":
                self._lower_fc(n)
                done.add(id(n))
            elif op == "SoftmaxOutput":
                x = self.tensor(n.inputs[0][0])
                if x.kind != "logits":
                    raise PlanError("SoftmaxOutput must follow FullyConnected")
                lab = self.tensors[id(n.inputs[1][0])]
                y = self._new_tensor(n, (x.n, x.c), F32, kind="prob", needs_grad=False)
                self.ops.append(PlanOp("softmax", n.name, x=x, label=lab, y=y,
                                       grad_scale=float(_parse(n.attrs.get("grad_scale", 1.0)))))
                done.add(id(n))
            else:
                raise PlanError("operator %s (%s) is not supported by the MI355X runtime" % (op, n.name))
        self.outputs = [self.tensor(n) for n, _ in self.symbol._outputs]
        self._fuse_bn_apply()
        self._mark_int8()

    def _mark_int8(self):
        """Quantized convolutions (a Quantization_int8 on both the data and the weight: resnet_int8,
        attach_quantize_node) whose input quantizer can also emit int8 codes run their forward on the
        int8 MFMAs (rn_conv_fwd_i8): exact integer sums of the codes, scaled by the two units, instead
        of bf16 / fp32 products of the fake-quantized values. RN_INT8_MFMA=0: the fake-quant path."""
        producer = {id(op.y): op for op in self.ops if op.kind == "quant"}
        on = os.environ.get("RN_INT8_MFMA", "1") != "0"
        for op in self.ops:
            if op.kind == "quant":
                op.emit_codes = False
        for op in self.ops:
            if op.kind != "conv":
                continue
            q = producer.get(id(op.x))
            op.int8 = bool(on and op.qweight is not None and q is not None and op.groups == 1 and
                           op.x.cp % 16 == 0 and q.q["nbits"] <= 8 and op.qweight["nbits"] <= 8 and
                           getattr(op, "xf", None) is None)
            op.qsrc = q if op.int8 else None
            if op.int8:
                q.emit_codes = True
        # (round 4's opt-in RN_QUANT_DEFER -- the values expanded from the codes on the weight-gradient stream
        # by rn_quant_int8_expand -- measured 4 % slower on C5 and was removed in round 5; the weight gradients
        # multiply the codes instead, codes_wgrad)
        users = {}
        for op in self.ops:
            for k in ("x", "a", "b", "res", "label"):
                t = getattr(op, k, None)
                if t is not None and hasattr(t, "numel"):
                    users.setdefault(id(t), []).append(op)
        for op in self.ops:
            if op.kind == "quant":
                op.value_users = users.get(id(op.y), [])
                op.codes_wgrad = False  # (the executor decides: _codes_wgrad)

    def _fuse_bn_apply(self):
        """BatchNorm+ReLU whose output feeds ONLY 1x1 convolutions (act1 -> conv1 / sc, act3 -> conv3
        of the pre-activation units, symbol/resnet.py:17-31) or poolings (relu0 -> pool0 of the stem and
        relu1 -> the global pool, symbol/resnet.py:94-97,111-113): the consumers stage max(x*sc+sh, 0)
        from the BN input while loading (rn_conv_fwd_x / rn_conv_bwd_filter_x / rn_pool_fwd_x) and the
        BN+ReLU output is never written or read back."""
        for op in self.ops:
            op.xf = None
            if op.kind == "bn":
                op.apply_fused = False
            if op.kind == "add":
                op.bn_a = op.bn_b = op.bn_a_key = None
        refs = {}
        for op in self.ops:
            for key in ("x", "res", "a", "b"):
                t = getattr(op, key, None)
                if isinstance(t, TensorSpec):
                    refs.setdefault(id(t), []).append((op, key))
        out_ids = {id(t) for t in self.outputs}
        self._fuse_bn_add(refs, out_ids)
        # default on since the LDS-DMA tiles apply it (igemm_big_kernel / wgrad_big_kernel XF): 22.82 ->
        # 22.17 ms per step on one box; RN_BN_APPLY_FUSION=0 writes act1 / act3
        if os.environ.get("RN_BN_APPLY_FUSION", "1") != "1":
            return
        # (the 3x3 stride-1 consumers too -- act2 -> conv2 of stage 1, RN_BN_APPLY_FUSION_3X3, rounds 4-5 -- measured
        # 0.6 % slower, then equal with the image-band forward: removed in round 6; the band kernels keep their
        # BN+ReLU-on-load forms, kernel-tested)
        def xf_ok(u):
            return u.groups == 1 and not getattr(u, "qweight", None) and tuple(u.kernel) == (1, 1)
        # (the poolings: rn_pool_fwd_x; round 6, RN_POOL_XF=0 for the A/B)
        pool_ok = os.environ.get("RN_POOL_XF", "1") == "1"
        for bn in self.ops:
            if bn.kind != "bn" or not bn.relu or id(bn.y) in out_ids:
                continue
            users = refs.get(id(bn.y), [])
            ok = users and all(key == "x" and ((u.kind == "conv" and xf_ok(u)) or (u.kind == "pool" and pool_ok))
                               for u, key in users)
            if not ok:
                continue
            bn.apply_fused = True
            bn.y.virtual = True
            for u, _ in users:
                u.xf = bn

    def _fuse_bn_add(self, refs, out_ids):
        """The post-activation unit tail (symbol/resnext.py:40-47, symbol/resnet.py:63-74: bn3 (+ the
        shortcut's BN) -> add -> relu): a BatchNorm without ReLU whose output only this add reads is
        applied inside the add (rn_bn_apply_add); its output is never written. RN_BN_ADD_FUSION=0 off."""
        if os.environ.get("RN_BN_ADD_FUSION", "1") != "1":
            return
        producer = {id(op.y): op for op in self.ops if op.kind == "bn"}
        for op in self.ops:
            if op.kind != "add" or op.a is op.b:
                continue
            fused = []
            for key in ("a", "b"):
                t = getattr(op, key)
                bn = producer.get(id(t))
                if bn is not None and not bn.relu and id(t) not in out_ids and len(refs.get(id(t), [])) == 1:
                    fused.append((key, bn))
            if not fused:
                continue
            op.bn_a_key, op.bn_a = fused[0]
            op.bn_b = fused[1][1] if len(fused) == 2 else None
            for _, bn in fused:
                bn.apply_fused = True
                bn.y.virtual = True

    def _is_stem(self, conv_node):
        src = conv_node.inputs[0][0]
        shp = self.shape_of(src)
        return len(shp) == 4 and shp[1] % 8 != 0

    def _param_node(self, node, idx):
        p = node.inputs[idx][0]
        if self._is_quant(p) and id(p) in self.qweight:
            return self.qweight[id(p)]["param"]
        if p.op != "null":
            raise PlanError("%s: computed weights are not supported" % node.name)
        return p.name

    def _weight_quant(self, node, idx=1):
        p = node.inputs[idx][0]
        return self.qweight.get(id(p)) if self._is_quant(p) else None

    def _conv_attrs(self, n):
        k = _tup(n.attrs["kernel"])
        st = _tup(n.attrs.get("stride", (1, 1))) or (1, 1)
        pd = _tup(n.attrs.get("pad", (0, 0))) or (0, 0)
        dl = _tup(n.attrs.get("dilate", (1, 1))) or (1, 1)
        g = int(_parse(n.attrs.get("num_group", 1)))
        if dl != (1, 1):
            raise PlanError("%s: dilation not supported" % n.name)
        return k, st, pd, g

    def _lower_conv(self, n, cons, fused):
        k, st, pd, g = self._conv_attrs(n)
        xshape = self.shape_of(n.inputs[0][0])
        yshape = self.shape_of(n)
        wname = self._param_node(n, 1)
        if not _parse(n.attrs.get("no_bias", False)):
            raise PlanError("%s: convolution bias not supported" % n.name)
        y = self._new_tensor(n, yshape)
        if self._is_stem(n):
            if g != 1:
                raise PlanError("%s: grouped stem convolution not supported" % n.name)
            src = self._var_input(n.inputs[0][0])
            squant = None
            if self._is_quant(src):
                squant = self._quant_info(src)
                src = self._var_input(src.inputs[0][0])
            bn = None
            if src.op == "BatchNorm":
                bn = src
                src = self._var_input(bn.inputs[0][0])
                if not _parse(bn.attrs.get("fix_gamma", True)):
                    raise PlanError("stem BatchNorm must have fix_gamma=True")
            if not (src.op == "null" and src.name in self.data_names):
                raise PlanError("%s: a conv over %d channels must read the data input" % (n.name, xshape[1]))
            kc = _pad8(k[0] * k[1] * xshape[1])
            kc = (kc + 31) // 32 * 32
            op = PlanOp("stem", n.name, x=self.tensors[id(src)], y=y, weight=wname, kernel=k, stride=st, pad=pd,
                        kc=kc, bn=None, quant=squant, qweight=self._weight_quant(n))
            if bn is not None:
                op.bn = dict(name=bn.name, gamma=self._param_node(bn, 1), beta=self._param_node(bn, 2),
                             mean=bn.inputs[3][0].name, var=bn.inputs[4][0].name,
                             eps=float(_parse(bn.attrs.get("eps", 1e-3))),
                             momentum=float(_parse(bn.attrs.get("momentum", 0.9))),
                             use_global_stats=bool(_parse(bn.attrs.get("use_global_stats", False))))
            self.ops.append(op)
            return
        x = self.tensor(n.inputs[0][0])
        if x.kind != "act":
            raise PlanError("%s: convolution over the raw data input needs C %% 8 != 0 (stem) here" % n.name)
        res = None
        if fused is not None:
            res = self.tensor(fused[1])
        if g != 1 and (xshape[1] % 8 or yshape[1] % 8):
            raise PlanError("%s: grouped convolution needs channel counts that are multiples of 8" % n.name)
        self.ops.append(PlanOp("conv", n.name, x=x, y=y, weight=wname, kernel=k, stride=st, pad=pd, res=res,
                               groups=g, qweight=self._weight_quant(n)))

    def _lower_bn(self, n, relu_node):
        x = self.tensor(n.inputs[0][0])
        shape = self.shape_of(n)
        y = self._new_tensor(n, shape)
        self.ops.append(PlanOp("bn", n.name, x=x, y=y, relu=relu_node is not None,
                               gamma=self._param_node(n, 1), beta=self._param_node(n, 2),
                               mean=n.inputs[3][0].name, var=n.inputs[4][0].name,
                               eps=float(_parse(n.attrs.get("eps", 1e-3))),
                               momentum=float(_parse(n.attrs.get("momentum", 0.9))),
                               fix_gamma=bool(_parse(n.attrs.get("fix_gamma", True))),
                               use_global_stats=bool(_parse(n.attrs.get("use_global_stats", False)))))

    def _chan_param(self, node_idx, c):
        """Name of a per-channel parameter Variable ((C,) or (1,C,1,1)), else None."""
        v = node_idx[0]
        shp = self.shapes.get((id(v), node_idx[1]))
        if v.op != "null" or v.name in self.data_names or shp is None:
            return None
        if int(np.prod(shp)) != c or (len(shp) == 4 and shp[1] != c):
            return None
        return v.name

    def _lower_affine(self, n, cons, done):
        """Per-channel affine y = [relu](x * scale + bias): the BroadcastScale -> broadcast_add pair that
        merge_bn folds an inference BatchNorm into (core/graph_optimize.py:90-93), a standalone
        broadcast_add of a per-channel parameter, or (two same-shape tensors) a plain add."""
        x = self.tensor(n.inputs[0][0])
        c = x.c
        scale = bias = None
        last = n
        if n.op == "_contrib_BroadcastScale":
            scale = self._chan_param(n.inputs[1], c)
            if scale is None:
                raise PlanError("%s: BroadcastScale needs a per-channel (1,C,1,1) scaler Variable" % n.name)
            cl = cons.get(id(n), [])
            if len(cl) == 1 and cl[0] is not None and cl[0].op == "broadcast_add" and cl[0].inputs[0][0] is n:
                bias = self._chan_param(cl[0].inputs[1], c)
                if bias is not None:
                    last = cl[0]
        else:
            bias = self._chan_param(n.inputs[1], c)
            if bias is None:
                other = self.tensor(n.inputs[1][0])
                if other.shape != x.shape:
                    raise PlanError("%s: broadcast_add of %s and %s not supported" % (n.name, x.shape, other.shape))
                y = self._new_tensor(n, self.shape_of(n))
                self.ops.append(PlanOp("add", n.name, a=x, b=other, y=y, relu=False, relu_name=None))
                done.add(id(n))
                return
        if x.kind != "act":
            raise PlanError("%s: per-channel affine over a non-activation tensor" % n.name)
        cl = cons.get(id(last), [])
        relu_node = None
        if len(cl) == 1 and cl[0] is not None and cl[0].op == "Activation" and \
                _parse(cl[0].attrs.get("act_type")) == "relu":
            relu_node = cl[0]
        y = self._new_tensor(n, self.shape_of(n))
        self.ops.append(PlanOp("affine", n.name, x=x, y=y, gamma=scale, beta=bias, relu=relu_node is not None,
                               relu_name=relu_node.name if relu_node is not None else None))
        done.add(id(n))
        for extra in (last, relu_node):
            if extra is not None and extra is not n:
                self.alias[id(extra)] = id(n)
                done.add(id(extra))

    def _lower_pool(self, n):
        x = self.tensor(n.inputs[0][0])
        y = self._new_tensor(n, self.shape_of(n))
        ptype = _parse(n.attrs.get("pool_type", "max"))
        if ptype not in ("max", "avg"):
            raise PlanError("pool_type %s not supported" % ptype)
        glob = bool(_parse(n.attrs.get("global_pool", False)))
        if _parse(n.attrs.get("pooling_convention", "valid")) != "valid" and not glob:
            raise PlanError("pooling_convention other than 'valid' not supported")
        k = _tup(n.attrs.get("kernel", (1, 1))) or (1, 1)
        st = _tup(n.attrs.get("stride", (1, 1))) or (1, 1)
        pd = _tup(n.attrs.get("pad", (0, 0))) or (0, 0)
        self.ops.append(PlanOp("pool", n.name, x=x, y=y, type=ptype, global_pool=glob, kernel=k, stride=st, pad=pd))

    def _lower_fc(self, n):
        x = self.tensor(n.inputs[0][0])
        if x.h != 1 or x.w != 1:
            raise PlanError("%s: FullyConnected over a spatial map is not supported" % n.name)
        nh = int(_parse(n.attrs["num_hidden"]))
        no_bias = bool(_parse(n.attrs.get("no_bias", False)))
        y = self._new_tensor(n, (x.n, nh), F32, kind="logits")
        self.ops.append(PlanOp("fc", n.name, x=x, y=y, weight=self._param_node(n, 1),
                               bias=None if no_bias else self._param_node(n, 2), nh=nh,
                               qweight=self._weight_quant(n)))

    def summary(self):
        kinds = {}
        for op in self.ops:
            kinds[op.kind] = kinds.get(op.kind, 0) + 1
        return kinds

    def train_flops(self):
        """Algorithmic FLOP per step (2 FLOP/MAC): fwd + dgrad (except the stem) + wgrad."""
        total = 0
        for op in self.ops:
            if op.kind in ("conv", "stem"):
                y = op.y
                cin = op.x.shape[1] // getattr(op, "groups", 1)
                macs = y.n * y.h * y.w * y.c * cin * op.kernel[0] * op.kernel[1]
                total += 2 * macs * (2 if op.kind == "stem" else 3)
            elif op.kind == "fc":
                total += 2 * op.x.n * op.x.c * op.nh * 3
        return total


# ============================================================================= executor (GPU)
class _GradState:
    """Gradient routing during backward-plan construction (req write/add, lazy fan-in)."""

    def __init__(self, ex):
        self.ex = ex
        self.has_value = set()
        self.pending = {}

    def read(self, t):
        key = id(t)
        pend = self.pending.pop(key, [])
        if key not in self.has_value:
            if not pend:
                return None
            if len(pend) == 1:
                return pend[0]
            buf = self.ex.grad_buf(t)
            self.ex._emit_bwd(("add", t.numel, pend[0], pend[1], buf))
            self.ex._gw[key] = ("other",)
            pend = pend[2:]
            self.has_value.add(key)
        else:
            buf = self.ex.grad_buf(t)
        for p in pend:
            self.ex._emit_bwd(("add", t.numel, buf, p, buf))
            self.ex._gw[key] = ("other",)
        return buf

    def contribute(self, t):
        """(out_buffer, add_src) for a kernel with an add_src operand."""
        key = id(t)
        buf = self.ex.grad_buf(t)
        if key in self.has_value:
            # another contribution lands in a buffer that already holds one: the previous writer's fused
            # BN reduction (self.ex._gw, pool / dgrad) saw a partial gradient. A fusing writer re-registers
            # itself after its call (its output then includes this add operand); any other writer leaves
            # the entry "other", so the BN backward runs its own reduction
            self.ex._gw[key] = ("other",)
            return buf, buf
        self.has_value.add(key)
        pend = self.pending.get(key)
        if pend:
            return buf, pend.pop(0)
        return buf, None

    def alias(self, t, buf):
        self.pending.setdefault(id(t), []).append(buf)


class Executor:
    """Device buffers + bound C calls for one Plan on one GPU."""

    def __init__(self, plan, device, bucket_bytes=None):
        if bucket_bytes is None:  # RCCL all-reduce bucket size (RN_BUCKET_MB, default 25 MB)
            bucket_bytes = int(float(os.environ.get("RN_BUCKET_MB", "25")) * (1 << 20))
        import torch
        self.torch = torch
        self.plan = plan
        self.device = torch.device(device)
        self.dtype = plan.dtype
        self.tdtype = torch.bfloat16 if self.dtype == BF16 else torch.float32
        self.lib = L.load()
        # device='cpu' builds the full call plan without launching anything (CPU dry-run tests)
        self.dry_run = self.device.type == "cpu"
        # every bound call shares ONE c_void_p stream argument, re-pointed at torch's current stream
        # whenever a call list runs: the plan then follows the caller's stream -- torch ops, RCCL
        # ordering and HIP-graph capture (torch.cuda.graph) all see the same stream
        self._spv = L.C.c_void_p(0)
        # weight gradients run on a second stream (RN_WGRAD_STREAM=0: all on one): each forks from
        # the compute stream right before it (its dy is final there, its x was final since the
        # forward) and the backward joins it at the end, so a layer's wgrad overlaps the next
        # layers' dgrad / BatchNorm kernels and fills the CUs their last rounds leave idle
        self._spv2 = L.C.c_void_p(0)
        self._side_stream = None
        if not self.dry_run and os.environ.get("RN_WGRAD_STREAM", "1") == "1":
            self._side_stream = torch.cuda.Stream(device=self.device)
        # the weight gradients' split-M grids: part of the chip when they overlap the data-gradient chain,
        # all of it when they run serialised (before the plan sizes its workspace from the same key)
        # (50 % for every graph; round 6, one box, timed steps without event packets: C2 18.82 / 18.83 vs
        # 19.08 / 19.03 ms at 45 %, 55 % 18.95 / 18.98, 60 % 18.97, 70 % 19.00; C4 26.79 vs 27.01, C5 21.23 vs 21.32)
        self.wgrad_split_pct = L.WGRAD_SPLIT_OVERLAPPED
        L.set_wgrad_split(os.environ.get("RN_WGRAD_STREAM", "1") == "1", self.wgrad_split_pct)
        self._side_idx = set()
        self._side_pre = set()  # (of _side_idx) SIDE_PRE_CALLS
        self._events = {}
        self._side_enabled = True  # False: the side-stream calls run on the compute stream (serialised timing)
        self._sync_stream()
        self._acts = {}
        self._grads = {}
        self._fwd_train, self._fwd_infer, self._bwd = [], [], []
        # Quantization_int8: activation EMA states initialise from the first training batch
        self._qfirst = L.C.c_int32(1)
        # SGD writes the dense weights' compute copies itself (rn_sgd_mom_update_pack); 0 = the
        # separate pack launches after every update
        self.fuse_packs = os.environ.get("RN_FUSED_PACK", "1") == "1"
        self._build_params()
        self._alloc_acts()
        self._build_forward()
        self._build_backward()
        self._route_wgrads()
        self._build_update()
        self.bucket_bytes = bucket_bytes
        # the trailing bucket (RN_TAIL_BUCKET_MB, default 5 MB): the parameters at the flat buffer's end --
        # the stem's and the first stage's, whose gradients the backward completes last -- get a bucket of
        # their own, so that only this small one is exposed after the backward's last kernel
        self.tail_bucket_bytes = int(float(os.environ.get("RN_TAIL_BUCKET_MB", "5")) * (1 << 20))
        self.num_update = 0

    @property
    def side_enabled(self):
        return self._side_enabled

    @side_enabled.setter
    def side_enabled(self, on):
        """False: the weight gradients run on the compute stream, serialised (bench.py's calibration step),
        with the whole chip's split-M grids -- as RN_WGRAD_STREAM=0 runs them (lib.set_wgrad_split; the
        workspace is sized for both)."""
        on = bool(on)
        if on != self._side_enabled and self._side_stream is not None:
            L.set_wgrad_split(on, self.wgrad_split_pct)
        self._side_enabled = on

    # ------------------------------------------------------------------ buffers
    def _zeros(self, numel, dtype):
        return self.torch.zeros(int(max(numel, 1)), dtype=dtype, device=self.device)

    def _tdt(self, d):
        return self.torch.bfloat16 if d == BF16 else self.torch.float32

    def act(self, t):
        b = self._acts.get(id(t))
        if b is None:
            b = self._zeros(t.numel, self._tdt(t.dtype))
            self._acts[id(t)] = b
        return b

    def grad_buf(self, t):
        b = self._grads.get(id(t))
        if b is None:
            b = self._zeros(t.numel, self.tdtype)
            self._grads[id(t)] = b
        return b

    def _build_params(self):
        torch = self.torch
        plan = self.plan
        # reverse forward order: grads of late layers complete first during backward
        order = []
        seen = set()
        for op in plan.ops:
            for key in ("weight", "bias"):
                nm = getattr(op, key, None)
                if nm and nm not in seen:
                    order.append(nm)
                    seen.add(nm)
            for key in ("gamma", "beta"):
                nm = getattr(op, key, None)
                if nm and nm not in seen:
                    order.append(nm)
                    seen.add(nm)
            if op.kind == "stem" and op.bn:
                for key in ("gamma", "beta"):
                    nm = op.bn[key]
                    if nm not in seen:
                        order.append(nm)
                        seen.add(nm)
        missing = [n for n in plan.param_names if n not in seen]
        if missing:
            raise PlanError("parameters not consumed by any lowered op: %s" % missing[:5])
        order = list(reversed(order))
        self.param_order = order
        self.param_off = {}
        self.param_shape = {}
        self.param_layout = {}
        off = 0
        conv_w = {op.weight for op in plan.ops if op.kind in ("conv", "stem")}
        for nm in order:
            shp = tuple(plan.param_shape(nm))
            self.param_shape[nm] = shp
            self.param_layout[nm] = "krsc" if (nm in conv_w and len(shp) == 4) else "plain"
            self.param_off[nm] = off
            off += int(np.prod(shp))
            off = (off + 3) // 4 * 4  # 16-byte aligned tensors
        self.nparam = off
        self.master = self._zeros(off, torch.float32)
        self.grad = self._zeros(off, torch.float32)
        self.mom = self._zeros(off, torch.float32)
        # aux (moving stats)
        self.aux_off = {}
        aoff = 0
        for nm in plan.aux_names:
            shp = tuple(plan.param_shape(nm))
            self.aux_off[nm] = (aoff, shp)
            aoff += int(np.prod(shp))
        self.aux = self._zeros(aoff, torch.float32)
        # device optimizer tables
        offs = [self.param_off[n] for n in order]
        nums = [int(np.prod(self.param_shape[n])) for n in order]
        self.opt_offsets = torch.tensor(offs, dtype=torch.int64, device=self.device)
        self.opt_numels = torch.tensor(nums, dtype=torch.int64, device=self.device)
        self.wd_mult = np.array([1.0 if (n.endswith("_weight") or n.endswith("_gamma")) else 0.0 for n in order],
                                dtype=np.float32)
        self.opt_wds = torch.zeros(len(order), dtype=torch.float32, device=self.device)
        self._wd_value = None

    def pview(self, name):
        o = self.param_off[name]
        return self.master[o:o + int(np.prod(self.param_shape[name]))]

    def gview(self, name):
        o = self.param_off[name]
        return self.grad[o:o + int(np.prod(self.param_shape[name]))]

    def aview(self, name):
        o, shp = self.aux_off[name]
        return self.aux[o:o + int(np.prod(shp))]

    def _alloc_acts(self):
        for t in self.plan.tensors.values():
            if not getattr(t, "virtual", False):  # a fused BN+ReLU output is never materialised
                self.act(t)
        # input pipeline (data/imagenet.py SyntheticDataIter hands pinned host batches): two device
        # buffers; the stem reads whichever _in_ptr points at
        t = self.plan.data_tensor
        self._in_bufs = [self.act(t), None]
        self._in_free = [None, None]
        self._in_idx = 0
        self._in_ptr = L.C.c_void_p(self._in_bufs[0].data_ptr())
        self._copy_stream = None
        self.stats = self._zeros(4, self.torch.float32)

    # ------------------------------------------------------------------ helpers
    def _p(self, t):
        return None if t is None else L.ptr(t)

    def _pp(self, name):
        return L.C.c_void_p(self.master.data_ptr() + 4 * self.param_off[name])

    def _gp(self, name):
        return L.C.c_void_p(self.grad.data_ptr() + 4 * self.param_off[name])

    def _ap(self, name):
        return L.C.c_void_p(self.aux.data_ptr() + 4 * self.aux_off[name][0])

    def _call(self, fname, *args):
        fn = getattr(self.lib, fname)
        return (fname, fn, args)

    def _emit_bwd(self, item):
        if item[0] == "add":
            _, n, a, b, dst = item
            self._bwd.append(self._call("rn_eltwise_add", n, self.dtype, self._p(a), self._p(b), self._p(dst), 0,
                                        self._sp()))
        else:
            self._bwd.append(item)

    def _sp(self):
        return self._spv

    @property
    def stream(self):
        return None if self.dry_run else self.torch.cuda.current_stream(self.device)

    def _sync_stream(self):
        if not self.dry_run:
            self._spv.value = self.torch.cuda.current_stream(self.device).cuda_stream
            if self._side_stream is not None:
                self._spv2.value = self._side_stream.cuda_stream if self.side_enabled else self._spv.value

    WGRAD_CALLS = ("rn_conv_bwd_filter", "rn_conv_bwd_filter_ws", "rn_conv_bwd_filter_x", "rn_conv_bwd_filter_i8",
                   "rn_stem_conv_wgrad_p4", "rn_stem_clip_wgrad", "rn_stem_clip_wgrad_chunk", "rn_stem_clip_dbeta")
    # side-stream calls that depend on the forward only, not on the backward so far: no fork of their own
    # (they run while the side stream waits for the next dy), except the first of a step
    SIDE_PRE_CALLS = ("rn_stem_clip_mask",)

    def _stem_clip_mask(self, op):
        """Does the int8 stem's input-quantizer clip gradient ride in its weight gradient (bf16 NHWC-8
        image, rn_stem_clip_*; RN_STEM_CLIP_MASK=0: the gather kernel rn_stem_quant_clip_grad)?"""
        return bool(op.kind == "stem" and op.quant and op.bn and self.dtype == BF16 and not op.p4 and
                    self.lib is not None and os.environ.get("RN_STEM_CLIP_MASK", "1") == "1" and
                    self.lib.rn_stem_clip_supported(L.C.byref(op.dfull)))

    def _route_wgrads(self):
        """Bind the weight-gradient calls of the backward plan to the side stream.

        Invariant: the shared split-M slab workspace (self.wgrad_ws) is used by these calls only, so
        with the side stream on it is touched by that one stream, in plan order."""
        if self._side_stream is None:
            return
        ws = self.wgrad_ws.data_ptr() if self.wgrad_ws is not None else None
        for i, (name, fn, args) in enumerate(self._bwd):
            if name in self.WGRAD_CALLS + self.SIDE_PRE_CALLS and args and args[-1] is self._spv:
                self._bwd[i] = (name, fn, args[:-1] + (self._spv2,))
                self._side_idx.add(i)
                if name in self.SIDE_PRE_CALLS:
                    self._side_pre.add(i)
            elif ws is not None and any(isinstance(a, L.C.c_void_p) and a.value == ws for a in args):
                raise PlanError("%s uses the weight-gradient slab workspace but is not routed to the side "
                                "stream" % name)

    def _event(self, key):
        """One persistent HIP event per fork / join point of the backward plan (re-recorded every
        step): no event is created or destroyed while a stream may still wait on it."""
        ev = self._events.get(key)
        if ev is None:
            ev = self._events[key] = self.torch.cuda.Event()
        return ev

    def _fork(self, key):
        """The side stream continues after everything enqueued on the compute stream so far."""
        ev = self._event(("fork", key))
        ev.record(self.torch.cuda.current_stream(self.device))
        self._side_stream.wait_event(ev)

    def _join(self):
        ev = self._event(("join",))
        ev.record(self._side_stream)
        self.torch.cuda.current_stream(self.device).wait_event(ev)

    def _conv_desc(self, n, h, w, c, c_real, k, kernel, stride, pad, groups=1):
        d = L.ConvDesc(dtype=self.dtype, n=n, h=h, w=w, c=c, c_real=c_real, k=k, k_pad=_pad8(k), r=kernel[0],
                       s=kernel[1], stride_h=stride[0], stride_w=stride[1], pad_h=pad[0], pad_w=pad[1],
                       groups=groups)
        L.check(self.lib.rn_conv_desc_init(L.C.byref(d)), "rn_conv_desc_init")
        return d

    def _codes_wgrad(self, plan):
        """Quantizers whose fake-quantized values only int8 convolutions read, each of whose weight
        gradients takes the int8 codes instead (rn_conv_bwd_filter_i8: dW = unit * sum dy * code, the
        streaming and 128 / 256-column kernels, every ResNet-50 layer but stage 1's 3x3): the forward
        writes the codes only,
        and the bf16 values -- 2 of the pass's 5 bytes per element -- are never written or read
        (RN_QUANT_CODES_WGRAD=0: values + bf16 weight gradients)."""
        on = os.environ.get("RN_QUANT_CODES_WGRAD", "1") == "1" and self.dtype == L.RN_BF16
        for op in plan.ops:
            if op.kind != "quant":
                continue
            us = getattr(op, "value_users", [])
            ok = on and op.emit_codes and bool(us) and \
                all(u.kind == "conv" and u.int8 and u.qsrc is op for u in us)
            if ok:
                for u in us:
                    x, y = u.x, u.y
                    d = self._conv_desc(x.n, x.h, x.w, x.cp, x.c, y.c, u.kernel, u.stride, u.pad, u.groups)
                    ok = ok and int(self.lib.rn_conv_wgrad_i8_supported(L.C.byref(d))) == 1
            op.codes_wgrad = bool(ok)

    # ------------------------------------------------------------------ forward
    def _build_forward(self):
        plan = self.plan
        sp = self._sp()
        ws_bytes = 64
        self._descs = []  # keep ctypes structs alive
        self._codes_wgrad(plan)
        self.packs = []   # weight pack calls (bind time / set_params)
        # every weight quantizer in one rn_weight_quant_pack (RN_WQUANT_BATCH=0: three calls per weight)
        self._wq_batch = os.environ.get("RN_WQUANT_BATCH", "1") == "1"
        self._wq_ops = []
        self.fused_packs = {}  # param -> rn_wpack fields: copies rewritten by the SGD kernel itself
        self.unfused_packs = []  # packs that still run after every update (grouped, fake-quantized)
        # the grouped layers' repacks in one rn_conv_weight_pack_multi (RN_GPACK_BATCH=0: one call each)
        self._gpack_batch = os.environ.get("RN_GPACK_BATCH", "1") == "1"
        self._gpacks = []
        self.bn_state = {}
        stem_ws = 64
        # BatchNorm statistics straight from the producing conv's epilogue (no separate stats pass)
        producer = {}
        for op in plan.ops:
            op.bnstats = False
            op.part_src = None
            if op.kind in ("conv", "stem"):
                producer[id(op.y)] = op
        # default on since the 256-row conv tiles (measured -0.6 % step time with the bwd fusion)
        # fused only where the producer runs the 256-row tile: the 128-row kernel's epilogue costs
        # more than the statistics pass it saves (RN_BN_EPILOGUE_STATS=2: every conv producer)
        stats_mode = os.environ.get("RN_BN_EPILOGUE_STATS", "1")
        if stats_mode in ("1", "2"):
            for op in plan.ops:
                if op.kind == "bn" and not op.use_global_stats:
                    src = producer.get(id(op.x))
                    if src is not None and src.kind == "conv" and src.y.c % 8 == 0 and src.y.cp == op.x.cp and \
                            (stats_mode == "2" or self._big_tile(src, 0) or self._grouped_fuse(src, 0)):
                        src.bnstats = True
                        op.part_src = src
                    elif src is not None and src.kind == "stem" and src.y.cp == op.x.cp and \
                            os.environ.get("RN_STEM_BN_STATS", "1") == "1":
                        # (bn0's statistics from the stem band kernel: kept only where the stem runs it with
                        # whole bands per workgroup, rn_stem_bnstats_blocks; decided when the stem is built)
                        src.bnstats = True
                        op.part_src = src
        for op in plan.ops:
            if op.kind == "bn":
                d = L.BNDesc(dtype=self.dtype, m=op.x.rows, c=op.x.cp, c_real=op.x.c, eps=op.eps,
                             momentum=op.momentum, fix_gamma=int(op.fix_gamma), relu=int(op.relu))
                ws_bytes = max(ws_bytes, self.lib.rn_bn_workspace_bytes(L.C.byref(d)))
                op.desc = d
            elif op.kind == "affine":
                d = L.BNDesc(dtype=self.dtype, m=op.x.rows, c=op.x.cp, c_real=op.x.c, eps=0.0, momentum=0.0,
                             fix_gamma=0, relu=int(op.relu))
                ws_bytes = max(ws_bytes, self.lib.rn_bn_workspace_bytes(L.C.byref(d)))
            elif op.kind == "stem":
                x = op.x
                b = op.bn or {}
                op.bn_desc = L.BNDesc(dtype=self.dtype, m=x.n * x.h * x.w, c=8, c_real=x.c, eps=b.get("eps", 1e-5),
                                      momentum=b.get("momentum", 0.9), fix_gamma=1, relu=0)
                ws_bytes = max(ws_bytes, 2 * 8 * 256 * 4 + 64)
        self.ws = self._zeros(ws_bytes // 4 + 16, self.torch.float32)
        wsp = self._p(self.ws)
        self.qws = self._zeros(4096, self.torch.float32)
        qwsp = self._p(self.qws)
        # activation quantizers whose BatchNorm(+ReLU) input nothing else reads (the int8 graph): the
        # quantizer applies the BN on load (rn_quant_int8_fwd_codes_bn, bit-identical) and the BN's
        # output is never written -- with the folded straight-through backward nothing reads it
        # (RN_QUANT_BN_FUSE=0: rn_bn_apply + rn_quant_int8_fwd_codes)
        groups = self._quant_groups() if os.environ.get("RN_QUANT_BN_FUSE", "1") == "1" else {}
        for op in plan.ops:
            op.bn_src = None
            op.bn_peer = None  # the second quantizer of the same BN output (written by this op's call)
            op.bn_lead = None  # (the quantizer whose call writes this one)
            op.want_mm = False
            op.mm_src = None
            if op.kind == "bn":
                op.apply_in_quant = False
        for bn, qs in groups.values():
            if all(q.emit_codes for q in qs) and bn.x.cp % 16 == 0:
                bn.apply_in_quant = True
                qs[0].bn_src = bn
                if len(qs) == 2:
                    qs[0].bn_peer, qs[1].bn_lead = qs[1], qs[0]
                # the quantizers' max from the producing int8 conv's per-block extremes of the BN input
                # (rn_conv_fwd_i8_mm -> rn_bn_desc.xmm) instead of a pass over it (RN_QUANT_BN_MM=0: the pass)
                src = bn.part_src
                if src is not None and getattr(src, "int8", False) and bn.relu and self.dtype == BF16 and \
                        os.environ.get("RN_QUANT_BN_MM", "1") == "1":
                    src.want_mm = True
                    src.mm_gamma = None if bn.fix_gamma else bn.gamma  # (its sign is the BN scale's)
                    bn.mm_src = src
        for op in plan.ops:
            F, I = [], []  # train-mode, infer-mode call lists
            op.wsrc = self._weight_source(op, qwsp, sp) if getattr(op, "qweight", None) else \
                (self._pp(op.weight) if getattr(op, "weight", None) else None)
            if op.kind == "stem":
                # conv0 over the 3-channel input: bn_data statistics straight from the NCHW batch, one
                # pass writing the normalised NHWC-8 copy, then the implicit GEMM in its small-C mode
                # (k = tap*8 + c flattened; symbol/resnet.py:90-93)
                x, y = op.x, op.y
                dfull = self._conv_desc(x.n, x.h, x.w, 8, x.c, y.c, op.kernel, op.stride, op.pad)
                assert (dfull.p, dfull.q) == (y.h, y.w), (op.name, dfull.p, dfull.q, y.h, y.w)
                op.dfull = op.desc = dfull
                # bf16 (not int8-quantized): the zero-bordered NHWC4 image instead of NHWC-8 (the
                # reduction runs over 8x8 taps x 4 channels = 256 instead of 7x7 x 8 = 392, and no
                # in-image tests); its border is zeroed here once, the prepare pass writes the inside
                hp = max(x.h + 2 * op.pad[0], (dfull.p - 1) * op.stride[0] + 8)
                wp = max(x.w + 2 * op.pad[1], (dfull.q - 1) * op.stride[1] + 8)
                op.p4 = None
                # (the NHWC4 stem's weight gradient adds with atomics: not in the deterministic mode)
                if self.dtype == BF16 and not op.quant and os.environ.get("RN_STEM_P4", "1") == "1" and \
                        os.environ.get("RN_DETERMINISTIC", "0") != "1" and \
                        self.lib.rn_stem_p4_supported(L.C.byref(dfull), hp, wp):
                    op.p4 = (hp, wp)
                    op.x8 = self._zeros(x.n * hp * wp * 4, self.tdtype)
                    op.wk = self._zeros(y.c * 256, self.tdtype)
                    c_ = self._call("rn_stem_weight_pack_p4", L.C.byref(dfull), op.wsrc, self._p(op.wk), sp)
                    self.packs.append(c_)
                    self.unfused_packs.append(c_)
                else:
                    op.x8 = self._zeros(x.n * x.h * x.w * 8, self.tdtype)
                    op.wk = self._zeros(y.c * op.kernel[0] * op.kernel[1] * 8, self.tdtype)
                    self._add_pack(op, dfull, op.wk, None, sp)
                stem_ws = max(stem_ws, y.h * y.w * y.cp + y.h * op.kernel[1] * y.c + y.c * op.kernel[0] * op.kernel[1] + 64)
                xnchw = self._in_ptr  # the current input buffer (double-buffered H2D pipeline)
                op.bnbuf = self._zeros(4 * 8, self.torch.float32)
                sm, si, sc, sh = [L.C.c_void_p(op.bnbuf.data_ptr() + 32 * i) for i in range(4)]
                op.bn_ptrs = (sm, si, sc, sh)
                b = op.bn
                if b:
                    bnargs = (self._pp(b["gamma"]), self._pp(b["beta"]), self._ap(b["mean"]), self._ap(b["var"]))
                    mode_f = 1 if b["use_global_stats"] else 0
                    mode_i = 1
                else:
                    bnargs = (None, None, None, None)
                    mode_f = mode_i = 2
                for lst, mode in ((F, mode_f), (I, mode_i)):
                    if op.p4:
                        lst.append(self._call("rn_stem_prepare_p4", L.C.byref(op.bn_desc), xnchw, x.n, x.c, x.h, x.w,
                                              self._p(op.x8), op.p4[0], op.p4[1], op.pad[0], op.pad[1], mode,
                                              *bnargs, sm, si, sc, sh, wsp, sp))
                    else:
                        lst.append(self._call("rn_stem_prepare", L.C.byref(op.bn_desc), xnchw, x.n, x.c, x.h, x.w,
                                              self._p(op.x8), mode, *bnargs, sm, si, sc, sh, wsp, sp))
                if op.quant:
                    q = op.quant
                    for lst, tr in ((F, 1), (I, 0)):
                        lst.append(self._call("rn_quant_int8_fwd", self.dtype, x.n * x.h * x.w * 8, self._p(op.x8),
                                              self._p(op.x8), self._ap(q["minmax"]), 0, tr, q["ema"], self._qfirst,
                                              q["nbits"], qwsp, sp))
                nblk = int(self.lib.rn_stem_bnstats_blocks(L.C.byref(dfull), *op.p4)) if (op.p4 and op.bnstats) else 0
                if op.bnstats and nblk <= 0:  # the BatchNorm runs its own statistics pass
                    op.bnstats = False
                    for o in plan.ops:
                        if getattr(o, "part_src", None) is op:
                            o.part_src = None
                if op.p4:
                    c_ = self._call("rn_stem_conv_fwd_p4", L.C.byref(dfull), self._p(op.x8), self._p(op.wk),
                                    self._p(self.act(y)), op.p4[0], op.p4[1], sp)
                    I.append(c_)
                    if op.bnstats:  # + bn0's statistics of the stored output, one block per band workgroup
                        op.part_blocks, op.part_rows = nblk, y.rows // nblk
                        op.part = self._zeros(nblk * 3 * y.cp, self.torch.float32)
                        F.append(self._call("rn_stem_conv_fwd_p4_bnstats", L.C.byref(dfull), self._p(op.x8),
                                            self._p(op.wk), self._p(self.act(y)), op.p4[0], op.p4[1],
                                            self._p(op.part), sp))
                    else:
                        F.append(c_)
                else:
                    I.append(self._call("rn_conv_fwd", L.C.byref(dfull), self._p(op.x8), self._p(op.wk),
                                        self._p(self.act(y)), self.dtype, None, None, sp))
                    F.append(self._conv_fwd_call(op, dfull, self._p(op.x8), None, sp))
            elif op.kind == "conv":
                x, y = op.x, op.y
                d = self._conv_desc(x.n, x.h, x.w, x.cp, x.c, y.c, op.kernel, op.stride, op.pad, op.groups)
                assert (d.p, d.q) == (y.h, y.w), (op.name, d.p, d.q, y.h, y.w)
                op.desc = d
                op.wc = self._zeros(self.lib.rn_conv_pack_numel(L.C.byref(d), 1), self.tdtype)
                if getattr(op, "int8", False):
                    # forward copy: the int8 codes (KRSC); the data-gradient copy stays the
                    # fake-quantized values in the compute dtype (STE backward)
                    op.wk = None
                    op.wk8 = self.torch.zeros(int(self.lib.rn_conv_pack_numel(L.C.byref(d), 0)),
                                              dtype=self.torch.int8, device=self.device)
                    if not self._wq_batch:  # (batched: written by rn_weight_quant_pack)
                        self._add_pack(op, d, None, op.wc, sp)
                        c_ = self._call("rn_conv_weight_pack_i8", L.C.byref(d), self._pp(op.weight),
                                        self._p(op.wunit), self._p(op.wk8), sp)
                        self.packs.append(c_)
                        self.unfused_packs.append(c_)
                else:
                    op.wk = self._zeros(self.lib.rn_conv_pack_numel(L.C.byref(d), 0), self.tdtype)
                    self._add_pack(op, d, op.wk, op.wc, sp)
                res = self._p(self.act(op.res)) if op.res is not None else None
                xin = self._p(self.act(op.xf.x)) if op.xf is not None else self._p(self.act(x))
                I.append(self._conv_fwd_call(op, d, xin, res, sp, stats=False))
                F.append(self._conv_fwd_call(op, d, xin, res, sp))
            elif op.kind == "bn":
                x, y = op.x, op.y
                c = x.cp
                op.buf = self._zeros(4 * c, self.torch.float32)
                op.sm, op.si, op.sc, op.sh = [L.C.c_void_p(op.buf.data_ptr() + 4 * c * i) for i in range(4)]
                gamma = self._pp(op.gamma)
                # fused into the 1x1 consumers' loads or the quantizer's: coefficients only
                yptr = None if op.apply_fused or op.apply_in_quant else self._p(self.act(y))
                if op.mm_src is not None and getattr(op.mm_src, "part_mm", None) is not None:
                    op.desc.xmm = op.mm_src.part_mm.data_ptr()
                    op.desc.xmm_blocks = op.mm_src.part_blocks
                infer = self._call("rn_bn_fwd_infer", L.C.byref(op.desc), self._p(self.act(x)), yptr,
                                   gamma, self._pp(op.beta), self._ap(op.mean), self._ap(op.var), op.sc, op.sh, sp)
                if op.use_global_stats:
                    F.append(infer)
                elif op.part_src is not None:
                    s_ = op.part_src
                    F.append(self._call("rn_bn_fwd_train_part", L.C.byref(op.desc), self._p(s_.part), s_.part_blocks,
                                        s_.part_rows, s_.y.cp, self._p(self.act(x)), yptr, gamma,
                                        self._pp(op.beta), self._ap(op.mean), self._ap(op.var), op.sm, op.si, op.sc,
                                        op.sh, wsp, sp))
                else:
                    F.append(self._call("rn_bn_fwd_train", L.C.byref(op.desc), self._p(self.act(x)),
                                        yptr, gamma, self._pp(op.beta), self._ap(op.mean),
                                        self._ap(op.var), op.sm, op.si, op.sc, op.sh, wsp, sp))
                I.append(infer)
            elif op.kind == "affine":
                # y = [relu](x*scale + bias) with per-channel parameters copied into channel-padded
                # coefficient vectors each forward (set_params / SGD may change them)
                x, y = op.x, op.y
                c = x.cp
                op.buf = self._zeros(4 * c, self.torch.float32)
                if op.gamma is None:
                    op.buf[:x.c] = 1.0
                op.sc, op.sh, op.zero, op.one = [L.C.c_void_p(op.buf.data_ptr() + 4 * c * i) for i in range(4)]
                op.buf[3 * c:3 * c + x.c] = 1.0
                op.desc = L.BNDesc(dtype=self.dtype, m=x.rows, c=c, c_real=x.c, eps=0.0, momentum=0.0,
                                   fix_gamma=int(op.gamma is None), relu=int(op.relu))
                for nm, dst in ((op.gamma, op.sc), (op.beta, op.sh)):
                    if nm is not None:
                        c_ = self._call("rn_cast", x.c, self._pp(nm), F32, dst, F32, sp)
                        F.append(c_)
                        I.append(c_)
                c_ = self._call("rn_bn_apply", L.C.byref(op.desc), self._p(self.act(x)), self._p(self.act(y)),
                                op.sc, op.sh, sp)
                F.append(c_)
                I.append(c_)
            elif op.kind == "relu":
                c = self._call("rn_eltwise_add", op.x.numel, self.dtype, self._p(self.act(op.x)), None,
                               self._p(self.act(op.y)), 1, sp)
                F.append(c)
                I.append(c)
            elif op.kind == "quant":
                q = op.q
                for o in (op, op.bn_peer):
                    if o is not None and o.emit_codes and getattr(o, "codes", None) is None:
                        # + the int8 codes and unit the consumers' int8 forward reads
                        o.codes = self.torch.zeros(o.x.numel, dtype=self.torch.int8, device=self.device)
                        o.unit = self._zeros(1, self.torch.float32)
                # (codes_wgrad: codes only, the weight gradients multiply them)
                vout = lambda o: None if o.codes_wgrad else self._p(self.act(o.y))
                for lst, tr in ((F, 1), (I, 0)):
                    if op.bn_lead is not None:
                        pass  # written by its peer's call
                    elif op.bn_peer is not None:
                        bn, o2 = op.bn_src, op.bn_peer
                        lst.append(self._call("rn_quant_int8_fwd_codes_bn2", L.C.byref(bn.desc),
                                              self._p(self.act(bn.x)), bn.sc, bn.sh, vout(op),
                                              self._p(op.codes), self._p(op.unit), self._ap(q["minmax"]), q["ema"],
                                              q["nbits"], vout(o2), self._p(o2.codes),
                                              self._p(o2.unit), self._ap(o2.q["minmax"]), o2.q["ema"],
                                              o2.q["nbits"], tr, self._qfirst, qwsp, sp))
                    elif op.bn_src is not None:
                        bn = op.bn_src
                        lst.append(self._call("rn_quant_int8_fwd_codes_bn", L.C.byref(bn.desc),
                                              self._p(self.act(bn.x)), bn.sc, bn.sh, vout(op),
                                              self._p(op.codes), self._p(op.unit), self._ap(q["minmax"]), tr,
                                              q["ema"], self._qfirst, q["nbits"], qwsp, sp))
                    elif op.emit_codes:
                        lst.append(self._call("rn_quant_int8_fwd_codes", self.dtype, op.x.numel,
                                              self._p(self.act(op.x)), vout(op), self._p(op.codes),
                                              self._p(op.unit), self._ap(q["minmax"]), 0, tr, q["ema"],
                                              self._qfirst, q["nbits"], qwsp, sp))
                    else:
                        lst.append(self._call("rn_quant_int8_fwd", self.dtype, op.x.numel, self._p(self.act(op.x)),
                                              self._p(self.act(op.y)), self._ap(q["minmax"]), 0, tr, q["ema"],
                                              self._qfirst, q["nbits"], qwsp, sp))
            elif op.kind == "add" and getattr(op, "bn_a", None) is not None:
                bna, bnb = op.bn_a, op.bn_b
                other = op.b if op.bn_a_key == "a" else op.a
                c = self._call("rn_bn_apply_add", L.C.byref(bna.desc), self._p(self.act(bna.x)), bna.sc, bna.sh,
                               self._p(self.act(bnb.x if bnb is not None else other)),
                               bnb.sc if bnb is not None else None, bnb.sh if bnb is not None else None,
                               self._p(self.act(op.y)), int(op.relu), sp)
                F.append(c)
                I.append(c)
            elif op.kind == "add":
                c = self._call("rn_eltwise_add", op.y.numel, self.dtype, self._p(self.act(op.a)),
                               self._p(self.act(op.b)), self._p(self.act(op.y)), int(op.relu), sp)
                F.append(c)
                I.append(c)
            elif op.kind == "pool":
                x, y = op.x, op.y
                d = L.PoolDesc(dtype=self.dtype, n=x.n, h=x.h, w=x.w, c=x.cp, r=op.kernel[0], s=op.kernel[1],
                               stride_h=op.stride[0], stride_w=op.stride[1], pad_h=op.pad[0], pad_w=op.pad[1],
                               type=L.RN_POOL_MAX if op.type == "max" else L.RN_POOL_AVG,
                               global_pool=int(op.global_pool))
                L.check(self.lib.rn_pool_desc_init(L.C.byref(d)), "rn_pool_desc_init")
                assert (d.p, d.q) == (y.h, y.w), (op.name, d.p, d.q, y.h, y.w)
                op.desc = d
                op.argmax = self.torch.zeros(max(y.rows * y.cp, 1), dtype=self.torch.uint8, device=self.device) \
                    if op.type == "max" else None
                if op.xf is not None:  # the producing BatchNorm+ReLU applied while loading
                    c = self._call("rn_pool_fwd_x", L.C.byref(d), self._p(self.act(op.xf.x)), self._p(self.act(y)),
                                   self._p(op.argmax), op.xf.sc, op.xf.sh, sp)
                else:
                    c = self._call("rn_pool_fwd", L.C.byref(d), self._p(self.act(x)), self._p(self.act(y)),
                                   self._p(op.argmax), sp)
                F.append(c)
                I.append(c)
            elif op.kind == "fc":
                x, y = op.x, op.y
                d = self._conv_desc(x.n, 1, 1, x.cp, x.c, op.nh, (1, 1), (1, 1), (0, 0))
                op.desc = d
                op.wk = self._zeros(op.nh * x.cp, self.tdtype)
                op.wc = self._zeros(x.cp * _pad8(op.nh), self.tdtype)
                self._add_pack(op, d, op.wk, op.wc, sp)
                bias = self._pp(op.bias) if op.bias else None
                c = self._call("rn_conv_fwd", L.C.byref(d), self._p(self.act(x)), self._p(op.wk),
                               self._p(self.act(y)), F32, None, bias, sp)
                F.append(c)
                I.append(c)
            elif op.kind == "softmax":
                x = op.x
                # gradient of the logits is produced here (SoftmaxOutput's backward needs no head grad)
                dl = self.grad_buf(x)
                F.append(self._call("rn_softmax_output", self.dtype, x.n, x.c, x.cp, self._p(self.act(x)),
                                    self._p(self.act(op.label)), self._p(self.act(op.y)), self._p(dl),
                                    op.grad_scale, self._p(self.stats), sp))
                I.append(self._call("rn_softmax_output", self.dtype, x.n, x.c, x.cp, self._p(self.act(x)),
                                    self._p(self.act(op.label)), self._p(self.act(op.y)), None, op.grad_scale,
                                    None, sp))
            self._fwd_train.extend(F)
            self._fwd_infer.extend(I)
        self.stem_ws = self._zeros(stem_ws, self.torch.float32)
        if self._wq_ops:
            items = []
            for op in self._wq_ops:
                shape = self.plan.param_shape(op.weight)
                k, creal = shape[0], shape[1]
                rs = int(np.prod(shape[2:])) if len(shape) > 2 else 1
                i8 = getattr(op, "int8", False)
                d = op.desc if i8 else None
                assert not i8 or (d.groups <= 1 and d.k == k and d.c_real == creal and d.r * d.s == rs)
                items.append(L.WQuantItem(
                    master=self._pp(op.weight).value, qw=op.qw.data_ptr(),
                    unit=op.wunit.data_ptr() if i8 else None, minmax=self._ap(op.qweight["minmax"]).value,
                    w_codes=op.wk8.data_ptr() if i8 else None, w_crsk=op.wc.data_ptr() if i8 else None,
                    k=k, rs=rs, c_real=creal, c=d.c if i8 else creal, k_pad=d.k_pad if i8 else k,
                    nbits=int(op.qweight["nbits"])))
            arr = (L.WQuantItem * len(items))(*items)
            self._wq_items = self.torch.frombuffer(bytearray(arr), dtype=self.torch.uint8).to(self.device)
            c_ = self._call("rn_weight_quant_pack", self._p(self._wq_items), len(items), self.dtype, qwsp, sp)
            self.packs.insert(0, c_)
            self.unfused_packs.insert(0, c_)
        if self._gpacks:
            n = len(self._gpacks)
            vp = lambda v: v.value if isinstance(v, L.C.c_void_p) else v  # noqa: E731
            self._gp_arrays = ((type(self._gpacks[0][0]) * n)(*[g[0] for g in self._gpacks]),
                               (L.C.c_void_p * n)(*[vp(g[1]) for g in self._gpacks]),
                               (L.C.c_void_p * n)(*[g[2].data_ptr() if g[2] is not None else None
                                                    for g in self._gpacks]),
                               (L.C.c_void_p * n)(*[g[3].data_ptr() if g[3] is not None else None
                                                    for g in self._gpacks]))
            self.unfused_packs.append(self._call("rn_conv_weight_pack_multi", *self._gp_arrays, n, sp))

    def _big_tile(self, op, mode, min_cols=None):
        """Does conv `op` run its forward (mode 0) / data gradient (mode 1) on a 256/224-row LDS-DMA
        tile of at least min_cols columns (the BN epilogue fusions run there; the fp64-accumulated
        variant on the 128/256-column tiles only)?"""
        if op.kind != "conv" or self.lib is None:
            return False
        if getattr(op, "int8", False) and mode == 0:  # the int8 forward's tile (its dgrad is the bf16 one)
            x, y = op.x, op.y
            d = self._conv_desc(x.n, x.h, x.w, x.cp, x.c, y.c, op.kernel, op.stride, op.pad, op.groups)
            mc = min_cols if min_cols is not None else 128
            return int(self.lib.rn_conv_tile(L.C.byref(d), 2)) >= mc
        if min_cols is None:  # (64, the 64-column tile too -- RN_BN_FUSION_MIN_COLS -- measured 0.6 % slower per step)
            min_cols = 128
        x, y = op.x, op.y
        d = self._conv_desc(x.n, x.h, x.w, x.cp, x.c, y.c, op.kernel, op.stride, op.pad, op.groups)
        return int(self.lib.rn_conv_tile(L.C.byref(d), mode)) >= min_cols

    def _grouped_fuse(self, op, mode):
        """Does grouped conv `op` carry the BN fusion in its forward (mode 0: the statistics epilogue of
        the block-diagonal 256x64 tile) / data gradient (mode 1: the BN-backward reduction of that tile
        or of the direct kernel, rn_conv_bwd_data_bnred)? RN_GROUPED_BN_FUSION=0: neither (A/B)."""
        if op.kind != "conv" or op.groups <= 1 or self.lib is None or self.dtype != L.RN_BF16 or \
                os.environ.get("RN_GROUPED_BN_FUSION", "1") != "1":
            return False
        x, y = op.x, op.y
        d = self._conv_desc(x.n, x.h, x.w, x.cp, x.c, y.c, op.kernel, op.stride, op.pad, op.groups)
        if mode == 1 and d.grouped_direct == 1:
            return True
        return int(self.lib.rn_conv_tile(L.C.byref(d), mode)) == 64

    def _conv_fwd_call(self, op, d, xptr, res, sp, stats=True):
        """Conv forward; emits the next BatchNorm's statistics when one consumes y (training), and
        applies the producing BatchNorm+ReLU on load when that BN is fused (op.xf)."""
        y = self._p(self.act(op.y))
        if getattr(op, "int8", False):
            part = None
            if stats and op.bnstats:
                if getattr(op, "part", None) is None:
                    op.part_rows = int(self.lib.rn_conv_bn_part_rows(L.C.byref(d), 2))
                    op.part_blocks = -(-op.y.rows // op.part_rows)
                    op.part = self._zeros(op.part_blocks * 3 * op.y.cp, self.torch.float32)
                part = self._p(op.part)
                if op.want_mm:  # + per-block max / min of y for the quantizers that read bn(y)
                    if getattr(op, "part_mm", None) is None:
                        op.part_mm = self._zeros(op.part_blocks * op.y.cp, self.torch.float32)
                    sign = self._pp(op.mm_gamma) if op.mm_gamma else None
                    return self._call("rn_conv_fwd_i8_mm", L.C.byref(d), self._p(op.qsrc.codes), self._p(op.wk8),
                                      y, self.dtype, res, self._p(op.qsrc.unit), self._p(op.wunit), part,
                                      self._p(op.part_mm), sign, sp)
            return self._call("rn_conv_fwd_i8", L.C.byref(d), self._p(op.qsrc.codes), self._p(op.wk8), y,
                              self.dtype, res, self._p(op.qsrc.unit), self._p(op.wunit), part, sp)
        xf = getattr(op, "xf", None)
        sc, sh = (xf.sc, xf.sh) if xf is not None else (None, None)
        part = None
        if stats and op.bnstats:
            if getattr(op, "part", None) is None:
                op.part_blocks = int(self.lib.rn_conv_bnstats_blocks(L.C.byref(d)))
                op.part_rows = int(self.lib.rn_conv_bn_part_rows(L.C.byref(d), 0))
                op.part = self._zeros(op.part_blocks * 3 * op.y.cp, self.torch.float32)
            part = self._p(op.part)
        if sc is None and part is None:
            return self._call("rn_conv_fwd", L.C.byref(d), xptr, self._p(op.wk), y, self.dtype, res, None, sp)
        return self._call("rn_conv_fwd_x", L.C.byref(d), xptr, self._p(op.wk), y, self.dtype, res, None, sc, sh,
                          part, sp)

    def _stem_chunks(self, op, dy):
        """Image chunks of the stem's BN-backward apply + weight gradient (RN_STEM_CHUNKS, default 4;
        1 = one rn_bn_bwd and one wgrad): the NHWC4 stem, or the int8 stem's NHWC-8 image with the clip
        masks (rn_stem_clip_wgrad_chunk), with a side stream, whose output gradient is the dx of the
        rn_bn_bwd call just emitted (no add operand, no paired gradient)."""
        nch = int(os.environ.get("RN_STEM_CHUNKS", "4"))
        side = self._side_stream is not None or (self.dry_run and os.environ.get("RN_WGRAD_STREAM", "1") == "1")
        if nch <= 1 or not (op.p4 or self._stem_clip_mask(op)) or not side or dy is None or op.dfull.n % nch or \
                not self._bwd:
            return 1
        name, _, args = self._bwd[-1]
        # (rn_bn_bwd_part: the pool backward reduced the BN, rn_pool_bwd_bnred)
        dx, add = (args[3], args[4]) if name == "rn_bn_bwd" else (args[5], args[6]) if name == "rn_bn_bwd_part" \
            else (None, None)
        if dx is None or add is not None:
            return 1
        bn = args[0]._obj
        if bn.dy2 or bn.c != op.dfull.k_pad or bn.m != op.dfull.n * op.dfull.p * op.dfull.q or \
                dx.value != self._p(dy).value:
            return 1
        return nch

    def _weight_source(self, op, qwsp, sp):
        """Quantization_int8 on a weight (int8_api.py:131-132): the compute copies are packed from a
        fake-quantized fp32 copy of the master, refreshed with every repack; the STE passes the
        gradient to the master unchanged."""
        q = op.qweight
        n = int(np.prod(self.plan.param_shape(op.weight)))
        op.qw = self._zeros(n, self.torch.float32)
        if getattr(op, "int8", False):  # also keeps the unit for the int8 codes of the forward copy
            op.wunit = self._zeros(1, self.torch.float32)
        if self._wq_batch:
            # one batched rn_weight_quant_pack for every weight quantizer (built after the forward):
            # the fake-quantized copy, and for the int8 convs their codes and data-gradient copy too
            self._wq_ops.append(op)
            return self._p(op.qw)
        if getattr(op, "int8", False):
            c = self._call("rn_quant_int8_fwd_codes", F32, n, self._pp(op.weight), self._p(op.qw), None,
                           self._p(op.wunit), self._ap(q["minmax"]), 1, 1, q["ema"], 0, q["nbits"], qwsp, sp)
        else:
            c = self._call("rn_quant_int8_fwd", F32, n, self._pp(op.weight), self._p(op.qw),
                           self._ap(q["minmax"]), 1, 1, q["ema"], 0, q["nbits"], qwsp, sp)
        self.packs.append(c)
        self.unfused_packs.append(c)
        return self._p(op.qw)

    def _add_pack(self, op, d, wk, wc, sp):
        """Compute copies of op's weight. Dense weights packed straight from the master are
        rewritten by the fused SGD kernel (rn_sgd_mom_update_pack); the bind-time pack below also
        writes their zero padding, which that kernel never touches."""
        c = self._call("rn_conv_weight_pack", L.C.byref(d), op.wsrc, self._p(wk), self._p(wc), sp)
        self.packs.append(c)
        if d.groups == 1 and not getattr(op, "qweight", None) and self.fuse_packs:
            self.fused_packs[op.weight] = (wk.data_ptr() if wk is not None else 0,
                                           wc.data_ptr() if wc is not None else 0,
                                           d.k, d.r * d.s, d.c_real, d.c, d.k_pad)
        elif d.groups > 1 and self._gpack_batch:
            self._gpacks.append((d, op.wsrc, wk, wc))  # -> one rn_conv_weight_pack_multi
        else:
            self.unfused_packs.append(c)

    # ------------------------------------------------------------------ backward
    def _wgrad_call(self, d, x, dy, dw, sp):
        """rn_conv_bwd_filter, through the split-M slab workspace where the kernel uses one."""
        if self.wgrad_ws is not None and int(self.lib.rn_conv_wgrad_ws_bytes(L.C.byref(d))) > 0:
            return self._call("rn_conv_bwd_filter_ws", L.C.byref(d), x, dy, dw, self._p(self.wgrad_ws),
                              self.wgrad_ws_bytes, sp)
        return self._call("rn_conv_bwd_filter", L.C.byref(d), x, dy, dw, sp)

    def _quant_groups(self):
        """{id(bn): (bn, [quant ops])} for the BatchNorm+ReLU outputs that only activation quantizers
        (Quantization_int8 of data, the int8 graph) read -- one, or two (symbol/resnet_int8.py: a stage's
        first unit quantizes act1 for conv1 and for the shortcut conv). Their straight-through backwards
        (zero where the input is >= the moving threshold, clip_grad_quantization_int8.py) fold into that
        BN's backward (rn_bn_desc.clip, and clip2 / dy2 for the second), so the quantizers cost no
        backward pass, and their forwards apply the BN on load (rn_quant_int8_fwd_codes_bn[2]): the BN
        output is never written. RN_QUANT_BWD_FOLD=0: separate rn_quant_int8_bwd passes."""
        if os.environ.get("RN_QUANT_BWD_FOLD", "1") != "1":
            return {}
        ops = self.plan.ops
        readers, qreaders = {}, {}
        for o in ops:
            for k in ("x", "a", "b", "res", "label"):
                t = getattr(o, k, None)
                if isinstance(t, TensorSpec):
                    readers[id(t)] = readers.get(id(t), 0) + 1
                    if o.kind == "quant" and k == "x" and not o.q.get("is_weight"):
                        qreaders.setdefault(id(t), []).append(o)
        outs = {id(t) for t in self.plan.outputs}
        groups = {}
        for bn in ops:
            if bn.kind != "bn" or not bn.relu or id(bn.y) in outs or getattr(bn, "apply_fused", False):
                continue
            qs = qreaders.get(id(bn.y), [])
            if qs and len(qs) == readers.get(id(bn.y)) and len(qs) <= 2:
                groups[id(bn)] = (bn, qs)
        return groups

    def _quant_folds(self):
        """{id(quant op): bn op} over _quant_groups (the quantizers whose backward folds into a BN's)."""
        return {id(q): bn for bn, qs in self._quant_groups().values() for q in qs}

    def _build_backward(self):
        plan = self.plan
        sp = self._sp()
        gs = _GradState(self)
        groups = self._quant_groups()
        folds = {id(q): bn for bn, qs in groups.values() for q in qs}
        for op in plan.ops:
            if op.kind == "bn":
                op.qpair = False
                op.qorder = []  # the folded quantizers in backward order (their gradients' pending order)
        for bn, qs in groups.values():
            if len(qs) == 1:
                bn.desc.clip = self._ap(qs[0].q["minmax"]).value  # (the threshold the forward just updated)
            else:
                bn.qpair = True  # clip / clip2 / dy2 set where its backward is bound
        wsp = self._p(self.ws)
        self.param_done_at = {}  # param -> index in self._bwd after which its grad is final
        self._gw = {}  # id(tensor) -> last writer of its gradient buffer: ("dgrad", call index, conv op)
        # default on where the dgrad runs the 256-row tile (see RN_BN_EPILOGUE_STATS; =2: every dgrad)
        for op in plan.ops:
            if op.kind == "bn":
                op.pre_part = None  # set by the residual add's fused ReLU backward (this build)
        bwd_fusion = os.environ.get("RN_BN_BWD_FUSION", "1") in ("1", "2")
        bwd_all = os.environ.get("RN_BN_BWD_FUSION", "1") == "2"
        # (removed in round 6, each measured slower or neutral, their kernels kept and kernel-tested: the BN backward
        # applied by a recomputed dgrad, RN_BN_BWD_RECOMPUTE -- rn_conv_bwd_data_bnapply; 19.78 vs 19.43 ms with the
        # streamed conv1 data gradients --, and a quantizer pair's clips folded into the later data gradient,
        # RN_QUANT_PAIR_FUSION -- rn_conv_bwd_data_bnred_clip2; C5 22.68 / 22.69 vs 22.69 / 22.68 ms)
        # one workspace for the weight gradients' split-M partial tiles (rn_conv_bwd_filter_ws),
        # sized for the largest layer. Shared safely because every call using it is a weight-gradient
        # call, and those all run in plan order on ONE stream (the side stream when it is on:
        # _route_wgrads enforces this)
        self.wgrad_ws, self.wgrad_ws_bytes = None, 0
        if os.environ.get("RN_WGRAD_SLAB", "1") == "1":
            def need_now():
                need = [int(self.lib.rn_conv_wgrad_ws_bytes(L.C.byref(op.desc))) for op in plan.ops
                        if op.kind in ("conv", "fc") and getattr(op, "desc", None) is not None]
                # (the stem's weight gradient; it needs a slab only in the deterministic mode)
                need += [int(self.lib.rn_conv_wgrad_ws_bytes(L.C.byref(op.dfull))) for op in plan.ops
                         if op.kind == "stem" and not op.p4]
                need += [int(self.lib.rn_stem_clip_wgrad_ws_bytes(L.C.byref(op.dfull))) for op in plan.ops
                         if op.kind == "stem" and self._stem_clip_mask(op)]
                need += [int(self.lib.rn_conv_wgrad_i8_ws_bytes(L.C.byref(op.desc))) for op in plan.ops
                         if op.kind == "conv" and getattr(op, "qsrc", None) is not None and op.qsrc.codes_wgrad]
                return max(need + [0])
            # sized for both weight-gradient grids: the overlapped one (part of the chip) and the whole
            # chip, which a serialised step (side_enabled False: bench.py's calibration) runs with
            overlapped = os.environ.get("RN_WGRAD_STREAM", "1") == "1"
            self.wgrad_ws_bytes = need_now()
            if overlapped:
                L.set_wgrad_split(False)
                self.wgrad_ws_bytes = max(self.wgrad_ws_bytes, need_now())
                L.set_wgrad_split(True, self.wgrad_split_pct)
            if self.wgrad_ws_bytes > 0:
                self.wgrad_ws = self._zeros(self.wgrad_ws_bytes // 4, self.torch.float32)
        for op in plan.ops:
            if op.kind == "stem" and self._stem_clip_mask(op):
                # the int8 stem's clip masks into the NHWC-8 image's free channels (rn_stem_clip_mask),
                # first on the weight-gradient stream: its clip gradient then rides in the stem's weight
                # gradient (rn_stem_clip_wgrad / rn_stem_clip_dbeta) instead of a gather at the step's end
                _, _, sc, sh = op.bn_ptrs
                op.clip_ext = self._zeros(op.dfull.k * op.dfull.r * op.dfull.s * 2 * op.dfull.c_real,
                                          self.torch.float32)
                self._bwd.append(self._call("rn_stem_clip_mask", L.C.byref(op.dfull), self._in_ptr, sc, sh,
                                            self._ap(op.quant["minmax"]), self._p(op.x8), sp))
        for op in reversed(plan.ops):
            if op.kind == "softmax":
                gs.has_value.add(id(op.x))  # dlogits written by the forward softmax call
                continue
            if op.kind == "bn" and op.qpair:
                # two folded quantizers: their output gradients stay separate (dy, rn_bn_desc.dy2)
                assert id(op.y) not in gs.has_value
                pend = gs.pending.pop(id(op.y), [])
                if not pend:
                    continue
                dy = pend[0]
                op.desc.clip = self._ap(op.qorder[0].q["minmax"]).value
                if len(pend) == 2:
                    op.desc.clip2 = self._ap(op.qorder[1].q["minmax"]).value
                    op.desc.dy2 = self._p(pend[1]).value
            else:
                dy = gs.read(op.y) if op.kind != "softmax" else None
            if dy is None:
                continue
            if op.kind == "fc":
                x = op.x
                self._bwd.append(self._wgrad_call(op.desc, self._p(self.act(x)), self._p(dy), self._gp(op.weight), sp))
                if op.bias:
                    self._bwd.append(self._call("rn_col_sum", self.dtype, x.n, op.nh, _pad8(op.nh), self._p(dy),
                                                self._gp(op.bias), 0, sp))
                    self.param_done_at[op.bias] = len(self._bwd)
                self.param_done_at[op.weight] = len(self._bwd)
                if x.needs_grad:
                    out, add = gs.contribute(x)
                    self._bwd.append(self._call("rn_conv_bwd_data", L.C.byref(op.desc), self._p(dy), self._p(op.wc),
                                                self._p(out), self._p(add), sp))
            elif op.kind == "conv":
                x = op.x
                if op.xf is not None:  # input = BN+ReLU(bn input), applied on load
                    ws = self.wgrad_ws is not None and int(self.lib.rn_conv_wgrad_ws_bytes(L.C.byref(op.desc))) > 0
                    self._bwd.append(self._call("rn_conv_bwd_filter_x", L.C.byref(op.desc), self._p(self.act(op.xf.x)),
                                                self._p(dy), self._gp(op.weight), op.xf.sc, op.xf.sh,
                                                self._p(self.wgrad_ws) if ws else None,
                                                self.wgrad_ws_bytes if ws else 0, sp))
                elif getattr(op, "qsrc", None) is not None and op.qsrc.codes_wgrad:  # the input's codes, x its unit
                    q, ws = op.qsrc, self.wgrad_ws is not None
                    self._bwd.append(self._call("rn_conv_bwd_filter_i8", L.C.byref(op.desc), self._p(q.codes),
                                                self._p(q.unit), self._p(dy), self._gp(op.weight),
                                                self._p(self.wgrad_ws) if ws else None,
                                                self.wgrad_ws_bytes if ws else 0, sp))
                else:
                    self._bwd.append(self._wgrad_call(op.desc, self._p(self.act(x)), self._p(dy), self._gp(op.weight),
                                                      sp))
                self.param_done_at[op.weight] = len(self._bwd)
                if x.needs_grad:
                    out, add = gs.contribute(x)
                    self._bwd.append(self._call("rn_conv_bwd_data", L.C.byref(op.desc), self._p(dy), self._p(op.wc),
                                                self._p(out), self._p(add), sp))
                    self._gw[id(x)] = ("dgrad", len(self._bwd) - 1, op, dy, out, add)
                if op.res is not None and op.res.needs_grad:
                    gs.alias(op.res, dy)
            elif op.kind == "stem":
                nch = self._stem_chunks(op, dy)
                if nch > 1:
                    # the stem BN's dx (= dy here) per image chunk, each chunk's weight gradient (side
                    # stream) starting as soon as its rows are applied: only the last chunk's wgrad
                    # stays on the step's critical path (rn_bn_bwd then reduces + finalizes only)
                    bname, bfn, bargs = self._bwd[-1]
                    if bname == "rn_bn_bwd":
                        self._bwd[-1] = (bname, bfn, bargs[:3] + (None,) + bargs[4:])
                    else:  # rn_bn_bwd_part: finalize only, its coefficients where rn_bn_bwd_apply_rows reads
                        # them (after the reduction partials of rn_bn_bwd's own layout in the workspace)
                        bd, part, nrb, xp_, dyp_, dxp_, _, gp_, smp, sip, scp, shp, dgp, dbp, wsp_, _ = bargs
                        coef = wsp_.value + 4 * 2 * int(self.lib.rn_bn_reduce_blocks(bd)) * bd._obj.c
                        self._bwd[-1] = self._call("rn_bn_bwd_finalize", bd, part, nrb, gp_, smp, sip, dgp, dbp,
                                                   L.C.c_void_p((coef + 15) // 16 * 16), sp)
                        bargs = (bd, xp_, dyp_, dxp_, None, gp_, smp, sip, scp, shp, dgp, dbp, wsp_, sp)
                    d = op.dfull
                    nc = d.n // nch
                    rows = nc * d.p * d.q
                    for i in range(nch):
                        dc = self._conv_desc(nc, d.h, d.w, d.c, d.c_real, d.k, (d.r, d.s), (d.stride_h, d.stride_w),
                                             (d.pad_h, d.pad_w))
                        self._descs.append(dc)
                        self._bwd.append(self._call("rn_bn_bwd_apply_rows", bargs[0], bargs[1], bargs[2], bargs[3],
                                                    None, bargs[8], bargs[9], bargs[12], i * rows, rows, sp))
                        dyc = L.C.c_void_p(self._p(dy).value + i * rows * d.k_pad * 2)
                        if op.p4:
                            hp, wp = op.p4
                            self._bwd.append(self._call(
                                "rn_stem_conv_wgrad_p4", L.C.byref(dc),
                                L.C.c_void_p(op.x8.data_ptr() + i * nc * hp * wp * 4 * 2), dyc, self._gp(op.weight),
                                hp, wp, sp))
                        else:  # the int8 stem: NHWC-8 chunks, clip masks in channels c_real..
                            ws = self.wgrad_ws is not None
                            self._bwd.append(self._call(
                                "rn_stem_clip_wgrad_chunk", L.C.byref(dc),
                                L.C.c_void_p(op.x8.data_ptr() + i * nc * d.h * d.w * 8 * 2), dyc, self._gp(op.weight),
                                self._p(op.clip_ext), self._p(self.wgrad_ws) if ws else None,
                                self.wgrad_ws_bytes if ws else 0, int(i == 0), int(i == nch - 1), sp))
                elif op.p4:
                    self._bwd.append(self._call("rn_stem_conv_wgrad_p4", L.C.byref(op.dfull), self._p(op.x8),
                                                self._p(dy), self._gp(op.weight), op.p4[0], op.p4[1], sp))
                elif self._stem_clip_mask(op):
                    ws = self.wgrad_ws is not None
                    self._bwd.append(self._call("rn_stem_clip_wgrad", L.C.byref(op.dfull), self._p(op.x8),
                                                self._p(dy), self._gp(op.weight), self._p(op.clip_ext),
                                                self._p(self.wgrad_ws) if ws else None,
                                                self.wgrad_ws_bytes if ws else 0, sp))
                else:
                    self._bwd.append(self._wgrad_call(op.dfull, self._p(op.x8), self._p(dy), self._gp(op.weight), sp))
                self.param_done_at[op.weight] = len(self._bwd)
                if op.bn:
                    self._bwd.append(self._call("rn_stem_shift_grad", L.C.byref(op.dfull), self._p(dy),
                                                op.wsrc, self._gp(op.bn["beta"]), self._p(self.stem_ws), sp))
                    if op.quant and self._stem_clip_mask(op):
                        self._bwd.append(self._call("rn_stem_clip_dbeta", L.C.byref(op.dfull), self._p(op.clip_ext),
                                                    op.wsrc, self._gp(op.bn["beta"]), sp))
                    elif op.quant:
                        _, _, sc, sh = op.bn_ptrs
                        self._bwd.append(self._call("rn_stem_quant_clip_grad", L.C.byref(op.dfull),
                                                    self._in_ptr, sc, sh, self._ap(op.quant["minmax"]),
                                                    self._p(dy), op.wsrc, self._gp(op.bn["beta"]), sp))
                    self.param_done_at[op.bn["beta"]] = len(self._bwd)
                    self.param_done_at[op.bn["gamma"]] = len(self._bwd)
            elif op.kind == "bn":
                x = op.x
                out, add = (gs.contribute(x) if x.needs_grad else (None, None))
                w = self._gw.get(id(op.y))
                if op.use_global_stats:
                    # moving statistics are constants of the graph (fix_bn): dx = gamma*invstd*dz
                    self._bwd.append(self._call("rn_bn_bwd_global", L.C.byref(op.desc), self._p(self.act(x)),
                                                self._p(dy), self._p(out), self._p(add), self._pp(op.gamma),
                                                self._ap(op.mean), self._ap(op.var), op.sc, op.sh,
                                                self._gp(op.gamma), self._gp(op.beta), wsp, sp))
                elif bwd_fusion and not op.desc.dy2 and w and w[0] == "dgrad" and dy is w[4] and \
                        op.y.c % 8 == 0 and op.y.c == op.y.cp and \
                        (bwd_all or self._big_tile(w[2], 1) or self._grouped_fuse(w[2], 1)) and \
                        (not op.desc.clip or self._big_tile(w[2], 1)):  # (the clip: bf16 LDS-DMA tiles)
                    # the conv dgrad that completes this BN's output gradient also reduces its backward
                    # (sum dz, sum dz*(x - mean)); the BN then needs only finalize + apply
                    _, ci, cop, cdy, cout, cadd = w
                    op.bnred_blocks = int(self.lib.rn_conv_bnred_blocks(L.C.byref(cop.desc)))
                    op.bnred = self._zeros(op.bnred_blocks * op.y.cp * 2, self.torch.float32)
                    if op.desc.clip:  # (a folded quantizer straight-through clip)
                        self._bwd[ci] = self._call("rn_conv_bwd_data_bnred_clip", L.C.byref(cop.desc),
                                                   self._p(cdy), self._p(cop.wc), self._p(cout), self._p(cadd),
                                                   self._p(self.act(x)), op.sm, op.sc, op.sh, int(op.relu),
                                                   L.C.c_void_p(op.desc.clip), self._p(op.bnred), sp)
                    else:
                        self._bwd[ci] = self._call("rn_conv_bwd_data_bnred", L.C.byref(cop.desc), self._p(cdy),
                                                   self._p(cop.wc), self._p(cout), self._p(cadd),
                                                   self._p(self.act(x)), op.sm, op.sc, op.sh, int(op.relu),
                                                   self._p(op.bnred), sp)
                    self._bwd.append(self._call("rn_bn_bwd_part", L.C.byref(op.desc), self._p(op.bnred),
                                                op.bnred_blocks, self._p(self.act(x)), self._p(dy), self._p(out),
                                                self._p(add), self._pp(op.gamma), op.sm, op.si, op.sc, op.sh,
                                                self._gp(op.gamma), self._gp(op.beta), wsp, sp))
                elif bwd_fusion and not op.desc.dy2 and not op.desc.clip and w and w[0] == "pool" and dy is w[4] and \
                        op.y.c == op.y.cp and self.dtype == BF16 and os.environ.get("RN_POOL_BN_FUSION", "1") == "1" and \
                        int(self.lib.rn_pool_bwd_bnred_blocks(L.C.byref(w[2].desc))) > 0:
                    # the max-pool backward that completes this BN's output gradient (the stem's bn0 ->
                    # relu0 -> pool0) also reduces its backward; the BN then needs only finalize + apply
                    _, pi, pop, pdy, pout, padd = w
                    op.bnred_blocks = int(self.lib.rn_pool_bwd_bnred_blocks(L.C.byref(pop.desc)))
                    op.bnred = self._zeros(op.bnred_blocks * op.y.cp * 2, self.torch.float32)
                    self._bwd[pi] = self._call("rn_pool_bwd_bnred", L.C.byref(pop.desc), self._p(pdy),
                                               self._p(pop.argmax), self._p(pout), self._p(padd),
                                               self._p(self.act(x)), op.sm, op.sc, op.sh, int(op.relu),
                                               self._p(op.bnred), sp)
                    self._bwd.append(self._call("rn_bn_bwd_part", L.C.byref(op.desc), self._p(op.bnred),
                                                op.bnred_blocks, self._p(self.act(x)), self._p(dy), self._p(out),
                                                self._p(add), self._pp(op.gamma), op.sm, op.si, op.sc, op.sh,
                                                self._gp(op.gamma), self._gp(op.beta), wsp, sp))
                elif getattr(op, "pre_part", None) is not None and not op.desc.dy2:
                    # the reduction was done by the residual add's ReLU backward (rn_relu_bwd_bnred)
                    self._bwd.append(self._call("rn_bn_bwd_part", L.C.byref(op.desc), self._p(op.pre_part),
                                                op.pre_nrb, self._p(self.act(x)), self._p(dy), self._p(out),
                                                self._p(add), self._pp(op.gamma), op.sm, op.si, op.sc, op.sh,
                                                self._gp(op.gamma), self._gp(op.beta), wsp, sp))
                else:
                    self._bwd.append(self._call("rn_bn_bwd", L.C.byref(op.desc), self._p(self.act(x)), self._p(dy),
                                                self._p(out), self._p(add), self._pp(op.gamma), op.sm, op.si, op.sc,
                                                op.sh, self._gp(op.gamma), self._gp(op.beta), wsp, sp))
                self.param_done_at[op.gamma] = len(self._bwd)
                self.param_done_at[op.beta] = len(self._bwd)
            elif op.kind == "affine":
                # the global-statistics BN backward with mean 0, variance 1, eps 0: dz = dy*[y > 0],
                # dscale = sum(dz*x), dbias = sum(dz), dx = scale*dz
                x = op.x
                out, add = (gs.contribute(x) if x.needs_grad else (None, None))
                if op.gamma is None or op.beta is None:
                    op.gscratch = self._zeros(x.cp, self.torch.float32)
                dg = self._gp(op.gamma) if op.gamma is not None else self._p(op.gscratch)
                db = self._gp(op.beta) if op.beta is not None else self._p(op.gscratch)
                self._bwd.append(self._call("rn_bn_bwd_global", L.C.byref(op.desc), self._p(self.act(x)),
                                            self._p(dy), self._p(out), self._p(add), op.sc, op.zero, op.one,
                                            op.sc, op.sh, dg, db, wsp, sp))
                for nm in (op.gamma, op.beta):
                    if nm is not None:
                        self.param_done_at[nm] = len(self._bwd)
            elif op.kind == "quant":
                if op.x.needs_grad and id(op) in folds:
                    # straight-through: the gradient passes unchanged to the BN output, whose backward
                    # applies the clip; the conv that wrote dy stays its last writer (BN reduction fusion)
                    gs.alias(op.x, dy)
                    bn = folds[id(op)]
                    bn.qorder.append(op)
                    if bn.qpair:
                        self._gw[id(op.x)] = ("other",)
                    elif id(op.y) in self._gw:
                        self._gw[id(op.x)] = self._gw[id(op.y)]
                elif op.x.needs_grad:
                    out, add = gs.contribute(op.x)
                    self._bwd.append(self._call("rn_quant_int8_bwd", self.dtype, op.x.numel, self._p(self.act(op.x)),
                                                self._p(dy), self._p(out), self._ap(op.q["minmax"]), 0, self._p(add),
                                                sp))
            elif op.kind == "relu":
                if op.x.needs_grad:
                    out, add = gs.contribute(op.x)
                    self._bwd.append(self._call("rn_relu_bwd", op.y.numel, self.dtype, self._p(self.act(op.y)),
                                                self._p(dy), self._p(out), self._p(add), sp))
            elif op.kind == "add":
                g = dy
                if op.relu:
                    # held by the executor: the bound call keeps only the raw pointer (a dropped
                    # tensor would be recycled by the caching allocator while the plan writes it)
                    gbuf = self._zeros(op.y.numel, self.tdtype)
                    self._grads[("relu_add", id(op))] = gbuf
                    # the BatchNorms applied inside this add (rn_bn_apply_add) get their backward
                    # reductions from the same pass (rn_relu_bwd_bnred)
                    bns = [b for b in (getattr(op, "bn_a", None), getattr(op, "bn_b", None))
                           if b is not None and not b.use_global_stats and dy is not None]
                    # (round 4's opt-in RN_RELU_BNRED_DGRAD -- this pass in the next unit's conv1 data-gradient
                    # epilogue -- measured 3 % slower on C4 and was removed in round 5: the epilogue streamed
                    # its extra tensors at ~3.5 TB/s, this pass runs at ~5.5)
                    if bns and len(bns) == len([b for b in (op.bn_a, op.bn_b) if b is not None]):
                        for b in bns:
                            b.pre_nrb = int(self.lib.rn_bn_reduce_blocks(L.C.byref(b.desc)))
                            b.pre_part = self._zeros(b.pre_nrb * b.x.cp * 2, self.torch.float32)
                        b2 = bns[1] if len(bns) == 2 else None
                        self._bwd.append(self._call(
                            "rn_relu_bwd_bnred", L.C.byref(bns[0].desc), self._p(self.act(op.y)), self._p(dy),
                            self._p(gbuf), self._p(self.act(bns[0].x)), bns[0].sm, self._p(bns[0].pre_part),
                            self._p(self.act(b2.x)) if b2 else None, b2.sm if b2 else None,
                            self._p(b2.pre_part) if b2 else None, sp))
                    else:
                        self._bwd.append(self._call("rn_relu_bwd", op.y.numel, self.dtype, self._p(self.act(op.y)),
                                                    self._p(dy), self._p(gbuf), None, sp))
                    g = gbuf
                for t in (op.a, op.b):
                    if t.needs_grad:
                        gs.alias(t, g)
            elif op.kind == "pool":
                x = op.x
                if x.needs_grad:
                    out, add = gs.contribute(x)
                    self._bwd.append(self._call("rn_pool_bwd", L.C.byref(op.desc), self._p(dy), self._p(op.argmax),
                                                self._p(out), self._p(add), sp))
                    self._gw[id(x)] = ("pool", len(self._bwd) - 1, op, dy, out, add)

    # ------------------------------------------------------------------ update
    def _build_update(self):
        self.wpack_calls = list(self.packs)
        self.opt_packs = None
        if self.fused_packs:
            dt = np.dtype([("krsc", "<u8"), ("crsk", "<u8"), ("k", "<i4"), ("rs", "<i4"), ("creal", "<i4"),
                           ("c", "<i4"), ("kpad", "<i4"), ("pad", "<i4")])
            tab = np.zeros(len(self.param_order), dtype=dt)
            for i, nm in enumerate(self.param_order):
                e = self.fused_packs.get(nm)
                if e is not None:
                    tab[i] = e + (0,)
            nums = np.array([int(np.prod(self.param_shape[n])) for n in self.param_order], dtype=np.int64)
            cap = int(sum((n + 4095) // 4096 for n in nums) + sum(
                ((e[2] + 63) // 64) * e[3] * ((e[4] + 63) // 64) for e in self.fused_packs.values()))
            work = np.zeros((cap, 4), dtype=np.int32)
            nwork = self.lib.rn_sgd_pack_work(len(nums), nums.ctypes.data_as(L.C.c_void_p),
                                              tab.ctypes.data_as(L.C.c_void_p), work.ctypes.data_as(L.C.c_void_p),
                                              cap)
            if nwork < 0:
                raise L.RNError("rn_sgd_pack_work: %s" % self.lib.rn_last_error().decode())
            self.opt_packs = self.torch.from_numpy(tab.view(np.uint8).copy()).to(self.device)
            self.opt_work = self.torch.from_numpy(work[:nwork].copy()).to(self.device)
            self.opt_nwork = int(nwork)

    # ------------------------------------------------------------------ running
    def _run(self, calls):
        if self.dry_run:  # the plan only (CPU tests): nothing is launched
            return
        for name, fn, args in calls:
            r = fn(*args)
            if r != 0:
                raise L.RNError("%s: %s" % (name, self.lib.rn_last_error().decode()))

    def set_input(self, data_np, label_np=None):
        """H2D copy of one batch (host numpy / torch) into the data/label buffers.

        A pinned host batch (mx.nd.array(..., ctx=cpu_pinned), data/imagenet.py:17-18) is copied
        asynchronously on a separate copy stream into the buffer the previous step is NOT using;
        the compute stream waits only for that copy. Because the host enqueues a whole step ahead of
        the GPU, step t+1's PCIe transfer overlaps step t's backward."""
        torch = self.torch
        t = self.plan.data_tensor
        src = torch.as_tensor(np.ascontiguousarray(data_np, dtype=np.float32)) if isinstance(data_np, np.ndarray) \
            else data_np
        src = src.reshape(-1)
        if src.dtype != torch.float32:
            src = src.to(torch.float32)
        if not self.dry_run and src.device.type == "cpu" and src.is_pinned():
            i = self._in_idx ^ 1
            if self._in_bufs[i] is None:
                self._in_bufs[i] = self._zeros(t.numel, torch.float32)
                self._copy_stream = torch.cuda.Stream(self.device)
            cs = self._copy_stream
            if self._in_free[i] is not None:
                cs.wait_event(self._in_free[i])  # the step that last read this buffer has finished
            with torch.cuda.stream(cs):
                self._in_bufs[i].copy_(src, non_blocking=True)
                done = torch.cuda.Event()
                done.record(cs)
            torch.cuda.current_stream(self.device).wait_event(done)
            self._in_idx = i
            self._in_ptr.value = self._in_bufs[i].data_ptr()
        else:
            self._in_bufs[self._in_idx].copy_(src, non_blocking=True)
        if label_np is not None:
            for tt in self.plan.tensors.values():
                if tt.kind == "label":
                    lsrc = torch.as_tensor(np.ascontiguousarray(label_np, dtype=np.float32)) \
                        if isinstance(label_np, np.ndarray) else label_np
                    self.act(tt).copy_(lsrc.reshape(-1).to(torch.float32), non_blocking=True)

    def _mark_input_read(self):
        if not self.dry_run and self._in_bufs[1] is not None:
            ev = self.torch.cuda.Event()
            ev.record(self.torch.cuda.current_stream(self.device))
            self._in_free[self._in_idx] = ev

    def forward(self, is_train=True):
        self._sync_stream()
        self._run(self._fwd_train if is_train else self._fwd_infer)
        if is_train:
            self._qfirst.value = 0
        self._mark_input_read()

    def backward(self, hooks=None):
        self._sync_stream()
        self.grad.zero_()
        side = self._side_stream if (self._side_idx and self.side_enabled) else None
        if not hooks and side is None:
            self._run(self._bwd)
            self._mark_input_read()
            return
        # hooks: {bwd index -> callable}, e.g. RCCL bucket all-reduce launches; with the wgrad side
        # stream a hook runs on it after a fork, so its collective follows both streams' writes
        hooks = hooks or {}
        forked = False
        for i, (name, fn, args) in enumerate(self._bwd):
            if side is not None and i in self._side_idx and (not forked or i not in self._side_pre):
                self._fork(i)  # (the first side call of the step waits for the forward too)
                forked = True
            r = 0 if self.dry_run else fn(*args)
            if r != 0:
                raise L.RNError("%s: %s" % (name, self.lib.rn_last_error().decode()))
            h = hooks.get(i + 1)
            if h is not None:
                if side is not None:
                    self._fork(("hook", i))
                    with self.torch.cuda.stream(side):
                        h()
                else:
                    h()
        if side is not None:
            self._join()
        self._mark_input_read()

    def repack_weights(self):
        self._sync_stream()
        self._run(self.wpack_calls)

    def sgd_update(self, lr, wd, momentum, rescale_grad, clip=-1.0):
        self._sync_stream()
        if self.dry_run:
            return
        if self._wd_value != wd:
            self.opt_wds.copy_(self.torch.from_numpy(self.wd_mult * np.float32(wd)))
            self._wd_value = wd
        if self.opt_packs is not None:
            L.check(self.lib.rn_sgd_mom_update_pack(len(self.param_order), self._p(self.opt_offsets),
                                                    self._p(self.opt_numels), self._p(self.opt_wds),
                                                    self._p(self.master), self._p(self.grad), self._p(self.mom),
                                                    self._p(self.opt_packs), self._p(self.opt_work),
                                                    self.opt_nwork, self.dtype, float(lr), None,
                                                    float(momentum), float(rescale_grad), float(clip), self._sp()),
                    "rn_sgd_mom_update_pack")
            self._run(self.unfused_packs)
            return
        L.check(self.lib.rn_sgd_mom_update(len(self.param_order), self._p(self.opt_offsets),
                                           self._p(self.opt_numels), self._p(self.opt_wds), self._p(self.master),
                                           self._p(self.grad), self._p(self.mom), None, F32, float(lr), None,
                                           float(momentum), float(rescale_grad), float(clip), self._sp()),
                "rn_sgd_mom_update")
        self.repack_weights()

    # ------------------------------------------------------------------ param I/O (MXNet layouts)
    def set_param(self, name, value):
        v = np.asarray(value, dtype=np.float32)
        if tuple(v.shape) != self.param_shape[name]:
            raise ValueError("shape mismatch for %s: %s vs %s" % (name, v.shape, self.param_shape[name]))
        if self.param_layout[name] == "krsc":
            v = v.transpose(0, 2, 3, 1)
        self.pview(name).copy_(self.torch.from_numpy(np.ascontiguousarray(v).reshape(-1)))

    def get_param(self, name, grad=False):
        src = self.gview(name) if grad else self.pview(name)
        shp = self.param_shape[name]
        v = src.detach().cpu().numpy()
        if self.param_layout[name] == "krsc":
            k, c, r, s = shp
            return v.reshape(k, r, s, c).transpose(0, 3, 1, 2).copy()
        return v.reshape(shp).copy()

    def set_aux(self, name, value):
        v = np.asarray(value, dtype=np.float32).reshape(-1)
        self.aview(name).copy_(self.torch.from_numpy(v))

    def get_aux(self, name):
        o, shp = self.aux_off[name]
        return self.aview(name).detach().cpu().numpy().reshape(shp).copy()

    def output(self, i=0):
        t = self.plan.outputs[i]
        a = self.act(t)
        if t.kind == "prob":
            return a.view(t.n, t.c)
        return a

    # ------------------------------------------------------------------ gradient buckets
    def buckets(self):
        """[(start, end, last_bwd_index)] over the flat grad buffer: ~bucket_bytes each, except the trailing
        bucket -- the longest suffix of the parameter order (the earliest layers, whose gradients are final
        last) within tail_bucket_bytes -- which stands alone so that little is left to sum once the backward
        has ended (core/solver.py:116-121: the kvstore push of the last gradients)."""
        out = []
        order = list(self.param_order)
        sizes = [int(np.prod(self.param_shape[nm])) for nm in order]
        tail_at = len(order)
        tb = getattr(self, "tail_bucket_bytes", 0)
        acc = 0
        while tail_at > 0 and (acc + sizes[tail_at - 1]) * 4 <= tb:
            tail_at -= 1
            acc += sizes[tail_at]
        if tail_at == 0 or acc == 0:
            tail_at = len(order)  # (everything within the tail size, or nothing fits: the plain plan)
        cur_start, cur_end, cur_last = None, None, 0
        for k, nm in enumerate(order):
            o = self.param_off[nm]
            n = sizes[k]
            last = self.param_done_at.get(nm, len(self._bwd))
            if k == tail_at and cur_start is not None:  # close the head before the trailing bucket
                out.append((cur_start, o, cur_last))
                cur_start = None
            if cur_start is None:
                cur_start, cur_end, cur_last = o, o + n, last
            else:
                cur_end, cur_last = o + n, max(cur_last, last)
            if k < tail_at and (cur_end - cur_start) * 4 >= self.bucket_bytes:
                out.append((cur_start, cur_end, cur_last))
                cur_start = None
        if cur_start is not None:
            out.append((cur_start, self.nparam, max(cur_last, 0)))
        # a bucket may only launch after every earlier bucket's params are final too
        fixed, run = [], 0
        for s, e, last in out:
            run = max(run, last)
            fixed.append((s, e, run))
        return fixed
