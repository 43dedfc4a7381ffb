"""mx.sym / mx.symbol: a small symbolic graph IR with MXNet's construction surface.

Mirrors what the reference's graph files call (symbol/resnet.py, resnext.py, resnet_int8.py,
int8_api.py, core/graph_optimize.py): op constructors with string-serialisable attrs,
auto-created parameter Variables named `<name>_<arg>`, Symbol.__add__, _set_attr/attr,
infer_shape, list_arguments/outputs/auxiliary_states, get_internals, tojson/load_json.
Execution happens in resnet.mxnet_amd/rn/executor.py, which lowers this IR onto librn.
"""
import ast
import json

from .base import MXNetError

# ----------------------------------------------------------------------------- naming
_name_counter = {}


def _auto_name(hint):
    hint = hint.lower()
    i = _name_counter.get(hint, 0)
    _name_counter[hint] = i + 1
    return "%s%d" % (hint, i)


def _parse(v):
    """Attribute value (python or MXNet string form) -> python value."""
    if not isinstance(v, str):
        return v
    s = v.strip()
    if s in ("True", "true"):
        return True
    if s in ("False", "false"):
        return False
    if s in ("None", "none"):
        return None
    try:
        return ast.literal_eval(s)
    except (ValueError, SyntaxError):
        return s


def _tup(v, n=2):
    v = _parse(v)
    if v is None:
        return None
    if isinstance(v, int):
        return (v,) * n
    return tuple(int(x) for x in v)


class _Node:
    __slots__ = ("op", "name", "attrs", "inputs", "user_attrs", "nout")

    def __init__(self, op, name, attrs=None, inputs=None, nout=1):
        self.op = op
        self.name = name
        self.attrs = dict(attrs or {})
        self.inputs = list(inputs or [])  # list of (node, out_idx)
        self.user_attrs = {}
        self.nout = nout

    def attr(self, key, default=None):
        return _parse(self.attrs.get(key, default))


# ----------------------------------------------------------------------------- op registry
class OpSpec:
    def __init__(self, name, args, aux=(), hint=None, param_args=None):
        self.name = name
        self.args = args          # callable(attrs) -> list of input arg names, or list
        self.aux = aux            # callable(attrs) -> list of aux names, or list
        self.hint = hint or name
        self.param_args = param_args  # args auto-created as Variables (default: all but first)

    def arg_names(self, node):
        return self.args(node) if callable(self.args) else list(self.args)

    def aux_names(self, node):
        return self.aux(node) if callable(self.aux) else list(self.aux)


def _conv_args(node):
    return ["data", "weight"] + ([] if node.attr("no_bias", False) else ["bias"])


def _fc_args(node):
    return ["data", "weight"] + ([] if node.attr("no_bias", False) else ["bias"])


OPS = {}


def _reg(spec):
    OPS[spec.name] = spec
    return spec


_reg(OpSpec("Convolution", _conv_args, hint="convolution"))
_reg(OpSpec("Deconvolution", _conv_args, hint="deconvolution"))
_reg(OpSpec("FullyConnected", _fc_args, hint="fullyconnected"))
_reg(OpSpec("BatchNorm", ["data", "gamma", "beta"], ["moving_mean", "moving_var"], hint="batchnorm"))
_reg(OpSpec("Activation", ["data"], hint="activation"))
_reg(OpSpec("Pooling", ["data"], hint="pooling"))
_reg(OpSpec("Flatten", ["data"], hint="flatten"))
_reg(OpSpec("SoftmaxOutput", ["data", "label"], hint="softmax"))
_reg(OpSpec("identity", ["data"], hint="identity"))
_reg(OpSpec("Cast", ["data"], hint="cast"))
_reg(OpSpec("_Plus", ["lhs", "rhs"], hint="_plus"))
_reg(OpSpec("elemwise_add", ["lhs", "rhs"], hint="_plus"))
_reg(OpSpec("broadcast_add", ["lhs", "rhs"], hint="broadcast_add"))
_reg(OpSpec("_contrib_Quantization_int8", ["data"], lambda n: ["minmax"], hint="quantization_int8"))
# the fork's per-channel scale (data * scaler, scaler (1,C,1,1)): what merge_bn folds a BatchNorm into
# (core/graph_optimize.py:90-93)
_reg(OpSpec("_contrib_BroadcastScale", ["data", "scaler"], hint="broadcastscale"))
_reg(OpSpec("Custom", lambda n: ["data"], hint="custom"))


def _variadic(opname, hint):
    spec = OpSpec(opname, lambda n: ["arg%d" % i for i in range(len(n.inputs))], hint=hint)
    _reg(spec)


_variadic("ElementWiseSum", "elementwisesum")
_variadic("Concat", "concat")

_ALIASES = {"elemwise_add": "_Plus", "add_n": "ElementWiseSum", "concat": "Concat", "flatten": "Flatten"}


# ----------------------------------------------------------------------------- Symbol
class Symbol:
    def __init__(self, outputs):
        self._outputs = list(outputs)  # list of (node, idx)

    # --- composition
    @property
    def name(self):
        if len(self._outputs) != 1:
            return None
        return self._outputs[0][0].name

    def __add__(self, other):
        if isinstance(other, Symbol):
            return _create("_Plus", [self, other], {}, None)
        raise MXNetError("scalar add is not supported on the training path")

    __radd__ = __add__

    def __getitem__(self, index):
        if isinstance(index, str):
            names = self.list_outputs()
            if index not in names:
                raise MXNetError("cannot find output %s" % index)
            index = names.index(index)
        return Symbol([self._outputs[index]])

    def __iter__(self):
        return (Symbol([o]) for o in self._outputs)

    def __len__(self):
        return len(self._outputs)

    def __repr__(self):
        return "<Symbol %s>" % (self.name if self.name else "Grouped")

    # --- attributes
    def _set_attr(self, **kwargs):
        for node, _ in self._outputs:
            for k, v in kwargs.items():
                node.user_attrs[k] = str(v)

    def attr(self, key):
        node = self._outputs[0][0]
        if key in node.user_attrs:
            return node.user_attrs[key]
        return node.attrs.get(key)

    def list_attr(self):
        node = self._outputs[0][0]
        d = {k: str(v) for k, v in node.attrs.items()}
        d.update(node.user_attrs)
        return d

    def attr_dict(self):
        return {n.name: {**{k: str(v) for k, v in n.attrs.items()}, **n.user_attrs} for n in self._topo()}

    # --- graph traversal
    def _topo(self):
        """Post-order DFS over inputs in order (MXNet's argument / execution order)."""
        order, seen = [], set()
        for head, _ in self._outputs:
            stack = [(head, 0)]
            while stack:
                node, i = stack.pop()
                if id(node) in seen:
                    continue
                if i < len(node.inputs):
                    stack.append((node, i + 1))
                    child = node.inputs[i][0]
                    if id(child) not in seen:
                        stack.append((child, 0))
                else:
                    seen.add(id(node))
                    order.append(node)
        return order

    def _is_aux_var(self):
        aux = set()
        for n in self._topo():
            if n.op != "null":
                spec = OPS[n.op]
                nargs = len(spec.arg_names(n))
                for (inp, _) in n.inputs[nargs:]:
                    aux.add(id(inp))
        return aux

    def list_arguments(self):
        aux = self._is_aux_var()
        return [n.name for n in self._topo() if n.op == "null" and id(n) not in aux]

    def list_auxiliary_states(self):
        aux = self._is_aux_var()
        return [n.name for n in self._topo() if n.op == "null" and id(n) in aux]

    def list_outputs(self):
        out = []
        for node, idx in self._outputs:
            if node.op == "null":
                out.append(node.name)
            elif node.nout > 1:
                out.append("%s_output%d" % (node.name, idx))
            else:
                out.append("%s_output" % node.name)
        return out

    def list_inputs(self):
        return [n.name for n in self._topo() if n.op == "null"]

    def get_internals(self):
        outs = []
        for n in self._topo():
            for i in range(n.nout if n.op != "null" else 1):
                outs.append((n, i))
        return Symbol(outs)

    def get_children(self):
        node = self._outputs[0][0]
        if not node.inputs:
            return None
        return Symbol(list(node.inputs))

    # --- shape inference
    def infer_shape(self, *args, **kwargs):
        try:
            return self._infer_shape(kwargs)
        except MXNetError:
            raise

    def infer_shape_partial(self, *args, **kwargs):
        return self._infer_shape(kwargs, partial=True)

    def _infer_shape(self, known, partial=False):
        shapes = {}  # (id(node), idx) -> shape
        for n in self._topo():
            if n.op == "null":
                if n.name in known:
                    shapes[(id(n), 0)] = tuple(known[n.name])
                elif "__shape__" in n.attrs:
                    shp = _parse(n.attrs["__shape__"])
                    if shp and all(d > 0 for d in shp):
                        shapes[(id(n), 0)] = tuple(shp)
        for n in self._topo():
            if n.op == "null":
                continue
            _infer_node(n, shapes, partial)
        aux = self._is_aux_var()
        topo = self._topo()
        arg_shapes = [shapes.get((id(n), 0)) for n in topo if n.op == "null" and id(n) not in aux]
        aux_shapes = [shapes.get((id(n), 0)) for n in topo if n.op == "null" and id(n) in aux]
        out_shapes = [shapes.get((id(n), i)) for n, i in self._outputs]
        if not partial and (None in arg_shapes or None in out_shapes or None in aux_shapes):
            return None, None, None
        return arg_shapes, out_shapes, aux_shapes

    def infer_type(self, *args, **kwargs):
        import numpy as np
        n_args = len(self.list_arguments())
        return [np.float32] * n_args, [np.float32] * len(self._outputs), \
            [np.float32] * len(self.list_auxiliary_states())

    # --- serialisation (MXNet JSON graph format)
    def tojson(self):
        topo = self._topo()
        index = {id(n): i for i, n in enumerate(topo)}
        nodes = []
        for n in topo:
            d = {"op": n.op, "name": n.name, "inputs": [[index[id(i)], j, 0] for i, j in n.inputs]}
            attrs = {k: str(v) for k, v in n.attrs.items()}
            attrs.update(n.user_attrs)
            if attrs:
                d["attrs"] = attrs
            nodes.append(d)
        arg_nodes = [i for i, n in enumerate(topo) if n.op == "null"]
        heads = [[index[id(n)], j, 0] for n, j in self._outputs]
        return json.dumps({"nodes": nodes, "arg_nodes": arg_nodes, "node_row_ptr": list(range(len(topo) + 1)),
                           "heads": heads, "attrs": {"mxnet_version": ["int", 10300]}}, indent=2)

    def save(self, fname):
        with open(fname, "w") as f:
            f.write(self.tojson())

    def debug_str(self):
        return "\n".join("%s %s" % (n.op, n.name) for n in self._topo())


# ----------------------------------------------------------------------------- shape rules
def _shape(shapes, node_idx):
    node, idx = node_idx
    return shapes.get((id(node), idx))


def _set(shapes, node_idx, shp):
    node, idx = node_idx
    key = (id(node), idx)
    shp = tuple(int(d) for d in shp)
    if key in shapes and shapes[key] != shp:
        raise MXNetError("shape mismatch for %s: %s vs %s" % (node.name, shapes[key], shp))
    shapes[key] = shp


def _infer_node(n, shapes, partial):
    op = n.op
    ins = n.inputs
    dshape = _shape(shapes, ins[0]) if ins else None
    if dshape is None:
        if partial:
            return
        raise MXNetError("cannot infer shape of %s (%s): input shape unknown" % (n.name, op))
    if op in ("Convolution", "Deconvolution"):
        k = _tup(n.attrs["kernel"])
        nf = int(_parse(n.attrs["num_filter"]))
        st = _tup(n.attrs.get("stride", (1, 1))) or (1, 1)
        pd = _tup(n.attrs.get("pad", (0, 0))) or (0, 0)
        dl = _tup(n.attrs.get("dilate", (1, 1))) or (1, 1)
        g = int(_parse(n.attrs.get("num_group", 1)))
        N, C, H, W = dshape
        if op == "Convolution":
            _set(shapes, ins[1], (nf, C // g) + k)
            P = (H + 2 * pd[0] - (dl[0] * (k[0] - 1) + 1)) // st[0] + 1
            Q = (W + 2 * pd[1] - (dl[1] * (k[1] - 1) + 1)) // st[1] + 1
        else:
            _set(shapes, ins[1], (C, nf // g) + k)
            P = (H - 1) * st[0] - 2 * pd[0] + k[0]
            Q = (W - 1) * st[1] - 2 * pd[1] + k[1]
        if len(ins) > 2:
            _set(shapes, ins[2], (nf,))
        _set(shapes, (n, 0), (N, nf, P, Q))
    elif op == "FullyConnected":
        nh = int(_parse(n.attrs["num_hidden"]))
        flat = _parse(n.attrs.get("flatten", True))
        if flat:
            feat = 1
            for d in dshape[1:]:
                feat *= d
            out = (dshape[0], nh)
        else:
            feat = dshape[-1]
            out = tuple(dshape[:-1]) + (nh,)
        _set(shapes, ins[1], (nh, feat))
        if len(ins) > 2:
            _set(shapes, ins[2], (nh,))
        _set(shapes, (n, 0), out)
    elif op == "BatchNorm":
        axis = int(_parse(n.attrs.get("axis", 1)))
        c = dshape[axis]
        for i in (1, 2):
            _set(shapes, ins[i], (c,))
        for i in (3, 4):
            if i < len(ins):
                _set(shapes, ins[i], (c,))
        _set(shapes, (n, 0), dshape)
    elif op in ("Activation", "identity", "Cast", "_contrib_Quantization_int8", "Custom"):
        if op == "_contrib_Quantization_int8" and len(ins) > 1:
            perch = _parse(n.attrs.get("is_weight_perchannel", False)) and _parse(n.attrs.get("is_weight", False))
            _set(shapes, ins[1], (dshape[0],) if perch else (1,))
        _set(shapes, (n, 0), dshape)
    elif op == "Pooling":
        N, C, H, W = dshape
        if _parse(n.attrs.get("global_pool", False)):
            _set(shapes, (n, 0), (N, C, 1, 1))
        else:
            k = _tup(n.attrs["kernel"])
            st = _tup(n.attrs.get("stride", (1, 1))) or (1, 1)
            pd = _tup(n.attrs.get("pad", (0, 0))) or (0, 0)
            conv = _parse(n.attrs.get("pooling_convention", "valid"))
            if conv == "full":
                P = -(-(H + 2 * pd[0] - k[0]) // st[0]) + 1
                Q = -(-(W + 2 * pd[1] - k[1]) // st[1]) + 1
            else:
                P = (H + 2 * pd[0] - k[0]) // st[0] + 1
                Q = (W + 2 * pd[1] - k[1]) // st[1] + 1
            _set(shapes, (n, 0), (N, C, P, Q))
    elif op == "Flatten":
        feat = 1
        for d in dshape[1:]:
            feat *= d
        _set(shapes, (n, 0), (dshape[0], feat))
    elif op == "SoftmaxOutput":
        _set(shapes, ins[1], (dshape[0],))
        _set(shapes, (n, 0), dshape)
    elif op in ("_Plus", "ElementWiseSum"):
        for i in ins[1:]:
            s = _shape(shapes, i)
            if s is None:
                _set(shapes, i, dshape)
        _set(shapes, (n, 0), dshape)
    elif op in ("broadcast_add", "_contrib_BroadcastScale"):
        other = _shape(shapes, ins[1])
        if other is None:
            # an unshaped per-channel operand (NCHW): (1, C, 1, 1)
            other = (1, dshape[1]) + (1,) * (len(dshape) - 2) if op == "_contrib_BroadcastScale" else dshape
            _set(shapes, ins[1], other)
        if len(other) != len(dshape) or any(o not in (1, d) for o, d in zip(other, dshape)):
            raise MXNetError("%s: operand shape %s does not broadcast to %s" % (n.name, other, dshape))
        _set(shapes, (n, 0), dshape)
    elif op == "Concat":
        dim = int(_parse(n.attrs.get("dim", 1)))
        shp = list(dshape)
        shp[dim] = sum(_shape(shapes, i)[dim] for i in ins)
        _set(shapes, (n, 0), shp)
    else:
        raise MXNetError("no shape rule for op %s" % op)


# ----------------------------------------------------------------------------- constructors
def Variable(name, attr=None, shape=None, lr_mult=None, wd_mult=None, dtype=None, init=None, stype=None, **kwargs):
    attrs = dict(attr or {})
    if shape is not None:
        attrs["__shape__"] = str(tuple(shape))
    if lr_mult is not None:
        attrs["__lr_mult__"] = str(lr_mult)
    if wd_mult is not None:
        attrs["__wd_mult__"] = str(wd_mult)
    if dtype is not None:
        attrs["__dtype__"] = str(dtype)
    if init is not None:
        attrs["__init__"] = init.dumps() if hasattr(init, "dumps") else str(init)
    for k, v in kwargs.items():
        attrs[k] = str(v)
    return Symbol([(_Node("null", name, attrs), 0)])


var = Variable


def _create(opname, pos_inputs, kwargs, name, attr=None):
    opname = _ALIASES.get(opname, opname)
    spec = OPS.get(opname)
    if spec is None:
        raise MXNetError("operator %s is not supported by this runtime" % opname)
    if name is None:
        name = _auto_name(spec.hint)
    sym_kwargs = {k: v for k, v in kwargs.items() if isinstance(v, Symbol)}
    attrs = {k: v for k, v in kwargs.items() if not isinstance(v, Symbol) and v is not None}
    node = _Node(opname, name, attrs)
    arg_names = spec.arg_names(_Node(opname, name, attrs, [None] * len(pos_inputs)))
    inputs = []
    pos = list(pos_inputs)
    for i, an in enumerate(arg_names):
        s = None
        if pos:
            s = pos.pop(0)
        elif an in sym_kwargs:
            s = sym_kwargs.pop(an)
        if s is None:
            if i == 0:
                raise MXNetError("%s: missing input %s" % (name, an))
            s = Variable("%s_%s" % (name, an))
        if len(s._outputs) != 1:
            raise MXNetError("%s: input %s must be a single-output symbol" % (name, an))
        inputs.append(s._outputs[0])
    for an in spec.aux_names(node):
        # aux states may come positionally after the arguments (BatchNorm(*children) in the graph passes
        # of core/graph_optimize.py:95) or by keyword
        s = pos.pop(0) if pos else sym_kwargs.pop(an, None)
        if s is None:
            s = Variable("%s_%s" % (name, an))
        inputs.append(s._outputs[0])
    if sym_kwargs:
        raise MXNetError("%s: unexpected symbol inputs %s" % (name, list(sym_kwargs)))
    node.inputs = inputs
    if attr:
        node.user_attrs.update({k: str(v) for k, v in attr.items()})
    return Symbol([(node, 0)])


def _make(opname):
    def ctor(*args, **kwargs):
        name = kwargs.pop("name", None)
        attr = kwargs.pop("attr", None)
        if opname == "Cast" and "dtype" in kwargs:
            d = kwargs["dtype"]
            kwargs["dtype"] = getattr(d, "__name__", str(d))
        return _create(opname, [a for a in args if isinstance(a, Symbol)], kwargs, name, attr)

    ctor.__name__ = opname
    return ctor


Convolution = _make("Convolution")
Deconvolution = _make("Deconvolution")
FullyConnected = _make("FullyConnected")
BatchNorm = _make("BatchNorm")
Activation = _make("Activation")
Pooling = _make("Pooling")
Flatten = _make("Flatten")
flatten = Flatten
SoftmaxOutput = _make("SoftmaxOutput")
identity = _make("identity")
Cast = _make("Cast")
elemwise_add = _make("_Plus")
broadcast_add = _make("broadcast_add")
Custom = _make("Custom")


def ElementWiseSum(*args, **kwargs):
    name = kwargs.pop("name", None)
    return _create("ElementWiseSum", list(args), kwargs, name)


add_n = ElementWiseSum


def Concat(*args, **kwargs):
    name = kwargs.pop("name", None)
    return _create("Concat", list(args), kwargs, name)


concat = Concat


def Group(symbols):
    outs = []
    for s in symbols:
        outs.extend(s._outputs)
    return Symbol(outs)


class _Contrib:
    Quantization_int8 = staticmethod(_make("_contrib_Quantization_int8"))
    BroadcastScale = staticmethod(_make("_contrib_BroadcastScale"))

    def __getattr__(self, item):
        raise MXNetError("contrib operator %s is not provided by this runtime" % item)


contrib = _Contrib()


class _Internal:
    def __getattr__(self, item):
        if item.startswith("_"):
            item = item[1:]
        if item in ("Plus", "plus"):
            return _make("_Plus")
        raise MXNetError("internal operator %s is not provided" % item)


_internal = _Internal()


def load_json(json_str):
    g = json.loads(json_str)
    nodes = []
    for d in g["nodes"]:
        attrs = dict(d.get("attrs", d.get("param", {})) or {})
        user = {k: v for k, v in attrs.items() if k.startswith("__") or k in ("mirror_stage", "force_mirroring")}
        for k in user:
            if d["op"] != "null" or k not in ("__shape__", "__lr_mult__", "__wd_mult__", "__dtype__", "__init__"):
                attrs.pop(k, None)
        op = d["op"]
        if op != "null":
            op = _ALIASES.get(op, op)
        n = _Node(op, d["name"], attrs if d["op"] != "null" else {**attrs, **user})
        if d["op"] != "null":
            n.user_attrs.update({k: v for k, v in user.items() if not (k in attrs)})
        n.inputs = [(nodes[i], j) for i, j, *_ in d["inputs"]]
        nodes.append(n)
    return Symbol([(nodes[i], j) for i, j, *_ in g["heads"]])


def load(fname):
    with open(fname) as f:
        return load_json(f.read())
