"""The reference's graph passes, driven through the `mxnet` shim's public API (test helper).

core/graph_optimize.py rebuilds a symbol node by node from `symbol.tojson()`: Variables through
`mx.sym.var(name, **dunder_attrs)`, every operator through `mx.sym.<op>` / `mx.sym.contrib.<op>` /
`mx.sym._internal.<op>` called with its JSON children positionally and its JSON attrs (strings) as
keywords. The three passes below make exactly those calls (the reference file itself cannot be
imported in this container), so a green test here means the reference's own passes can run on the
MI355X runtime:

  fix_bn                core/graph_optimize.py:114-157  BatchNorm -> use_global_stats=True
  merge_bn              core/graph_optimize.py:37-112   inference BN after a conv -> BroadcastScale +
                                                        broadcast_add with folded parameters
  attach_quantize_node  core/graph_optimize.py:159-292  Quantization_int8 on conv / fc inputs
"""
import json

import mxnet as mx


def _operator(op_name):
    """The constructor the reference looks up for a JSON op name (graph_optimize.py:99-105)."""
    if op_name.startswith("_contrib_"):
        return getattr(mx.sym.contrib, op_name[len("_contrib_"):])
    if op_name.startswith("_"):
        return getattr(mx.sym._internal, op_name)
    return getattr(mx.sym, op_name)


def _rebuild(symbol, visit):
    """Walk symbol.tojson() in node order; visit(node, children, attrs, op_of) returns the new Symbol
    for an operator node or None to re-create it unchanged. op_of[(nid, out)] is the op name that
    produced an input (node_op_map of the reference)."""
    graph = json.loads(symbol.tojson())
    built, op_of = {}, {}
    for nid, node in enumerate(graph["nodes"]):
        kids = [built[i][j] for i, j, *_ in node["inputs"]]
        attrs = dict(node.get("attrs", {}))
        if node["op"] == "null":
            out = mx.sym.var(node["name"], **{k: v for k, v in attrs.items() if k.startswith("__")})
            op_of[nid] = "Variable"
        else:
            out = visit(node, kids, attrs, op_of)
            if out is None:
                out = _operator(node["op"])(*kids, name=node["name"], **attrs)
            op_of[nid] = node["op"]
        built[nid] = out
    heads = [built[i][j] for i, j, *_ in graph["heads"]]
    return heads[0] if len(heads) == 1 else mx.sym.Group(heads)


def fix_bn(symbol):
    def visit(node, kids, attrs, op_of):
        if node["op"] != "BatchNorm":
            return None
        if attrs.get("use_global_stats", "False") == "False":
            attrs["use_global_stats"] = "True"
        return mx.sym.BatchNorm(*kids, name=node["name"], **attrs)

    return _rebuild(symbol, visit)


def merge_bn(symbol, args, auxs):
    """Folds each use_global_stats BatchNorm whose input is a Convolution into a per-channel scale and
    bias (graph_optimize.py:69-93); args / auxs (NDArray dicts) are updated like the reference does."""
    def visit(node, kids, attrs, op_of):
        if node["op"] != "BatchNorm":
            return None
        src = node["inputs"][0]
        if attrs.get("use_global_stats") != "True" or op_of.get(src[0]) != "Convolution":
            return mx.sym.BatchNorm(*kids, name=node["name"], **attrs)
        _, gamma, beta, mean, var = kids
        gn, bn_, mn, vn = gamma.name, beta.name, mean.name, var.name
        eps = float(attrs["eps"])
        if mn in auxs:
            # beta first: it uses the unscaled gamma (graph_optimize.py:75-77)
            args[bn_] -= args[gn] * auxs[mn] / mx.nd.sqrt(eps + auxs[vn])
            args[gn] /= mx.nd.sqrt(eps + auxs[vn])
            if args[gn].ndim == 1:
                for d, k in ((args, gn), (args, bn_), (auxs, mn), (auxs, vn)):
                    d[k] = d[k].expand_dims(axis=0).expand_dims(axis=-1).expand_dims(axis=-1)
            auxs[mn][:] = 0.0
            auxs[vn][:] = 1.0
            args[node["name"] + "_gamma"] = args[gn]
            args[node["name"] + "_beta"] = args[bn_]
        g = mx.sym.var(node["name"] + "_gamma", shape=args[node["name"] + "_gamma"].shape)
        b = mx.sym.var(node["name"] + "_beta", shape=args[node["name"] + "_beta"].shape)
        return mx.sym.broadcast_add(mx.sym.contrib.BroadcastScale(data=kids[0], scaler=g), b)

    return _rebuild(symbol, visit), args, auxs


def _quant_node(var, setting):
    """create_quant_node for quantize_op_name 'Quantization_int8' (graph_optimize.py:165-168)."""
    assert setting["quantize_op_name"] == "Quantization_int8"
    minmax = mx.sym.var(name=var.name + "_minmax", init=mx.init.Constant(setting.get("init_value") or 0))
    return mx.sym.contrib.Quantization_int8(name=var.name, data=var, minmax=minmax, **setting["attrs"])


def attach_quantize_node(symbol, out_shape_dict, weight_setting, act_setting,
                         quantized_op=("Convolution", "FullyConnected", "Deconvolution"), skip_quantize_counts=None):
    counts = {}
    made = {}  # quantized tensor name -> its Quantization_int8 node (one node per tensor)

    def quant(v, setting):
        if v.name not in made:
            made[v.name] = _quant_node(v, setting)
        return made[v.name]

    def visit(node, kids, attrs, op_of):
        op = node["op"]
        if op not in quantized_op:
            return None
        counts[op] = counts.get(op, 0) + 1
        if skip_quantize_counts and counts[op] <= skip_quantize_counts.get(op, 0):
            new_kids = kids
        elif op in ("Convolution", "FullyConnected", "Deconvolution"):
            new_kids = [quant(kids[0], act_setting), quant(kids[1], weight_setting)] + kids[2:]
        else:
            new_kids = [quant(k, act_setting) for k in kids]
        return getattr(mx.sym, op)(*new_kids, name=node["name"], **attrs)

    # Variables carry their inferred shape (graph_optimize.py:227-230)
    graph = json.loads(symbol.tojson())
    for node in graph["nodes"]:
        if node["op"] == "null":
            assert node["name"] in out_shape_dict, node["name"]
            a = node.setdefault("attrs", {})
            if "__shape__" not in a:
                a["__shape__"] = str(tuple(out_shape_dict[node["name"]]))
                a["__dtype__"] = "0"
    return _rebuild(mx.sym.load_json(json.dumps(graph)), visit)


def shape_dict(symbol, data_shape, label_shape):
    """train.py:114-116: out_shape_dictoinary from get_internals().infer_shape."""
    internals = symbol.get_internals()
    _, out_shapes, _ = internals.infer_shape(data=data_shape, softmax_label=label_shape)
    return dict(zip(internals.list_outputs(), out_shapes))
