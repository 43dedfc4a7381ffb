"""mx.operator: CustomOp registration surface.

The reference registers Python CustomOps at import time (symbol/clip_grad_quantization_int8.py:70,
symbol/quant_ops.py:44, core/operator/*.py), so the classes must exist for `from symbol import *`
to succeed. Executing a Python CustomOp inside the MI355X plan is not supported: a graph that
contains mx.sym.Custom fails at bind with a clear error.
"""

_REGISTRY = {}


class CustomOp:
    def __init__(self):
        pass

    def forward(self, is_train, req, in_data, out_data, aux):
        raise NotImplementedError

    def backward(self, req, out_grad, in_data, out_data, in_grad, aux):
        raise NotImplementedError

    def assign(self, dst, req, src):
        if req == "null":
            return
        if req in ("write", "inplace"):
            dst[:] = src
        elif req == "add":
            dst[:] = dst.asnumpy() + (src.asnumpy() if hasattr(src, "asnumpy") else src)


class CustomOpProp:
    def __init__(self, need_top_grad=True):
        self.need_top_grad_ = need_top_grad

    def list_arguments(self):
        return ["data"]

    def list_outputs(self):
        return ["output"]

    def list_auxiliary_states(self):
        return []

    def infer_shape(self, in_shape):
        return in_shape, (in_shape[0],) * len(self.list_outputs()), ()

    def declare_backward_dependency(self, out_grad, in_data, out_data):
        return out_grad + in_data + out_data


def register(reg_name):
    def do_register(prop_cls):
        _REGISTRY[reg_name] = prop_cls
        return prop_cls

    return do_register


def get_registry():
    return dict(_REGISTRY)
