"""mxnet.module (core/solver.py:5 `from mxnet.module import Module`)."""
from .module import Module, BaseModule, BatchEndParam
