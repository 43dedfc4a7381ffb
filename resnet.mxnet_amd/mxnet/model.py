"""mx.model: checkpoints in MXNet's own file format (train.py:218,224-227, core/solver.py:173-175).

`prefix-symbol.json` is the MXNet JSON graph; `prefix-%04d.params` is MXNet's NDArray-list
binary format (kMXAPINDArrayListMagic 0x112, NDArray V2 records, fp32, keys 'arg:NAME' /
'aux:NAME'), so checkpoints written here load in MXNet and MXNet checkpoints load here.
"""
import struct

import numpy as np

from .base import MXNetError

_LIST_MAGIC = 0x112
_V2_MAGIC = 0xF993FAC9
_V1_MAGIC = 0xF993FAC8
_DTYPES = {0: np.float32, 1: np.float64, 2: np.float16, 3: np.uint8, 4: np.int32, 5: np.int8, 6: np.int64}
_DTYPE_IDS = {np.dtype(v): k for k, v in _DTYPES.items()}


def _to_numpy(v):
    return v.asnumpy() if hasattr(v, "asnumpy") else np.asarray(v)


def _save_params(fname, data):
    if isinstance(data, dict):
        names, arrays = list(data.keys()), [_to_numpy(v) for v in data.values()]
    else:
        names, arrays = [], [_to_numpy(v) for v in data]
    with open(fname, "wb") as f:
        f.write(struct.pack("<QQQ", _LIST_MAGIC, 0, len(arrays)))
        for a in arrays:
            a = np.ascontiguousarray(a)
            if a.dtype not in _DTYPE_IDS:
                a = a.astype(np.float32)
            f.write(struct.pack("<Ii", _V2_MAGIC, 0))  # magic, storage type (default)
            f.write(struct.pack("<I", a.ndim))
            f.write(struct.pack("<%dq" % a.ndim, *a.shape))
            f.write(struct.pack("<ii", 1, 0))  # context cpu(0)
            f.write(struct.pack("<i", _DTYPE_IDS[a.dtype]))
            f.write(a.tobytes())
        f.write(struct.pack("<Q", len(names)))
        for n in names:
            b = n.encode()
            f.write(struct.pack("<Q", len(b)))
            f.write(b)


def _load_params(fname):
    from .ndarray import NDArray
    with open(fname, "rb") as f:
        buf = f.read()
    off = 0

    def rd(fmt):
        nonlocal off
        v = struct.unpack_from(fmt, buf, off)
        off += struct.calcsize(fmt)
        return v

    magic, _, n = rd("<QQQ")
    if magic != _LIST_MAGIC:
        raise MXNetError("%s is not an MXNet NDArray list file" % fname)
    arrays = []
    for _ in range(n):
        (m,) = rd("<I")
        if m == _V2_MAGIC:
            (stype,) = rd("<i")
            if stype != 0:
                raise MXNetError("sparse NDArray in %s not supported" % fname)
            (ndim,) = rd("<I")
            shape = rd("<%dq" % ndim) if ndim else ()
        elif m == _V1_MAGIC:
            (ndim,) = rd("<I")
            shape = rd("<%dq" % ndim) if ndim else ()
        else:  # legacy: magic word is ndim, uint32 dims
            ndim = m
            shape = rd("<%dI" % ndim) if ndim else ()
        if ndim == 0:
            arrays.append(NDArray(np.zeros(0, np.float32)))
            continue
        rd("<ii")
        (tflag,) = rd("<i")
        dt = np.dtype(_DTYPES[tflag])
        cnt = int(np.prod(shape))
        a = np.frombuffer(buf, dtype=dt, count=cnt, offset=off).reshape(shape).copy()
        off += cnt * dt.itemsize
        arrays.append(NDArray(a))
    (nn,) = rd("<Q")
    names = []
    for _ in range(nn):
        (ln,) = rd("<Q")
        names.append(buf[off:off + ln].decode())
        off += ln
    if names:
        return dict(zip(names, arrays))
    return arrays


def save_checkpoint(prefix, epoch, symbol, arg_params, aux_params):
    if symbol is not None:
        symbol.save("%s-symbol.json" % prefix)
    save_dict = {("arg:%s" % k): v for k, v in arg_params.items()}
    save_dict.update({("aux:%s" % k): v for k, v in aux_params.items()})
    _save_params("%s-%04d.params" % (prefix, epoch), save_dict)


def load_params(prefix, epoch):
    save_dict = _load_params("%s-%04d.params" % (prefix, epoch))
    arg_params, aux_params = {}, {}
    for k, v in save_dict.items():
        tp, name = k.split(":", 1)
        if tp == "arg":
            arg_params[name] = v
        if tp == "aux":
            aux_params[name] = v
    return arg_params, aux_params


def load_checkpoint(prefix, epoch):
    from . import symbol as sym
    symbol = sym.load("%s-symbol.json" % prefix)
    arg_params, aux_params = load_params(prefix, epoch)
    return symbol, arg_params, aux_params


class FeedForward:
    """The legacy model API as test.py:64-71 drives it: FeedForward(symbol, ctx, arg_params=...,
    aux_params=...).score(val_iter). Evaluation only (fit is Module's / Solver's job): a Module bound
    for inference on the iterator's shapes, parameters the symbol does not use are ignored like
    MXNet's FeedForward._init_params does."""

    def __init__(self, symbol, ctx=None, num_epoch=None, epoch_size=None, optimizer="sgd", initializer=None,
                 numpy_batch_size=128, arg_params=None, aux_params=None, allow_extra_params=False,
                 begin_epoch=0, **kwargs):
        from .context import gpu
        self.symbol = symbol
        self.ctx = ctx if ctx is not None else gpu(0)
        self.arg_params, self.aux_params = arg_params, aux_params
        self._mod = None
        self._shapes = None

    def _module(self, it):
        from .module import Module
        shapes = (tuple(it.provide_data), tuple(it.provide_label or ()))
        if self._mod is None or self._shapes != shapes:
            data_names = [d[0] if isinstance(d, tuple) else d.name for d in it.provide_data]
            label_names = [d[0] if isinstance(d, tuple) else d.name for d in (it.provide_label or [])]
            mod = Module(self.symbol, data_names=data_names, label_names=label_names, context=self.ctx)
            mod.bind(it.provide_data, it.provide_label, for_training=False)
            mod.init_params(arg_params=self.arg_params, aux_params=self.aux_params, allow_missing=False,
                            allow_extra=True)
            self._mod, self._shapes = mod, shapes
        return self._mod

    def score(self, X, eval_metric="acc", num_batch=None, batch_end_callback=None, reset=True):
        """The metric's value over X (FeedForward.score returns eval_metric.get()[1])."""
        from . import metric
        m = eval_metric if isinstance(eval_metric, metric.EvalMetric) else metric.create(eval_metric)
        self._module(X).score(X, m, num_batch=num_batch, batch_end_callback=batch_end_callback, reset=reset)
        return m.get()[1]

    def predict(self, X, num_batch=None, return_data=False, reset=True):
        return self._module(X).predict(X, num_batch=num_batch, reset=reset).asnumpy()
