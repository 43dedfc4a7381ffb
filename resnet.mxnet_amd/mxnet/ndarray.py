"""mx.nd: a minimal NDArray over numpy (host) or a torch tensor (device).

Covers what the reference's hot path touches: mx.nd.array(..., ctx=cpu_pinned) in the synthetic
iterator (data/imagenet.py:17-18), asnumpy() on outputs/labels in metrics, waitall(), save/load of
parameter dicts for checkpoints, and the host-side parameter arithmetic of the graph passes
(core/graph_optimize.py:76-86: `-=`, `*`, `/`, `mx.nd.sqrt`, `expand_dims`, `[:] = v`). Math
helpers used only inside Python CustomOps are not provided.
"""
import numpy as np

from .context import Context, cpu


class NDArray:
    def __init__(self, data, ctx=None):
        self._data = data  # numpy array or torch tensor
        self._ctx = ctx or cpu()

    # --- properties
    @property
    def shape(self):
        return tuple(self._data.shape)

    @property
    def dtype(self):
        if isinstance(self._data, np.ndarray):
            return self._data.dtype.type
        return np.float32

    @property
    def context(self):
        return self._ctx

    ctx = context

    @property
    def size(self):
        return int(np.prod(self.shape))

    @property
    def ndim(self):
        return len(self.shape)

    def _torch(self):
        import torch
        if isinstance(self._data, np.ndarray):
            t = torch.from_numpy(np.ascontiguousarray(self._data))
            if self._ctx.device_type == "cpu_pinned":
                # page-locked for the H2D copy stream; a host without a GPU has nothing to pin for
                # (RN_DRY_RUN plans on the CPU)
                if torch.cuda.is_available():
                    t = t.pin_memory()
                self._data = t
            return t
        return self._data

    def asnumpy(self):
        if isinstance(self._data, np.ndarray):
            return self._data
        return self._data.detach().float().cpu().numpy().reshape(self.shape)

    def asscalar(self):
        return self.asnumpy().reshape(-1)[0]

    def astype(self, dtype, copy=True):
        return NDArray(self.asnumpy().astype(dtype), self._ctx)

    def copy(self):
        return NDArray(np.array(self.asnumpy()), self._ctx)

    def copyto(self, other):
        if isinstance(other, Context):
            return NDArray(np.array(self.asnumpy()), other)
        other[:] = self
        return other

    as_in_context = copyto

    def wait_to_read(self):
        if not isinstance(self._data, np.ndarray):
            import torch
            torch.cuda.synchronize()

    def reshape(self, *shape):
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = shape[0]
        return NDArray(self.asnumpy().reshape(shape), self._ctx)

    def __getitem__(self, k):
        return NDArray(self.asnumpy()[k], self._ctx)

    def __setitem__(self, k, v):
        v = v.asnumpy() if isinstance(v, NDArray) else v
        if isinstance(self._data, np.ndarray):
            self._data[k] = v
        else:
            import torch
            if k == slice(None):
                self._data.copy_(torch.as_tensor(np.asarray(v, dtype=np.float32)).reshape(self._data.shape))
            else:
                arr = self.asnumpy().copy()
                arr[k] = v
                self._data.copy_(torch.as_tensor(arr).reshape(self._data.shape))

    def __len__(self):
        return self.shape[0]

    # --- host arithmetic (numpy semantics, fp32 results like MXNet's default dtype)
    def _binary(self, other, fn):
        b = other.asnumpy() if isinstance(other, NDArray) else other
        return NDArray(np.asarray(fn(self.asnumpy(), b), dtype=np.float32), self._ctx)

    def _inplace(self, other, fn):
        r = self._binary(other, fn).asnumpy()
        if isinstance(self._data, np.ndarray) and self._data.shape == r.shape:
            self._data[...] = r
        elif isinstance(self._data, np.ndarray):
            self._data = r
        else:
            self[:] = r
        return self

    def __add__(self, o):
        return self._binary(o, np.add)

    def __radd__(self, o):
        return self._binary(o, lambda a, b: np.add(b, a))

    def __sub__(self, o):
        return self._binary(o, np.subtract)

    def __rsub__(self, o):
        return self._binary(o, lambda a, b: np.subtract(b, a))

    def __mul__(self, o):
        return self._binary(o, np.multiply)

    def __rmul__(self, o):
        return self._binary(o, lambda a, b: np.multiply(b, a))

    def __truediv__(self, o):
        return self._binary(o, np.divide)

    def __rtruediv__(self, o):
        return self._binary(o, lambda a, b: np.divide(b, a))

    def __neg__(self):
        return NDArray(-self.asnumpy(), self._ctx)

    def __iadd__(self, o):
        return self._inplace(o, np.add)

    def __isub__(self, o):
        return self._inplace(o, np.subtract)

    def __imul__(self, o):
        return self._inplace(o, np.multiply)

    def __itruediv__(self, o):
        return self._inplace(o, np.divide)

    def expand_dims(self, axis):
        return NDArray(np.expand_dims(self.asnumpy(), axis), self._ctx)

    def squeeze(self, axis=None):
        return NDArray(np.squeeze(self.asnumpy(), axis), self._ctx)

    def __repr__(self):
        return "\n%s\n<NDArray %s @%s>" % (self.asnumpy(), "x".join(map(str, self.shape)), self._ctx)


def array(source, ctx=None, dtype=None):
    a = source.asnumpy() if isinstance(source, NDArray) else np.asarray(source)
    a = np.array(a, dtype=dtype if dtype is not None else (a.dtype if a.dtype != np.float64 else np.float32))
    return NDArray(a, ctx)


def zeros(shape, ctx=None, dtype=np.float32):
    return NDArray(np.zeros(shape, dtype=dtype), ctx)


def ones(shape, ctx=None, dtype=np.float32):
    return NDArray(np.ones(shape, dtype=dtype), ctx)


def empty(shape, ctx=None, dtype=np.float32):
    return zeros(shape, ctx, dtype)


def sqrt(x):
    return NDArray(np.sqrt(x.asnumpy()).astype(np.float32), x.context)


def expand_dims(x, axis):
    return x.expand_dims(axis)


def waitall():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.synchronize()
    except ImportError:
        pass


def concatenate(arrays, axis=0):
    return NDArray(np.concatenate([a.asnumpy() for a in arrays], axis=axis), arrays[0].context)


def save(fname, data):
    """Parameter dict / list -> file (an .npz container keyed like MXNet's 'arg:' / 'aux:')."""
    from .model import _save_params
    _save_params(fname, data)


def load(fname):
    from .model import _load_params
    return _load_params(fname)
