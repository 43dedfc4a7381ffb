"""mxnet.base: error type of the shim (mirrors MXNetError raised by MXNet's C API wrappers)."""


class MXNetError(RuntimeError):
    pass


string_types = (str,)
numeric_types = (float, int)
