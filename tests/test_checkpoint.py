"""Checkpoint format: `prefix-symbol.json` + `prefix-%04d.params` as written by
mx.model.save_checkpoint / Module.save_checkpoint (reference train.py:218,224-227,
core/solver.py:173-175) and read back by load_checkpoint (train.py:90-95, test.py).

MXNet itself is not importable here and the reference ships no .params file, so the binary layout
is pinned by an independent minimal reader written in this test from MXNet 1.x's NDArray-list
format (src/c_api + src/ndarray/ndarray.cc, un-vendored): uint64 magic 0x112, uint64 reserved,
uint64 count; per array uint32 0xF993FAC9, int32 storage type 0, uint32 ndim, int64 dims,
int32 dev_type, int32 dev_id, int32 type flag, raw little-endian data; then uint64 count of
names and (uint64 length, bytes) per name. Parity against MXNet's own reader: unpinned.
"""
import struct

import numpy as np
import pytest

import mxnet as mx
from oracle import net as onet
from rn import graphs

_FLAGS = {0: np.float32, 1: np.float64, 2: np.float16, 3: np.uint8, 4: np.int32, 5: np.int8, 6: np.int64}


def read_ndarray_list(path):
    """Independent reader of the MXNet 1.x NDArray-list file (see module docstring)."""
    with open(path, "rb") as f:
        b = f.read()
    magic, reserved, n = struct.unpack_from("<QQQ", b, 0)
    assert magic == 0x112 and reserved == 0
    off, arrays = 24, []
    for _ in range(n):
        m, stype, ndim = struct.unpack_from("<IiI", b, off)
        off += 12
        assert m == 0xF993FAC9 and stype == 0
        shape = struct.unpack_from("<%dq" % ndim, b, off)
        off += 8 * ndim
        dev_type, dev_id, flag = struct.unpack_from("<iii", b, off)
        off += 12
        assert (dev_type, dev_id) == (1, 0)  # saved from cpu(0)
        dt = np.dtype(_FLAGS[flag])
        cnt = int(np.prod(shape))
        arrays.append(np.frombuffer(b, dt, cnt, off).reshape(shape))
        off += cnt * dt.itemsize
    (nn,) = struct.unpack_from("<Q", b, off)
    off += 8
    names = []
    for _ in range(nn):
        (ln,) = struct.unpack_from("<Q", b, off)
        names.append(b[off + 8:off + 8 + ln].decode())
        off += 8 + ln
    assert off == len(b)
    return dict(zip(names, arrays))


def _resnet20_params():
    g = onet.resnet20_cifar()
    args, aux = onet.init_params(g, dtype=np.float32)
    rng = np.random.default_rng(3)
    aux = {k: (v + rng.standard_normal(v.shape).astype(np.float32) * 0.1) for k, v in aux.items()}
    return args, aux


def test_checkpoint_layout_and_round_trip(tmp_path):
    sym = graphs.resnet_cifar10([3, 3, 3], 3, [16, 16, 32, 64], 10)
    args, aux = _resnet20_params()
    prefix = str(tmp_path / "resnet20")
    mx.model.save_checkpoint(prefix, 7, sym, {k: mx.nd.array(v) for k, v in args.items()},
                             {k: mx.nd.array(v) for k, v in aux.items()})
    raw = read_ndarray_list(prefix + "-0007.params")
    assert set(raw) == {"arg:" + k for k in args} | {"aux:" + k for k in aux}
    for k, v in args.items():
        np.testing.assert_array_equal(raw["arg:" + k], v)
    for k, v in aux.items():
        np.testing.assert_array_equal(raw["aux:" + k], v)
    sym2, args2, aux2 = mx.model.load_checkpoint(prefix, 7)
    assert sym2.list_arguments() == sym.list_arguments()
    assert sym2.list_auxiliary_states() == sym.list_auxiliary_states()
    for k in args:
        np.testing.assert_array_equal(args2[k].asnumpy(), args[k])
    for k in aux:
        np.testing.assert_array_equal(aux2[k].asnumpy(), aux[k])


def test_params_reader_accepts_older_records(tmp_path):
    """load_params also reads the V1 record (magic 0xF993FAC8, no storage type) and the legacy
    record (first word = ndim, uint32 dims) of older MXNet versions, plus unnamed lists."""
    a = np.arange(6, dtype=np.float32).reshape(2, 3)
    c = np.array([1.5, -2.0], dtype=np.float64)
    path = str(tmp_path / "old-0000.params")
    with open(path, "wb") as f:
        f.write(struct.pack("<QQQ", 0x112, 0, 2))
        f.write(struct.pack("<II", 0xF993FAC8, 2) + struct.pack("<2q", 2, 3) + struct.pack("<iii", 1, 0, 0))
        f.write(a.tobytes())
        f.write(struct.pack("<I", 1) + struct.pack("<I", 2) + struct.pack("<iii", 1, 0, 1))
        f.write(c.tobytes())
        f.write(struct.pack("<Q", 2))
        for n in (b"arg:w", b"aux:m"):
            f.write(struct.pack("<Q", len(n)) + n)
    args, aux = mx.model.load_params(str(tmp_path / "old"), 0)
    np.testing.assert_array_equal(args["w"].asnumpy(), a)
    np.testing.assert_array_equal(aux["m"].asnumpy(), c)


def test_not_a_params_file(tmp_path):
    path = tmp_path / "bad-0001.params"
    path.write_bytes(b"\x00" * 32)
    with pytest.raises(mx.base.MXNetError):
        mx.model.load_params(str(tmp_path / "bad"), 1)
