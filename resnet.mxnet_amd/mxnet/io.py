"""mx.io: the DataIter protocol (data/imagenet.py:9-41 SyntheticDataIter is built on it)."""
from collections import namedtuple

import numpy as np

from .base import MXNetError
from . import ndarray as nd


class DataDesc(namedtuple("DataDesc", ["name", "shape"])):
    def __new__(cls, name, shape, dtype=np.float32, layout="NCHW"):
        ret = super().__new__(cls, name, tuple(shape))
        ret.dtype = dtype
        ret.layout = layout
        return ret


class DataBatch:
    def __init__(self, data, label=None, pad=None, index=None, bucket_key=None, provide_data=None,
                 provide_label=None):
        self.data = data
        self.label = label
        self.pad = pad
        self.index = index
        self.bucket_key = bucket_key
        self.provide_data = provide_data
        self.provide_label = provide_label


class DataIter:
    def __init__(self, batch_size=0):
        self.batch_size = batch_size

    def __iter__(self):
        return self

    def reset(self):
        pass

    def next(self):
        raise StopIteration

    def __next__(self):
        return self.next()

    @property
    def provide_data(self):
        return []

    @property
    def provide_label(self):
        return []


class NDArrayIter(DataIter):
    def __init__(self, data, label=None, batch_size=1, shuffle=False, last_batch_handle="pad",
                 data_name="data", label_name="softmax_label"):
        super().__init__(batch_size)
        self.data = np.asarray(data.asnumpy() if isinstance(data, nd.NDArray) else data, dtype=np.float32)
        self.label = None if label is None else np.asarray(label.asnumpy() if isinstance(label, nd.NDArray)
                                                            else label, dtype=np.float32)
        self.data_name, self.label_name = data_name, label_name
        self.cursor = 0

    @property
    def provide_data(self):
        return [DataDesc(self.data_name, (self.batch_size,) + self.data.shape[1:])]

    @property
    def provide_label(self):
        return [] if self.label is None else [DataDesc(self.label_name, (self.batch_size,))]

    def reset(self):
        self.cursor = 0

    def next(self):
        if self.cursor + self.batch_size > self.data.shape[0]:
            raise StopIteration
        s = slice(self.cursor, self.cursor + self.batch_size)
        self.cursor += self.batch_size
        return DataBatch([nd.array(self.data[s])], None if self.label is None else [nd.array(self.label[s])], pad=0,
                         provide_data=self.provide_data, provide_label=self.provide_label)


class ResizeIter(DataIter):
    """Resize an iterator to `size` batches per epoch (train.py:153)."""

    def __init__(self, data_iter, size, reset_internal=True):
        super().__init__(data_iter.batch_size)
        self.data_iter, self.size, self.reset_internal = data_iter, size, reset_internal
        self.cur = 0

    @property
    def provide_data(self):
        return self.data_iter.provide_data

    @property
    def provide_label(self):
        return self.data_iter.provide_label

    def reset(self):
        self.cur = 0
        if self.reset_internal:
            self.data_iter.reset()

    def next(self):
        if self.cur == self.size:
            raise StopIteration
        try:
            batch = self.data_iter.next()
        except StopIteration:
            self.data_iter.reset()
            batch = self.data_iter.next()
        self.cur += 1
        return batch


def ImageRecordIter(**kwargs):
    """RecordIO images -> augmented NCHW float32 batches (mxnet/image_iter.py)."""
    from .image_iter import ImageRecordIter as _It
    return _It(**kwargs)
