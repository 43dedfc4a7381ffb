"""mx.recordio: MXNet's RecordIO container (read and write), the format behind the reference's
ImageNet / CIFAR `.rec` files (data/imagenet.py:153-208, data/cifar10.py:12-46).

Layout of one record (dmlc-core recordio, as MXNet 1.x writes it): uint32 magic 0xced7230a,
uint32 lrecord = (cflag << 29) | length, `length` payload bytes, zero padding to a multiple of 4.
cflag 0 is a whole record; a payload longer than 2^29 - 1 bytes is split into parts flagged 1 (first),
2 (middle), 3 (last), which read() joins. An image record's payload is IRHeader = struct 'IfQQ'
(flag, label, id, id2) followed, when flag > 0, by `flag` float32 labels, then the encoded image.
The `.idx` companion file of MXIndexedRecordIO holds one "key<TAB>byte offset" line per record.
"""
import io
import os
import struct
from collections import namedtuple

import numpy as np

from .base import MXNetError

kMagic = 0xCED7230A
_LEN_MASK = (1 << 29) - 1
IRHeader = namedtuple("HEADER", ["flag", "label", "id", "id2"])
_IR_FORMAT = "IfQQ"
_IR_SIZE = struct.calcsize(_IR_FORMAT)


class MXRecordIO:
    """Sequential reader / writer of a .rec file (flag 'r' or 'w')."""

    def __init__(self, uri, flag):
        self.uri = str(uri)
        self.flag = flag
        self.handle = None
        self.is_open = False
        self.open()

    def open(self):
        if self.flag == "w":
            self.handle = open(self.uri, "wb")
            self.writable = True
        elif self.flag == "r":
            self.handle = open(self.uri, "rb")
            self.writable = False
        else:
            raise ValueError("Invalid flag %s" % self.flag)
        self.is_open = True

    def __del__(self):
        self.close()

    def __getstate__(self):
        d = dict(self.__dict__)
        d["handle"] = None
        d["is_open"] = False
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)
        self.open()

    def close(self):
        if getattr(self, "is_open", False):
            self.handle.close()
            self.is_open = False

    def reset(self):
        self.close()
        self.open()

    def tell(self):
        return self.handle.tell()

    def seek(self, pos):
        assert not self.writable
        self.handle.seek(pos)

    def write(self, buf):
        assert self.writable
        buf = bytes(buf)
        n = len(buf)
        parts = [buf[i:i + _LEN_MASK] for i in range(0, n, _LEN_MASK)] or [b""]
        for i, part in enumerate(parts):
            cflag = 0 if len(parts) == 1 else (1 if i == 0 else (3 if i == len(parts) - 1 else 2))
            self.handle.write(struct.pack("<II", kMagic, (cflag << 29) | len(part)))
            self.handle.write(part)
            self.handle.write(b"\0" * ((4 - len(part) % 4) % 4))

    def _read_part(self):
        head = self.handle.read(8)
        if len(head) == 0:
            return None, None
        if len(head) < 8:
            raise MXNetError("%s: truncated record header" % self.uri)
        magic, lrec = struct.unpack("<II", head)
        if magic != kMagic:
            raise MXNetError("%s: invalid RecordIO magic 0x%08x at byte %d" % (self.uri, magic, self.handle.tell() - 8))
        n = lrec & _LEN_MASK
        data = self.handle.read(n)
        if len(data) < n:
            raise MXNetError("%s: truncated record" % self.uri)
        self.handle.seek((4 - n % 4) % 4, os.SEEK_CUR)
        return lrec >> 29, data

    def read(self):
        """The next record's payload (multi-part records joined), or None at the end of the file."""
        assert not self.writable
        cflag, data = self._read_part()
        if cflag is None:
            return None
        if cflag == 0:
            return data
        if cflag != 1:
            raise MXNetError("%s: record continuation without a start" % self.uri)
        out = [data]
        while True:
            cflag, data = self._read_part()
            if cflag not in (2, 3):
                raise MXNetError("%s: unterminated multi-part record" % self.uri)
            out.append(data)
            if cflag == 3:
                return b"".join(out)

    def scan_offsets(self):
        """Byte offset of every record (one pass over the headers, payloads skipped)."""
        assert not self.writable
        self.handle.seek(0)
        offs = []
        while True:
            pos = self.handle.tell()
            head = self.handle.read(8)
            if len(head) < 8:
                break
            magic, lrec = struct.unpack("<II", head)
            if magic != kMagic:
                raise MXNetError("%s: invalid RecordIO magic at byte %d" % (self.uri, pos))
            if lrec >> 29 in (0, 1):
                offs.append(pos)
            n = lrec & _LEN_MASK
            self.handle.seek(n + (4 - n % 4) % 4, os.SEEK_CUR)
        self.handle.seek(0)
        return offs


class MXIndexedRecordIO(MXRecordIO):
    """Random access through the .idx file ("key\\toffset" lines)."""

    def __init__(self, idx_path, uri, flag, key_type=int):
        self.idx_path = idx_path
        self.idx = {}
        self.keys = []
        self.key_type = key_type
        self.fidx = None
        super().__init__(uri, flag)

    def open(self):
        super().open()
        self.idx = {}
        self.keys = []
        self.fidx = open(self.idx_path, self.flag)
        if not self.writable:
            for line in iter(self.fidx.readline, ""):
                line = line.strip().split("\t")
                key = self.key_type(line[0])
                self.idx[key] = int(line[1])
                self.keys.append(key)

    def close(self):
        if getattr(self, "is_open", False):
            super().close()
            self.fidx.close()

    def read_idx(self, idx):
        self.seek(self.idx[idx])
        return self.read()

    def write_idx(self, idx, buf):
        key = self.key_type(idx)
        pos = self.tell()
        self.write(buf)
        self.fidx.write("%s\t%d\n" % (str(key), pos))
        self.idx[key] = pos
        self.keys.append(key)


def pack(header, s):
    """IRHeader + payload -> record bytes (a label array sets flag = its length)."""
    header = IRHeader(*header)
    if isinstance(header.label, (int, float, np.floating, np.integer)):
        header = header._replace(flag=0)
        out = struct.pack(_IR_FORMAT, *header)
    else:
        label = np.asarray(header.label, dtype=np.float32)
        header = header._replace(flag=label.size, label=0)
        out = struct.pack(_IR_FORMAT, *header) + label.tobytes()
    return out + bytes(s)


def unpack(s):
    """record bytes -> (IRHeader, payload); a multi-label header carries its labels as an array."""
    header = IRHeader(*struct.unpack(_IR_FORMAT, s[:_IR_SIZE]))
    s = s[_IR_SIZE:]
    if header.flag > 0:
        header = header._replace(label=np.frombuffer(s, np.float32, header.flag))
        s = s[header.flag * 4:]
    return header, s


def pack_img(header, img, quality=95, img_fmt=".jpg"):
    """IRHeader + HWC uint8 image -> record bytes, encoded by PIL. As MXNet's (cv2.imencode), a
    3-channel image is taken in BGR order (2-D: gray); the file stores it as a normal RGB image."""
    from PIL import Image
    buf = io.BytesIO()
    fmt = {".jpg": "JPEG", ".jpeg": "JPEG", ".png": "PNG"}[img_fmt.lower()]
    kw = {"quality": int(quality)} if fmt == "JPEG" else {"compress_level": 1}
    a = np.asarray(img, dtype=np.uint8)
    if a.ndim == 3 and a.shape[2] == 3:
        a = np.ascontiguousarray(a[:, :, ::-1])  # BGR -> RGB for the encoder
    Image.fromarray(a).save(buf, format=fmt, **kw)
    return pack(header, buf.getvalue())


def unpack_img(s, iscolor=-1):
    """record bytes -> (IRHeader, HWC uint8 image in BGR order as MXNet's cv2.imdecode; 2-D gray for
    iscolor=0). (ImageRecordIter decodes to RGB itself, as MXNet's iterator does.)"""
    from PIL import Image
    header, s = unpack(s)
    im = Image.open(io.BytesIO(s))
    if iscolor == 0:
        return header, np.asarray(im.convert("L"))
    return header, np.ascontiguousarray(np.asarray(im.convert("RGB"))[:, :, ::-1])
