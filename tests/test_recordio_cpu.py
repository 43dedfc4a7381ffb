"""mx.recordio + mx.io.ImageRecordIter (data/imagenet.py:153-208,
data/cifar10.py:12-46): the RecordIO byte layout, multi-part records, the .idx index, IRHeader
packing, and the image iterator's batches. The val path (resize + centre crop + normalize) is
deterministic and is compared with an independent PIL/numpy recomputation; the random train
augmentations by shape, range and seeded determinism. MXNet's own iterator cannot run here, so the
augmenters' parity with its C++ implementation is unpinned (mxnet/image_iter.py header)."""
import io
import struct

import numpy as np
import pytest
from PIL import Image

import mxnet as mx
from mxnet import recordio

MAGIC = 0xCED7230A


def _images(n, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        h, w = int(rng.integers(30, 70)), int(rng.integers(30, 70))
        out.append(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))
    return out


def _write_rec(path, imgs, fmt=".png", labels=None):
    w = recordio.MXIndexedRecordIO(str(path) + ".idx", str(path), "w")
    for i, im in enumerate(imgs):
        lab = float(i) if labels is None else labels[i]
        # pack_img takes BGR (MXNet's cv2 convention): the file then holds `im` as RGB
        w.write_idx(i, recordio.pack_img(recordio.IRHeader(0, lab, i, 0), im[:, :, ::-1], img_fmt=fmt))
    w.close()


def test_record_layout_and_roundtrip(tmp_path):
    path = tmp_path / "a.rec"
    bufs = [b"", b"x", b"abc", b"hello", bytes(range(256)) * 3]
    w = recordio.MXRecordIO(str(path), "w")
    for b in bufs:
        w.write(b)
    w.close()
    raw = path.read_bytes()
    # record 1 ("x"): magic, length 1 with cflag 0, payload, 3 zero bytes of padding
    assert struct.unpack("<II", raw[:8]) == (MAGIC, 0)
    assert struct.unpack("<II", raw[8:16]) == (MAGIC, 1) and raw[16:20] == b"x\0\0\0"
    assert len(raw) == sum(8 + (len(b) + 3) // 4 * 4 for b in bufs)
    r = recordio.MXRecordIO(str(path), "r")
    assert [r.read() for _ in bufs] == bufs
    assert r.read() is None
    r.reset()
    assert r.read() == b""
    assert len(r.scan_offsets()) == len(bufs)


def test_multipart_record(tmp_path):
    """A record split into parts flagged 1 / 2 / 3 (lrecord bits 29-31) reads back joined."""
    parts = [b"abcde", b"fgh", b"ijklmn"]
    raw = b""
    for cflag, p in zip((1, 2, 3), parts):
        raw += struct.pack("<II", MAGIC, (cflag << 29) | len(p)) + p + b"\0" * ((4 - len(p) % 4) % 4)
    raw += struct.pack("<II", MAGIC, 2) + b"zz\0\0"
    path = tmp_path / "m.rec"
    path.write_bytes(raw)
    r = recordio.MXRecordIO(str(path), "r")
    assert r.read() == b"".join(parts)
    assert r.read() == b"zz"
    assert r.read() is None
    assert r.scan_offsets() == [0, len(raw) - 12]
    path.write_bytes(raw[:6])
    with pytest.raises(mx.MXNetError):
        recordio.MXRecordIO(str(path), "r").read()


def test_indexed_random_access(tmp_path):
    path = tmp_path / "i.rec"
    w = recordio.MXIndexedRecordIO(str(path) + ".idx", str(path), "w")
    for i in range(20):
        w.write_idx(i, b"rec%03d" % i * (i + 1))
    w.close()
    r = recordio.MXIndexedRecordIO(str(path) + ".idx", str(path), "r")
    assert r.keys == list(range(20))
    for i in (17, 3, 0, 19, 3):
        assert r.read_idx(i) == b"rec%03d" % i * (i + 1)


def test_pack_unpack_labels():
    h, s = recordio.unpack(recordio.pack(recordio.IRHeader(0, 7.0, 3, 4), b"payload"))
    assert (h.flag, h.label, h.id, h.id2, s) == (0, 7.0, 3, 4, b"payload")
    h, s = recordio.unpack(recordio.pack(recordio.IRHeader(0, [1.0, 2.5, -3.0], 9, 0), b"xy"))
    assert h.flag == 3 and np.array_equal(h.label, [1.0, 2.5, -3.0]) and s == b"xy"


def test_pack_img_png_exact():
    img = _images(1, 3)[0]
    h, out = recordio.unpack_img(recordio.pack_img(recordio.IRHeader(0, 5.0, 1, 0), img, img_fmt=".png"))
    assert h.label == 5.0 and np.array_equal(out, img)


def test_pack_img_channel_order_bgr():
    """pack_img / unpack_img use MXNet's (OpenCV's) BGR order: a BGR blue pixel (255, 0, 0) is stored
    as RGB (0, 0, 255), and the iterator (RGB, as MXNet's ImageRecordIter) reads it as blue."""
    bgr = np.zeros((4, 4, 3), np.uint8)
    bgr[..., 0] = 255
    rec = recordio.pack_img(recordio.IRHeader(0, 0.0, 0, 0), bgr, img_fmt=".png")
    _, payload = recordio.unpack(rec)
    rgb = np.asarray(Image.open(io.BytesIO(payload)).convert("RGB"))
    assert (rgb[..., 2] == 255).all() and (rgb[..., :2] == 0).all()
    assert np.array_equal(recordio.unpack_img(rec)[1], bgr)
    assert recordio.unpack_img(rec, iscolor=0)[1].ndim == 2


def test_round_batch_false_pads_with_zeros(tmp_path):
    """round_batch=False: the last batch holds only its own records; its pad slots are zeros."""
    path = tmp_path / "rb.rec"
    _write_rec(path, _images(5, 4))
    it = mx.io.ImageRecordIter(path_imgrec=str(path), data_shape=(3, 24, 24), batch_size=4, resize=24,
                               round_batch=False)
    b = list(it)
    assert [x.pad for x in b] == [0, 3]
    last = b[1].data[0].asnumpy()
    assert b[1].label[0].asnumpy()[0] == 4.0 and not last[1:].any() and last[0].any()


MEAN = np.array([123.68, 116.28, 103.53])
STD = np.array([58.395, 57.12, 57.375])
NORM = dict(mean_r=MEAN[0], mean_g=MEAN[1], mean_b=MEAN[2], std_r=STD[0], std_g=STD[1], std_b=STD[2])


def _val_reference(img, resize, out_hw):
    """resize the shorter side (area resampling = PIL BOX), centre crop, normalize: computed here
    independently of mxnet/image_iter.py"""
    h, w = img.shape[:2]
    if w < h:
        nw, nh = resize, int(round(h * resize / w))
    else:
        nw, nh = int(round(w * resize / h)), resize
    im = Image.fromarray(img).resize((nw, nh), Image.BOX)
    a = np.asarray(im, dtype=np.float64)
    y0, x0 = (nh - out_hw) // 2, (nw - out_hw) // 2
    a = a[y0:y0 + out_hw, x0:x0 + out_hw]
    return ((a - MEAN) / STD).transpose(2, 0, 1)


def test_val_iterator_exact(tmp_path):
    """data/imagenet.py:188-208 (val): resize 36, centre 32x32, mean/std; batch 4 over 10 records:
    3 batches, the last one wraps around (pad 2); labels in file order."""
    imgs = _images(10, 1)
    path = tmp_path / "val.rec"
    _write_rec(path, imgs)
    it = mx.io.ImageRecordIter(path_imgrec=str(path), label_width=1, data_name="data", label_name="softmax_label",
                               resize=36, batch_size=4, data_shape=(3, 32, 32), scale=1, inter_method=2,
                               rand_crop=False, rand_mirror=False, preprocess_threads=3, **NORM)
    assert it.provide_data[0].shape == (4, 3, 32, 32) and it.provide_label[0].shape == (4,)
    batches = list(it)
    assert len(batches) == 3 and [b.pad for b in batches] == [0, 0, 2]
    got = np.concatenate([b.data[0].asnumpy() for b in batches])
    lab = np.concatenate([b.label[0].asnumpy() for b in batches])
    order = list(range(10)) + [0, 1]
    assert np.array_equal(lab, np.array(order, dtype=np.float32))
    for k, i in enumerate(order):
        ref = _val_reference(imgs[i], 36, 32)
        assert np.abs(got[k] - ref).max() < 1e-4, k
    it.reset()
    assert np.array_equal(next(it).data[0].asnumpy(), got[:4])


@pytest.mark.parametrize("parts", [1, 3])
def test_parts_cover_records_once(tmp_path, parts):
    """num_parts / part_index (data/imagenet.py:184-185 with kv.num_workers / kv.rank)."""
    path = tmp_path / "p.rec"
    _write_rec(path, _images(11, 2))
    seen = []
    for k in range(parts):
        it = mx.io.ImageRecordIter(path_imgrec=str(path), data_shape=(3, 24, 24), batch_size=2, resize=24,
                                   num_parts=parts, part_index=k, round_batch=False)
        for b in it:
            seen += list(b.label[0].asnumpy()[: 2 - b.pad])
    assert sorted(seen) == list(range(11))


TRAIN_KW = dict(label_width=1, data_name="data", label_name="softmax_label", resize=40, pad=0, fill_value=127,
                random_resized_crop=True, max_random_area=1.0, min_random_area=0.08, max_aspect_ratio=4.0 / 3.0,
                min_aspect_ratio=3.0 / 4.0, brightness=0.4, contrast=0.4, saturation=0.4, pca_noise=0.1, scale=1,
                inter_method=2, rand_mirror=True, shuffle=True, shuffle_chunk_size=4096, preprocess_threads=4,
                prefetch_buffer=16, num_parts=1, part_index=0, **NORM)


def test_train_iterator_reference_arguments(tmp_path):
    """The train iterator with the argument set of data/imagenet.py:153-186: shapes, the value range
    of the un-normalized pixels, seeded determinism, shuffling, and different crops per epoch."""
    path = tmp_path / "train.rec"
    _write_rec(path, _images(12, 4), fmt=".jpg")
    mk = lambda: mx.io.ImageRecordIter(path_imgrec=str(path), data_shape=(3, 32, 32), batch_size=6, seed=11,
                                       **TRAIN_KW)
    a, b = mk(), mk()
    bs = list(a)
    ea = [x.data[0].asnumpy() for x in bs]
    la = [x.label[0].asnumpy() for x in bs]
    eb = [x.data[0].asnumpy() for x in b]
    assert len(ea) == 2 and all(e.shape == (6, 3, 32, 32) for e in ea)
    assert all(np.array_equal(x, y) for x, y in zip(ea, eb))
    px = np.concatenate(ea).transpose(0, 2, 3, 1) * STD + MEAN
    assert px.min() >= -1e-3 and px.max() <= 255 + 1e-3
    assert sorted(np.concatenate(la)) == list(range(12)) and list(np.concatenate(la)) != list(range(12))
    a.reset()
    e2 = [x.data[0].asnumpy() for x in a]
    assert not all(np.array_equal(x, y) for x, y in zip(ea, e2))


def test_cifar_arguments(tmp_path):
    """data/cifar10.py:12-33: pad 4 with fill 127, random 28x28 crops, mirror; the geometric / HSL
    augmenters the reference passes as 0 are accepted, non-zero ones raise."""
    path = tmp_path / "c.rec"
    _write_rec(path, [im[:32, :32] for im in _images(5, 5)])
    kw = dict(path_imgrec=str(path), label_width=1, data_name="data", label_name="softmax_label",
              data_shape=(3, 28, 28), batch_size=5, pad=4, fill_value=127, rand_crop=True, max_random_scale=1.0,
              min_random_scale=1.0, max_aspect_ratio=0, random_h=0, random_s=0, random_l=0, max_rotate_angle=0,
              max_shear_ratio=0, rand_mirror=True, shuffle=True, num_parts=1, part_index=0)
    x = next(mx.io.ImageRecordIter(**kw)).data[0].asnumpy()
    assert x.shape == (5, 3, 28, 28) and x.min() >= 0 and x.max() <= 255
    with pytest.raises(mx.MXNetError):
        mx.io.ImageRecordIter(**dict(kw, max_rotate_angle=10))


def test_module_trains_on_recordio_cpu(tmp_path):
    """A Module on mx.cpu() fed by the RecordIO iterator: ResNet-20 (symbol/resnet.py:123-148) steps
    over a tiny CIFAR-shaped .rec and its loss is finite."""
    from rn import graphs
    path = tmp_path / "t.rec"
    _write_rec(path, [im[:32, :32] for im in _images(8, 6)], labels=[float(i % 10) for i in range(8)])
    it = mx.io.ImageRecordIter(path_imgrec=str(path), data_shape=(3, 32, 32), batch_size=4, rand_mirror=True,
                               shuffle=True, **NORM)
    mod = mx.mod.Module(graphs.resnet20_cifar(), context=mx.cpu())
    mod.bind(data_shapes=it.provide_data, label_shapes=it.provide_label, for_training=True)
    mod.init_params(initializer=mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
    mod.init_optimizer(kvstore="local", optimizer="sgd", optimizer_params={"learning_rate": 0.05, "momentum": 0.9})
    metric = mx.metric.create("acc")
    for batch in it:
        mod.forward(batch, is_train=True)
        mod.backward()
        mod.update()
        mod.update_metric(metric, batch.label)
    prob = mod.get_outputs()[0].asnumpy()
    assert prob.shape == (4, 10) and np.isfinite(prob).all()
    assert 0.0 <= metric.get()[1] <= 1.0
