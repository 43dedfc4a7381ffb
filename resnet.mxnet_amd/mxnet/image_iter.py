"""mx.io.ImageRecordIter: the real-data input of the reference (data/imagenet.py:153-208 train / val,
data/imagenet.py:54-80 MultipleDataIter, data/cifar10.py:12-46) over RecordIO files
(mxnet/recordio.py).

Host side, as MXNet's own iterator: records are read from the .rec file, decoded (PIL) and augmented
by `preprocess_threads` worker threads (PIL releases the GIL while decoding and resampling), and
assembled into NCHW float32 batches in pinned host memory, `prefetch_buffer` batches ahead; the
Module's executor copies each batch to HBM on its copy stream, overlapped with the previous step.

Augmentation, in MXNet 1.x DefaultImageAugmenter order: resize (shorter side to `resize`), pad
(`pad`, `fill_value`), crop (random_resized_crop: area fraction U[min_random_area, max_random_area],
aspect ratio log-uniform in [min_aspect_ratio, max_aspect_ratio], 10 attempts, else the centre
square; rand_crop: a random data_shape window of the (scaled) image; else the centre window),
resampling with `inter_method` (0 nearest, 1 bilinear, 2 area, 3 bicubic, 4 lanczos, 9/10 bilinear),
colour (brightness / contrast / saturation in random order, then pca_noise lighting, clipped to the
uint8 range), mirror, then (x - mean) / std * scale per RGB channel. Parity with MXNet's C++
augmenter (its RNG streams and OpenCV resamplers) is unpinned: MXNet is not available here; the
deterministic val path is checked against an independent PIL/numpy recomputation
(tests/test_recordio_cpu.py).
"""
import concurrent.futures as cf
import io
import math
import threading

import numpy as np

from . import ndarray as nd
from .base import MXNetError
from .context import cpu_pinned
from .io import DataBatch, DataDesc, DataIter
from .recordio import MXRecordIO, unpack

_PCA_EIGVAL = np.array([55.46, 4.794, 1.148])
_PCA_EIGVEC = np.array([[-0.5675, 0.7192, 0.4009], [-0.5808, -0.0045, -0.8140], [-0.5836, -0.6948, 0.4203]])
_LUMA = np.array([0.299, 0.587, 0.114], dtype=np.float32)


def _resample(method):
    from PIL import Image
    return {0: Image.NEAREST, 1: Image.BILINEAR, 2: Image.BOX, 3: Image.BICUBIC, 4: Image.LANCZOS}.get(
        int(method), Image.BILINEAR)


class ImageRecordIter(DataIter):
    _UNSUPPORTED = ("max_rotate_angle", "max_shear_ratio", "random_h", "random_s", "random_l", "max_img_size",
                    "min_img_size", "rotate")

    def __init__(self, path_imgrec, data_shape, batch_size, label_width=1, data_name="data",
                 label_name="softmax_label", path_imgidx=None, resize=-1, pad=0, fill_value=127, rand_crop=False,
                 random_resized_crop=False, max_random_area=1.0, min_random_area=1.0, max_aspect_ratio=0.0,
                 min_aspect_ratio=None, max_random_scale=1.0, min_random_scale=1.0, brightness=0.0, contrast=0.0,
                 saturation=0.0, pca_noise=0.0, mean_r=0.0, mean_g=0.0, mean_b=0.0, std_r=1.0, std_g=1.0,
                 std_b=1.0, scale=1.0, inter_method=1, rand_mirror=False, shuffle=False, shuffle_chunk_size=0,
                 preprocess_threads=4, prefetch_buffer=4, num_parts=1, part_index=0, round_batch=True, seed=0,
                 dtype="float32", **kwargs):
        super().__init__(batch_size)
        for k, v in kwargs.items():
            if k in self._UNSUPPORTED and v:
                raise MXNetError("ImageRecordIter: %s=%r is not implemented (geometric / HSL augmenters)" % (k, v))
            if k not in self._UNSUPPORTED and k not in ("verbose", "data_nthreads"):
                raise MXNetError("ImageRecordIter: unknown argument %s" % k)
        if len(data_shape) != 3 or data_shape[0] not in (1, 3):
            raise MXNetError("ImageRecordIter: data_shape must be (3, H, W) or (1, H, W)")
        self.data_shape = tuple(int(v) for v in data_shape)
        self.data_name, self.label_name = data_name, label_name
        self.label_width = int(label_width)
        self.resize, self.pad, self.fill_value = int(resize), int(pad), int(fill_value)
        self.rand_crop, self.random_resized_crop = bool(rand_crop), bool(random_resized_crop)
        self.area = (float(min_random_area), float(max_random_area))
        lo = float(min_aspect_ratio) if min_aspect_ratio is not None else (
            1.0 / max_aspect_ratio if max_aspect_ratio else 1.0)
        self.ratio = (lo, float(max_aspect_ratio) if max_aspect_ratio else 1.0)
        self.scale_rng = (float(min_random_scale), float(max_random_scale))
        self.brightness, self.contrast, self.saturation = float(brightness), float(contrast), float(saturation)
        self.pca_noise = float(pca_noise)
        self.mean = np.array([mean_r, mean_g, mean_b], dtype=np.float32)[: self.data_shape[0]]
        self.std = np.array([std_r, std_g, std_b], dtype=np.float32)[: self.data_shape[0]]
        self.scale = float(scale)
        self.inter_method = int(inter_method)
        self.rand_mirror, self.shuffle = bool(rand_mirror), bool(shuffle)
        self.round_batch = bool(round_batch)
        self.seed = int(seed)
        self.epoch = 0
        self.threads = max(1, int(preprocess_threads))
        self.prefetch = max(1, int(prefetch_buffer))

        rec = MXRecordIO(path_imgrec, "r")
        if path_imgidx:
            with open(path_imgidx) as f:
                offs = sorted(int(line.split("\t")[1]) for line in f if line.strip())
        else:
            offs = rec.scan_offsets()
        rec.close()
        self.path = path_imgrec
        # MXNet splits the input into num_parts contiguous parts (InputSplit); part_index reads one.
        # The split here is by record count; MXNet's InputSplit cuts by bytes and moves each cut to the
        # next record boundary, so parts can differ by a few records (sharding parity unpinned)
        n = len(offs)
        a, b = n * int(part_index) // int(num_parts), n * (int(part_index) + 1) // int(num_parts)
        self.offsets = offs[a:b]
        if not self.offsets:
            raise MXNetError("ImageRecordIter: part %d of %d of %s holds no records" % (part_index, num_parts,
                                                                                       path_imgrec))
        self._local = threading.local()
        self._pool = cf.ThreadPoolExecutor(max_workers=self.threads)
        self._prefetcher = cf.ThreadPoolExecutor(max_workers=1)
        self._pending = []
        self.reset()

    # ------------------------------------------------------------------ DataIter protocol
    @property
    def provide_data(self):
        return [DataDesc(self.data_name, (self.batch_size,) + self.data_shape)]

    @property
    def provide_label(self):
        shp = (self.batch_size,) if self.label_width == 1 else (self.batch_size, self.label_width)
        return [DataDesc(self.label_name, shp)]

    def reset(self):
        for f in self._pending:
            f.cancel()
        self._pending = []
        order = np.arange(len(self.offsets))
        if self.shuffle:
            np.random.default_rng((self.seed, self.epoch)).shuffle(order)
        self.epoch += 1
        self._order = order
        self._cursor = 0
        self._epoch_seed = (self.seed, self.epoch)
        self._batch_no = 0
        self._fill()

    def _fill(self):
        while len(self._pending) < self.prefetch and self._cursor < len(self._order):
            idx = self._order[self._cursor:self._cursor + self.batch_size]
            pad = self.batch_size - len(idx)
            if pad and self.round_batch:  # the last batch is filled from the first records; `pad` counts them
                idx = np.concatenate([idx, np.resize(self._order, pad)])
            # round_batch=False: the last batch keeps only its own records, the `pad` slots are zeros
            # (MXNet's BatchLoader leaves them unfilled and reports the same pad)
            self._cursor += self.batch_size
            self._pending.append(self._prefetcher.submit(self._make_batch, idx, pad, self._batch_no))
            self._batch_no += 1

    def next(self):
        if not self._pending:
            raise StopIteration
        batch = self._pending.pop(0).result()
        self._fill()
        return batch

    # ------------------------------------------------------------------ one batch
    def _reader(self):
        r = getattr(self._local, "rec", None)
        if r is None:
            r = self._local.rec = MXRecordIO(self.path, "r")
        return r

    def _make_batch(self, idx, pad, batch_no):
        c, h, w = self.data_shape
        data = np.zeros((self.batch_size, c, h, w), dtype=np.float32)
        label = np.zeros((self.batch_size, self.label_width), dtype=np.float32)

        def one(i):
            r = self._reader()
            r.seek(self.offsets[idx[i]])
            header, img = unpack(r.read())
            rng = np.random.default_rng(self._epoch_seed + (batch_no, i))
            data[i] = self.augment(img, rng)
            lab = np.atleast_1d(np.asarray(header.label, dtype=np.float32))
            label[i] = lab[: self.label_width]

        list(self._pool.map(one, range(len(idx))))
        lab = label[:, 0] if self.label_width == 1 else label
        return DataBatch([nd.array(data, ctx=cpu_pinned(0))], [nd.array(lab, ctx=cpu_pinned(0))], pad=pad,
                         provide_data=self.provide_data, provide_label=self.provide_label)

    # ------------------------------------------------------------------ augmentation
    def augment(self, encoded, rng):
        """encoded image bytes -> (C, H, W) float32 normalized, data/imagenet.py's pipeline."""
        from PIL import Image
        c, oh, ow = self.data_shape
        im = Image.open(io.BytesIO(encoded))
        im = im.convert("L" if c == 1 else "RGB")
        method = _resample(self.inter_method)
        if self.resize > 0:  # shorter side -> resize
            W, H = im.size
            if W < H:
                nw, nh = self.resize, int(round(H * self.resize / W))
            else:
                nw, nh = int(round(W * self.resize / H)), self.resize
            if (nw, nh) != (W, H):
                im = im.resize((nw, nh), method)
        if self.pad > 0:
            W, H = im.size
            canvas = Image.new(im.mode, (W + 2 * self.pad, H + 2 * self.pad),
                               self.fill_value if c == 1 else (self.fill_value,) * 3)
            canvas.paste(im, (self.pad, self.pad))
            im = canvas
        W, H = im.size
        if self.random_resized_crop:
            box = None
            for _ in range(10):
                target = W * H * rng.uniform(*self.area)
                ratio = math.exp(rng.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
                cw = int(round(math.sqrt(target * ratio)))
                ch = int(round(math.sqrt(target / ratio)))
                if 0 < cw <= W and 0 < ch <= H:
                    x0 = int(rng.integers(0, W - cw + 1))
                    y0 = int(rng.integers(0, H - ch + 1))
                    box = (x0, y0, x0 + cw, y0 + ch)
                    break
            if box is None:  # the centre square
                s = min(W, H)
                box = ((W - s) // 2, (H - s) // 2, (W - s) // 2 + s, (H - s) // 2 + s)
            im = im.resize((ow, oh), method, box=box)
        else:
            if self.rand_crop and self.scale_rng != (1.0, 1.0):
                sc = rng.uniform(*self.scale_rng)
                im = im.resize((max(ow, int(round(W * sc))), max(oh, int(round(H * sc)))), method)
                W, H = im.size
            if W < ow or H < oh:  # too small for the window: scale up the shorter side
                f = max(ow / W, oh / H)
                im = im.resize((max(ow, int(math.ceil(W * f))), max(oh, int(math.ceil(H * f)))), method)
                W, H = im.size
            if self.rand_crop:
                x0, y0 = int(rng.integers(0, W - ow + 1)), int(rng.integers(0, H - oh + 1))
            else:
                x0, y0 = (W - ow) // 2, (H - oh) // 2
            im = im.crop((x0, y0, x0 + ow, y0 + oh))
        a = np.asarray(im, dtype=np.float32)
        if a.ndim == 2:
            a = a[:, :, None]
        if c == 3 and (self.brightness or self.contrast or self.saturation or self.pca_noise):
            a = self._color(a, rng)
        if self.rand_mirror and rng.random() < 0.5:
            a = a[:, ::-1]
        a = (a - self.mean) / self.std
        if self.scale != 1.0:
            a = a * self.scale
        return a.transpose(2, 0, 1)

    def _color(self, a, rng):
        jit = []
        if self.brightness:
            jit.append("b")
        if self.contrast:
            jit.append("c")
        if self.saturation:
            jit.append("s")
        for k in rng.permutation(jit):
            if k == "b":
                a = a * (1.0 + rng.uniform(-self.brightness, self.brightness))
            elif k == "c":
                alpha = 1.0 + rng.uniform(-self.contrast, self.contrast)
                gray = float((a @ _LUMA).mean())
                a = a * alpha + gray * (1.0 - alpha)
            else:
                alpha = 1.0 + rng.uniform(-self.saturation, self.saturation)
                gray = (a @ _LUMA)[:, :, None]
                a = a * alpha + gray * (1.0 - alpha)
        if self.pca_noise:
            alpha = rng.normal(0.0, self.pca_noise, 3)
            a = a + (_PCA_EIGVEC @ (alpha * _PCA_EIGVAL)).astype(np.float32)
        return np.clip(a, 0.0, 255.0).astype(np.float32)

    def __del__(self):
        for ex in (getattr(self, "_prefetcher", None), getattr(self, "_pool", None)):
            if ex is not None:
                ex.shutdown(wait=False)
