"""mx.metric: Accuracy / TopKAccuracy / CrossEntropy (train.py:205-207, core/solver.py:134-139).

When the module owns the predictions on the GPU, `update_device` queues the per-batch device
counters produced by the fused SoftmaxOutput kernel (loss sum, top-1 hits, top-5 hits) and
they are only read back when the value is requested (Speedometer every `frequent` batches),
instead of forcing a device->host sync every step. Host `update` keeps MXNet's semantics.
"""
import numpy as np

from .base import MXNetError


class EvalMetric:
    _dev_slot = None

    def __init__(self, name, output_names=None, label_names=None, **kwargs):
        self.name = str(name)
        self.output_names, self.label_names = output_names, label_names
        self._kwargs = kwargs
        self.reset()

    def reset(self):
        self.num_inst = 0
        self.sum_metric = 0.0
        self._pending = []

    def update_device(self, stats, n):
        """stats: a device tensor snapshot [loss, top1, top5, _]; n: batch rows."""
        if self._dev_slot is None:
            raise MXNetError("metric %s has no device path" % self.name)
        self._pending.append((stats, n))

    def _resolve(self):
        if self._pending:
            import torch
            vals = torch.stack([s for s, _ in self._pending]).cpu().numpy()
            for (s, n), v in zip(self._pending, vals):
                self.sum_metric += float(v[self._dev_slot])
                self.num_inst += n
            self._pending = []

    def get(self):
        self._resolve()
        if self.num_inst == 0:
            return self.name, float("nan")
        return self.name, self.sum_metric / self.num_inst

    def get_name_value(self):
        name, value = self.get()
        if not isinstance(name, list):
            name, value = [name], [value]
        return list(zip(name, value))

    def update(self, labels, preds):
        raise NotImplementedError

    def __str__(self):
        return "EvalMetric: {}".format(dict(self.get_name_value()))


def _np(x):
    return x.asnumpy() if hasattr(x, "asnumpy") else np.asarray(x)


class Accuracy(EvalMetric):
    _dev_slot = 1

    def __init__(self, axis=1, name="accuracy", **kwargs):
        super().__init__(name, **kwargs)
        self.axis = axis

    def update(self, labels, preds):
        for label, pred in zip(labels, preds):
            pred = _np(pred)
            if pred.ndim > 1 and pred.shape != _np(label).shape:
                pred = np.argmax(pred, axis=self.axis)
            label = _np(label).astype("int32").ravel()
            pred = pred.astype("int32").ravel()
            self.sum_metric += float((pred == label).sum())
            self.num_inst += len(pred)


class TopKAccuracy(EvalMetric):
    def __init__(self, top_k=1, name="top_k_accuracy", **kwargs):
        super().__init__(name, **kwargs)
        self.top_k = top_k
        self.name += "_%d" % top_k
        if top_k == 5:
            self._dev_slot = 2
        elif top_k == 1:
            self._dev_slot = 1

    def update(self, labels, preds):
        for label, pred in zip(labels, preds):
            pred = _np(pred).astype("float32")
            label = _np(label).astype("int32").ravel()
            order = np.argsort(pred, axis=1)
            top = order[:, -self.top_k:]
            self.sum_metric += float((top == label[:, None]).any(axis=1).sum())
            self.num_inst += pred.shape[0]


class CrossEntropy(EvalMetric):
    _dev_slot = 0

    def __init__(self, eps=1e-12, name="cross-entropy", **kwargs):
        super().__init__(name, **kwargs)
        self.eps = eps

    def update(self, labels, preds):
        for label, pred in zip(labels, preds):
            pred = _np(pred)
            label = _np(label).ravel().astype("int64")
            prob = pred[np.arange(label.shape[0]), label]
            self.sum_metric += float((-np.log(prob + self.eps)).sum())
            self.num_inst += label.shape[0]


class CompositeEvalMetric(EvalMetric):
    def __init__(self, metrics=None, name="composite", **kwargs):
        self.metrics = [create(m) for m in (metrics or [])]
        super().__init__(name, **kwargs)

    def add(self, metric):
        self.metrics.append(create(metric))

    def reset(self):
        for m in getattr(self, "metrics", []):
            m.reset()

    def update(self, labels, preds):
        for m in self.metrics:
            m.update(labels, preds)

    def update_device(self, stats, n):
        for m in self.metrics:
            m.update_device(stats, n)

    def get(self):
        names, values = [], []
        for m in self.metrics:
            n, v = m.get()
            names.append(n)
            values.append(v)
        return names, values

    @property
    def _dev_slot(self):
        return 0 if all(m._dev_slot is not None for m in self.metrics) else None


_ALIASES = {"acc": Accuracy, "accuracy": Accuracy, "top_k_accuracy": TopKAccuracy, "top_k_acc": TopKAccuracy,
            "ce": CrossEntropy, "cross-entropy": CrossEntropy}


def create(metric, *args, **kwargs):
    if isinstance(metric, EvalMetric):
        return metric
    if isinstance(metric, (list, tuple)):
        return CompositeEvalMetric([create(m) for m in metric])
    if callable(metric) and not isinstance(metric, str):
        raise MXNetError("custom metric functions are not supported")
    cls = _ALIASES.get(metric.lower())
    if cls is None:
        raise MXNetError("metric %s not supported" % metric)
    return cls(*args, **kwargs)
