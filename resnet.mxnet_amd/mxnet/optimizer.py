"""mx.optimizer: SGD with momentum, MXNet 1.x semantics (train.py:186-194).

The arithmetic runs in librn (rn_sgd_mom_update, one fused multi-tensor launch); this class
holds the hyper-parameters and the learning-rate schedule like MXNet's Optimizer does.
"""
from .base import MXNetError


class Optimizer:
    def __init__(self, rescale_grad=1.0, param_idx2name=None, wd=0.0, clip_gradient=None, learning_rate=0.01,
                 lr_scheduler=None, sym=None, begin_num_update=0, multi_precision=False, param_dict=None, **kwargs):
        self.rescale_grad = rescale_grad
        self.lr = learning_rate
        self.lr_scheduler = lr_scheduler
        if lr_scheduler is not None:
            # MXNet: Optimizer.__init__ sets lr_scheduler.base_lr = learning_rate
            self.lr_scheduler.base_lr = learning_rate
        self.wd = wd
        self.begin_num_update = begin_num_update
        self.num_update = begin_num_update
        self.clip_gradient = clip_gradient
        self.multi_precision = multi_precision
        self.idx2name = dict(param_idx2name or {})
        self.lr_mult, self.wd_mult = {}, {}

    def _get_lr(self):
        if self.lr_scheduler is not None:
            return self.lr_scheduler(self.num_update)
        return self.lr

    def step_lr(self):
        """Advance num_update (MXNet _update_count) and return the lr for this update."""
        self.num_update += 1
        return self._get_lr()

    @property
    def learning_rate(self):
        return self._get_lr()

    def set_learning_rate(self, lr):
        if self.lr_scheduler is not None:
            raise UserWarning("LRScheduler of the optimizer has already been defined")
        self.lr = lr


class SGD(Optimizer):
    def __init__(self, momentum=0.0, lazy_update=True, **kwargs):
        super().__init__(**kwargs)
        self.momentum = momentum


_REG = {"sgd": SGD}


def create(name, **kwargs):
    if isinstance(name, Optimizer):
        return name
    cls = _REG.get(name.lower())
    if cls is None:
        raise MXNetError("optimizer %s is not supported by the MI355X runtime (supported: %s)" % (name, list(_REG)))
    return cls(**kwargs)


def register(klass):
    _REG[klass.__name__.lower()] = klass
    return klass
