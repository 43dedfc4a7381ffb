"""mx.init: Xavier(rnd_type='gaussian', factor_type='in', magnitude=2) as used by train.py:221.

Name-suffix dispatch follows MXNet 1.x Initializer.__call__: *_weight -> _init_weight,
*_bias / *_beta / *moving_mean -> 0, *_gamma / *moving_var -> 1. Random numbers come from
numpy (seedable via mx.random.seed); MXNet's own RNG stream cannot be reproduced.
"""
import json

import numpy as np

from . import random as _random


class InitDesc(str):
    def __new__(cls, name, attrs=None, global_init=None):
        ret = super().__new__(cls, name)
        ret.attrs = attrs or {}
        ret.global_init = global_init
        return ret


class Initializer:
    def __init__(self, **kwargs):
        self._kwargs = kwargs

    def dumps(self):
        return json.dumps([self.__class__.__name__.lower(), self._kwargs])

    def __call__(self, desc, arr):
        name = str(desc)
        if name.endswith("_weight"):
            self._init_weight(name, arr)
        elif name.endswith("_bias") or name.endswith("_beta") or name.endswith("moving_mean") or \
                name.endswith("minmax"):
            arr[:] = 0.0
        elif name.endswith("_gamma") or name.endswith("moving_var") or name.endswith("moving_inv_var"):
            arr[:] = 1.0
        else:
            self._init_default(name, arr)

    def _init_weight(self, name, arr):
        raise NotImplementedError

    def _init_default(self, name, arr):
        raise ValueError("Unknown initialization pattern for %s" % name)


class Xavier(Initializer):
    def __init__(self, rnd_type="uniform", factor_type="avg", magnitude=3):
        super().__init__(rnd_type=rnd_type, factor_type=factor_type, magnitude=magnitude)
        self.rnd_type, self.factor_type, self.magnitude = rnd_type, factor_type, float(magnitude)

    def _init_weight(self, name, arr):
        shape = arr.shape
        hw = float(np.prod(shape[2:])) if len(shape) > 2 else 1.0
        fan_in, fan_out = shape[1] * hw, shape[0] * hw
        factor = {"avg": (fan_in + fan_out) / 2.0, "in": fan_in, "out": fan_out}[self.factor_type]
        scale = np.sqrt(self.magnitude / factor)
        rng = _random.rng()
        if self.rnd_type == "uniform":
            arr[:] = rng.uniform(-scale, scale, shape).astype(np.float32)
        else:
            arr[:] = rng.normal(0, scale, shape).astype(np.float32)


class Constant(Initializer):
    def __init__(self, value):
        super().__init__(value=value)
        self.value = value

    def __call__(self, desc, arr):
        arr[:] = self.value

    _init_weight = __call__


class Zero(Constant):
    def __init__(self):
        super().__init__(0.0)


class One(Constant):
    def __init__(self):
        super().__init__(1.0)


class Normal(Initializer):
    def __init__(self, sigma=0.01):
        super().__init__(sigma=sigma)
        self.sigma = sigma

    def _init_weight(self, name, arr):
        arr[:] = _random.rng().normal(0, self.sigma, arr.shape).astype(np.float32)


class Uniform(Initializer):
    def __init__(self, scale=0.07):
        super().__init__(scale=scale)
        self.scale = scale

    def _init_weight(self, name, arr):
        arr[:] = _random.rng().uniform(-self.scale, self.scale, arr.shape).astype(np.float32)


class MSRAPrelu(Xavier):
    def __init__(self, factor_type="avg", slope=0.25):
        super().__init__("gaussian", factor_type, 2.0 / (1 + slope ** 2))
