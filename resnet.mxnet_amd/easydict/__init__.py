"""Minimal `easydict` (not installed in this image) so config/edict_config.py imports unchanged."""


class EasyDict(dict):
    def __init__(self, d=None, **kwargs):
        super().__init__()
        d = dict(d or {}, **kwargs)
        for k, v in d.items():
            setattr(self, k, v)

    def __setattr__(self, name, value):
        if isinstance(value, dict) and not isinstance(value, EasyDict):
            value = EasyDict(value)
        elif isinstance(value, (list, tuple)):
            value = type(value)(EasyDict(x) if isinstance(x, dict) and not isinstance(x, EasyDict) else x
                                for x in value)
        super().__setattr__(name, value)
        super().__setitem__(name, value)

    __setitem__ = __setattr__

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name)

    def __delattr__(self, name):
        del self[name]

    def update(self, e=None, **f):
        d = dict(e or {}, **f)
        for k, v in d.items():
            setattr(self, k, v)

    def pop(self, k, *args):
        if hasattr(self, k) and k in self.__dict__:
            object.__delattr__(self, k)
        return super().pop(k, *args)
