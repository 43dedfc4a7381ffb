"""mx.Context / mx.cpu / mx.gpu (train.py:34, data/imagenet.py:17)."""


class Context:
    devtype2str = {1: "cpu", 2: "gpu", 3: "cpu_pinned"}
    devstr2type = {"cpu": 1, "gpu": 2, "cpu_pinned": 3}
    _default = None

    def __init__(self, device_type, device_id=0):
        if isinstance(device_type, Context):
            device_type, device_id = device_type.device_type, device_type.device_id
        self.device_type = device_type if isinstance(device_type, str) else self.devtype2str[device_type]
        self.device_id = int(device_id)

    @property
    def device_typeid(self):
        return self.devstr2type[self.device_type]

    def torch_device(self):
        return "cuda:%d" % self.device_id if self.device_type == "gpu" else "cpu"

    def __eq__(self, other):
        return isinstance(other, Context) and (self.device_type, self.device_id) == (other.device_type,
                                                                                      other.device_id)

    def __hash__(self):
        return hash((self.device_type, self.device_id))

    def __repr__(self):
        return "%s(%d)" % (self.device_type, self.device_id)

    __str__ = __repr__


def cpu(device_id=0):
    return Context("cpu", device_id)


def cpu_pinned(device_id=0):
    return Context("cpu_pinned", device_id)


def gpu(device_id=0):
    return Context("gpu", device_id)


def current_context():
    return Context._default or cpu()


def num_gpus():
    import torch
    return torch.cuda.device_count()
