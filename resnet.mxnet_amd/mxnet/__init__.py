"""`mxnet` drop-in for the XiaotaoChen/resnet.mxnet training path, running on MI355X.

Put `resnet.mxnet_amd/` on PYTHONPATH and the reference's train.py / core/solver.py /
symbol/resnet*.py / resnext*.py import this package as `mxnet`: graphs are built with the
same mx.sym operator surface and executed by the C-ABI HIP runtime librn (rn/), with
RCCL data parallelism replacing the kvstore. Only the hot path is provided.
"""
__version__ = "1.3.0-mi355x"

from .base import MXNetError
from .context import Context, cpu, gpu, cpu_pinned, current_context, num_gpus
from . import base
from . import context
from . import ndarray
from . import ndarray as nd
from . import symbol
from . import symbol as sym
from . import io
from . import recordio
from . import initializer
from . import initializer as init
from . import optimizer
from . import lr_scheduler
from . import metric
from . import callback
from . import model
from . import operator
from . import kvstore
from . import kvstore as kv
from . import module
from . import module as mod
from . import random
from . import viz
