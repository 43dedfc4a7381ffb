"""rn: host side of the MI355X runtime -- librn binding, graph lowering/executor, RCCL DP."""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
if _ROOT not in sys.path:  # makes the `mxnet` shim importable next to rn
    sys.path.insert(0, _ROOT)
