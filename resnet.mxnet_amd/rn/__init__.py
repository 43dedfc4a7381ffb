"""rn: host side of the MI355X runtime -- librn binding, graph lowering/executor, RCCL DP."""
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
if _ROOT not in sys.path:  # makes the `mxnet` shim importable next to rn
    sys.path.insert(0, _ROOT)

# Hardware queues per process (RN_HW_QUEUES, default 8; HIP's own default is 4). HIP deals its streams
# round-robin over GPU_MAX_HW_QUEUES hardware queues, and a queue runs its packets in order whichever
# stream they came from. With 4, once RCCL's process group had taken streams from torch's pool the
# executor's weight-gradient stream landed on the compute stream's queue and the two branches of the
# backward ran serialised: 25.96 vs 20.45 ms per step at world 1 with the all-reduce hooks on; with 8
# queues 20.82 vs 20.45 (profiles/r05/streams). Only effective before the process's first HIP call,
# which importing rn precedes in bench.py, train.py (via the mxnet shim) and the tests. Several ranks
# sharing ONE GPU (the gloo rehearsals of the N > 1 path, tests/test_dist_gpu.py) keep HIP's 4: 8 per
# process there oversubscribe the hardware queue slots (a world-2 test step took minutes).
_shared = os.environ.get("RN_DIST_BACKEND") == "gloo" and int(os.environ.get("WORLD_SIZE", "1") or 1) > 1
_q = os.environ.get("RN_HW_QUEUES", "4" if _shared else "8")
try:
    if (_shared or int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < int(_q)) and 1 <= int(_q) <= 32:
        os.environ["GPU_MAX_HW_QUEUES"] = _q
except ValueError:
    pass
