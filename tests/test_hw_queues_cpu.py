"""rn/__init__.py raises HIP's hardware-queue count before the process's first HIP call (profiles/r05/streams:
with HIP's 4 queues the RCCL process group's pool streams moved the weight-gradient stream onto the compute
stream's queue and the two branches of the backward ran serialised, 25.8 vs 20.4 ms per step). Each case
imports rn in a fresh interpreter with a given environment and reads GPU_MAX_HW_QUEUES back."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _queues(**env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("GPU_MAX_HW_QUEUES", "RN_HW_QUEUES", "RN_DIST_BACKEND", "WORLD_SIZE")}
    e.update(env)
    code = ("import os, sys; sys.path.insert(0, %r); import rn; print(os.environ.get('GPU_MAX_HW_QUEUES'))"
            % os.path.join(REPO, "resnet.mxnet_amd"))
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


@pytest.mark.parametrize("env,want", [
    ({}, "8"),                                                      # one process per GPU: 8 queues
    ({"GPU_MAX_HW_QUEUES": "4"}, "8"),                              # HIP's default raised
    ({"GPU_MAX_HW_QUEUES": "16"}, "16"),                            # a larger setting is kept
    ({"RN_HW_QUEUES": "6"}, "6"),                                   # explicit count
    ({"RN_HW_QUEUES": "64"}, "None"),                               # beyond 32: left alone
    ({"RN_DIST_BACKEND": "gloo", "WORLD_SIZE": "2"}, "4"),          # ranks sharing one GPU (rehearsal)
    ({"RN_DIST_BACKEND": "gloo", "WORLD_SIZE": "2", "GPU_MAX_HW_QUEUES": "8"}, "4"),
    ({"RN_DIST_BACKEND": "nccl", "WORLD_SIZE": "8"}, "8"),          # one rank per GPU over RCCL
])
def test_hardware_queue_count(env, want):
    assert _queues(**env) == want


@pytest.mark.parametrize("ids,want", [((0, 0), "4"), ((0, 1), "8")])
def test_module_workers_queue_count(monkeypatch, ids, want):
    """mx.mod.Module over repeated device ids (two contexts on one GPU) spawns workers that
    import rn while unpickling, before the worker sets WORLD_SIZE: the shared-GPU queue count (4) must be
    in the environment the spawn copies, and the parent's own 8 must not leak into them. Distinct
    devices keep 8 per process."""
    import mxnet as mx
    from rn import graphs
    monkeypatch.setenv("RN_DRY_RUN", "1")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("RN_DIST_BACKEND", raising=False)
    monkeypatch.delenv("RN_HW_QUEUES", raising=False)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "8")  # what the parent's `import rn` wrote
    mod = mx.mod.Module(graphs.resnet20_cifar(), context=[mx.gpu(i) for i in ids])
    try:
        mod.bind(data_shapes=[("data", (4, 3, 32, 32))], label_shapes=[("softmax_label", (4,))])
        assert mod._group.call("env", "GPU_MAX_HW_QUEUES") == [want, want]
        assert os.environ["GPU_MAX_HW_QUEUES"] == "8" and "RN_DIST_BACKEND" not in os.environ  # parent unchanged
    finally:
        mod.close()
