"""bench.py's multi-GPU launch: `python bench.py --gpus N`, as the driver runs it,
must start N rank processes itself (one per GPU, torch.distributed env set as torch.distributed.run
would), or, under a launcher, agree with its WORLD_SIZE. The reference drives its GPUs from one
`python train.py` (train.py:34-35, core/solver.py:58-61,121); here each GPU gets its own rank."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_disagreeing_with_launcher_world_is_an_error():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="3", RANK="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "disagrees with WORLD_SIZE=3" in r.stderr


def test_nccl_launch_needs_as_many_gpus_as_ranks():
    # no GPU in this container: an RCCL launch of 2 ranks is refused before any rank starts
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("needs a host with fewer than 2 GPUs")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(RN_DIST_BACKEND="nccl"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "GPU(s) visible" in r.stderr


def test_launched_rank_failure_propagates():
    # gloo rehearsal on a host without a GPU: both ranks start and fail at their first GPU call;
    # the launcher reports the failing rank and exits non-zero instead of hanging
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline"], env=_env(RN_DIST_BACKEND="gloo"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "exited with" in r.stderr
    assert r.stdout.strip() == ""  # no JSON line from a failed job


@pytest.mark.gpu
def test_bench_gpus2_runs_two_ranks(gpu):
    """`python bench.py --gpus 2` on the one-GPU box with gloo as the transport: two rank processes
    share cuda:0 and the JSON line reports the two-rank job (whole-job images/s, dp2, global batch
    512, the all-reduce backend and buckets)."""
    cmd = [sys.executable, "-u", BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
           "--pcie-steps", "0"]
    r = subprocess.run(cmd, env=_env(RN_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=600,
                       cwd=REPO)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    print(json.dumps({k: out[k] for k in ("value", "ms_per_step", "n_gpus", "config", "allreduce")}))
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 512
    assert out["allreduce"]["backend"] == "gloo" and out["allreduce"]["world"] == 2
    assert out["allreduce"]["buckets"] >= 4  # 102 MB of gradients in 25 MB buckets
    assert out["allreduce"]["launch"].startswith("one process per GPU (bench.py --gpus")
    assert abs(out["config"]["per_gpu_images_per_sec"] * 2 - out["value"]) < 0.05 * out["value"]
    assert out["outputs_finite"]
    assert "cpu_baseline" not in out
