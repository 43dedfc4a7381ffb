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
    # overlap evidence: per-bucket launch offsets inside the backward, the exposed
    # communication after it, bus bandwidth
    ar = out["allreduce"]
    for key in ("exposed_ms", "exposed_ms_max_over_ranks", "backward_ms", "comm_window_ms",
                "bucket_launch_offsets_ms", "bus_gbs", "bytes_per_step", "steps_timed"):
        assert key in ar, key
    # (the event records ride on the last timed step only: on every step they cost ~1.7 % of it)
    assert ar["steps_timed"] == 1 and len(ar["bucket_launch_offsets_ms"]) == ar["buckets"]
    assert out["family_timing"] == "HIP events on the last of the 3 timed steps"
    offs = ar["bucket_launch_offsets_ms"]
    # the first bucket leaves during the backward (the same step's: two ranks sharing one GPU vary a lot)
    assert offs == sorted(offs) and offs[0] < ar["backward_ms_last"]
    assert ar["exposed_ms"] >= 0 and ar["bus_gbs"] > 0
    assert out["allreduce"]["launch"].startswith("one process per GPU (bench.py --gpus")
    assert abs(out["config"]["per_gpu_images_per_sec"] * 2 - out["value"]) < 0.05 * out["value"]
    assert out["outputs_finite"]
    assert "cpu_baseline" not in out


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGINT"])
def test_launcher_signal_stops_every_rank(tmp_path, sig):
    """the ranks run in their own sessions, so a SIGTERM / SIGINT to the launcher (a
    driver timeout, Ctrl-C) must take them down explicitly instead of orphaning them on their GPUs.
    Two stand-in ranks (sleepers that record their pids) under bench.launch_ranks; the launcher
    is signalled and must exit non-zero with both ranks gone."""
    import signal
    import time
    pidfile = tmp_path / "pids"
    rank_cmd = [sys.executable, "-c",
                "import os, time; open(%r, 'a').write('%%d\\n' %% os.getpid()); time.sleep(300)" % str(pidfile)]
    code = ("import sys; sys.path.insert(0, %r); import bench; sys.exit(bench.launch_ranks(2, [], cmd=%r))"
            % (REPO, rank_cmd))
    parent = subprocess.Popen([sys.executable, "-c", code], env=_env(RN_DIST_BACKEND="gloo"),
                              stderr=subprocess.PIPE, text=True)
    deadline = time.time() + 120
    while time.time() < deadline:
        if pidfile.exists() and len(pidfile.read_text().split()) == 2:
            break
        time.sleep(0.2)
    pids = [int(x) for x in pidfile.read_text().split()]
    assert len(pids) == 2
    parent.send_signal(getattr(signal, sig))
    _, err = parent.communicate(timeout=60)
    assert parent.returncode == 128 + getattr(signal, sig), err
    assert "stopping every rank" in err
    for pid in pids:
        gone = False
        for _ in range(50):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                gone = True
                break
            time.sleep(0.1)
        assert gone, pid


def test_pmc_traffic_reads_the_committed_summary(tmp_path):
    """roofline.traffic went null when the PMC summary started nesting families
    under "hbm". The committed summary must resolve the dominant family; the flat round-2 form and a
    missing family are handled."""
    sys.path.insert(0, REPO)
    import bench
    b, src = bench.pmc_traffic("igemm_big_kernel<224x256>")
    assert src is not None and src.startswith("profiles/")
    # (~275 MB per launch in r03-r05; 185 MB in r06, whose streamed conv1 data gradients left the family)
    assert 1.5e8 < b < 4.0e8, b
    flat = tmp_path / "flat.json"
    flat.write_text(json.dumps({"fam": {"launches": 3, "hbm_bytes": 123.0}}))
    assert bench.pmc_traffic("fam", str(flat))[0] == 123.0
    assert bench.pmc_traffic("other", str(flat)) == (None, None)
    nested = tmp_path / "nested.json"
    nested.write_text(json.dumps({"hbm": {"fam": {"hbm_bytes": 7.0}}, "sq": {}, "last_step_hbm_bytes": 1.0}))
    assert bench.pmc_traffic("fam", str(nested))[0] == 7.0
    # another model reads its own summary, never ResNet-50's
    for m in ("resnext50", "resnet50_int8"):
        p = bench.pmc_json_path(m)
        assert p is None or p.endswith("pmc_hbm_bytes_per_launch_%s.json" % m), p
