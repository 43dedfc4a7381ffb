"""Headline benchmark: ResNet-50 v2 training throughput on MI355X (BASELINE.json configs[1..2]).

`python bench.py --gpus N --steps K --warmup W`: for N > 1 bench.py starts one rank process per
GPU itself (or runs as one rank of `python -m torch.distributed.run --nproc-per-node N`), RCCL
all-reduce between them. One step = forward(is_train) + backward + bucketed all-reduce + SGD
update over one synthetic 224x224 batch of 256 images per GPU (data/imagenet.py:9-41 restated:
seeded U(-1,1) data, random labels), bf16 activations/weights with fp32 master weights,
gradients and BN statistics. Inputs are resident in HBM before the timed region.

Rank 0 prints ONE JSON line (contract in the task statement), including
  roofline     : the dominant kernel family (most kernel time per step in a serialised calibration
                 step; every family's time is listed) -- algorithmic FLOP and bytes per launch /
                 average launch duration from HIP events around every launch of that family on the
                 stream it runs on (eager mode: the last of the K timed steps -- the event packets cost
                 ~1.7 % of a step, so the other K - 1 run without them; HIP-graph mode: in one eager
                 step right after it, graph nodes carry no timing events); "bound" from the family's
                 algorithmic FLOP/byte vs the 312.5 FLOP/B ridge (2.5 PF bf16 / 8 TB/s), both the MFMA
                 and the HBM fraction reported
  critical_path: the same record for the compute stream's largest family (the data-gradient chain that
                 sets the step while the weight gradients run overlapped on the side stream)
  weight_gradients: the same record for the weight-gradient family (side stream)
  pcie_inclusive: the same step fed the iterator's pinned host batch every step (not `value`)
  cpu_baseline : torch-CPU fp32 (oneDNN) restatement of the same step (oracle/torch_cpu.py,
                 "port") on every host core, batch 32 (rank 0, N=1 only)
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "resnet.mxnet_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)
import rn  # noqa: E402,F401  (before any HIP call: rn sets the process's hardware-queue count, rn/__init__.py)

METRIC = "images/sec/GPU ResNet-50 224px bf16 bs256; 1→8 GPU scaling"
# the other BASELINE configs (C4, C5) are reported under their own names, never as the headline metric
MODEL_METRIC = {"resnet50": METRIC,
                "resnext50": "images/sec/GPU ResNeXt-50 32x4d 224px bf16 bs256 (BASELINE C4)",
                "resnet50_int8": "images/sec/GPU ResNet-50 int8 QAT 224px (int8 fwd, bf16 bwd) bs256 (BASELINE C5)"}
PEAK_BF16_TFLOPS = 2500.0
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: 8 TB/s spec (6.3 TB/s achievable)
RIDGE = PEAK_BF16_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)  # 312.5 FLOP/B: below it a kernel is HBM-bound


def conv_call_flops(name, args):
    """Algorithmic FLOP (2/MAC) of one rn_conv_* call from its descriptor."""
    d = args[0]._obj
    cin = d.c_real
    macs_fwd = d.n * d.p * d.q * d.k * cin * d.r * d.s
    return 2 * macs_fwd


def conv_call_bytes(ex, name, args):
    """Algorithmic HBM bytes of one conv call: every operand read once, every output written once."""
    d = args[0]._obj
    es = 2 if ex.dtype == 0 else 4
    x = d.n * d.h * d.w * d.c * es
    y = d.n * d.p * d.q * d.k_pad * es
    w = d.k * d.r * d.s * d.c_real * es
    if name in ("rn_conv_fwd", "rn_conv_fwd_bnstats", "rn_conv_fwd_x"):
        yb = d.n * d.p * d.q * d.k_pad * (4 if args[4] == 1 else es)
        return x + w + yb + (y if args[5] is not None else 0)
    if name in ("rn_conv_bwd_data", "rn_conv_bwd_data_bnred"):
        bnx = x if name == "rn_conv_bwd_data_bnred" else 0  # the fused BN-backward reduction reads the BN input
        return y + w + x + (x if args[4] is not None else 0) + bnx
    return x + y + 2 * d.k * d.r * d.s * d.c_real * 4  # wgrad: fp32 dW read-modify-write (slabs not counted)


PMC_ROUNDS = ("r06", "r05", "r04", "r03")  # newest first: the committed PMC summary of the latest round that has one


def pmc_json_path(model="resnet50"):
    """The committed PMC summary of this model's bench (profiles/<round>/pmc_hbm_bytes_per_launch_<model>.json;
    the unsuffixed file is ResNet-50's): another model's per-launch bytes are not this one's."""
    env = os.environ.get("RN_PMC_JSON")
    if env:
        return env
    for r in PMC_ROUNDS:
        names = ["pmc_hbm_bytes_per_launch_%s.json" % model] + (["pmc_hbm_bytes_per_launch.json"]
                                                                if model == "resnet50" else [])
        for nm in names:
            p = os.path.join(REPO, "profiles", r, nm)
            if os.path.exists(p):
                return p
    return None


def pmc_traffic(family, path=None, model="resnet50"):
    """HBM bytes per launch of `family` from the committed rocprofv3 PMC summary (tools/pmc_bench.sh +
    tools/pmc_summary.py: FETCH_SIZE doubled per the gfx950 correction, plus WRITE_SIZE). The summary
    nests the families under "hbm" (with "sq" and "last_step_hbm_bytes" beside it); a flat
    {family: record} file (round 2) is read too."""
    path = path or pmc_json_path(model)
    if not path:
        return None, None
    try:
        with open(path) as f:
            doc = json.load(f)
    except OSError:
        return None, None
    fams = doc.get("hbm") if isinstance(doc.get("hbm"), dict) else doc
    rec = fams.get(family)
    if not rec or "hbm_bytes" not in rec:
        return None, None
    return rec["hbm_bytes"], os.path.relpath(path, REPO)


FWD_CALLS = ("rn_conv_fwd", "rn_conv_fwd_bnstats", "rn_conv_fwd_x")
DGRAD_CALLS = ("rn_conv_bwd_data", "rn_conv_bwd_data_bnred")


def family_of(ex, name, args):
    if name in ("rn_conv_bwd_filter", "rn_conv_bwd_filter_ws", "rn_conv_bwd_filter_x"):  # slab reduction included
        return "wgrad_kernel<bf16,*>" if ex.dtype == 0 else "wgrad_kernel<f32,*>"
    if name in FWD_CALLS + DGRAD_CALLS:
        d = args[0]._obj
        dgrad = name in DGRAD_CALLS
        ncol = d.c if dgrad else d.k
        out_f32 = not dgrad and args[4] == 1 and ex.dtype == 0
        plain = dgrad or args[6] is None
        # the library's own choice (rn_conv_tile), so the family always matches the kernel that runs
        big = ex.lib.rn_conv_tile(args[0], 1 if dgrad else 0) if (ex.dtype == 0 and not out_f32 and plain) else 0
        if name == "rn_conv_fwd_x" and args[7] is not None and big < 128:
            big = 0  # the BN+ReLU input transform runs on the 224-row tiles only, else the 128-row kernel
        if big:  # tile rows: 256, or 224 (one BN partial block per 128/256-column tile)
            rows = ex.lib.rn_conv_bn_part_rows(args[0], 1 if dgrad else 0) if big >= 128 else 256
            return "igemm_big_kernel<%dx%d>" % (rows, big)
        tile = "128x64" if ncol <= 64 else "128x128"
        return "igemm_kernel<bf16,%s,%s>" % ("f32" if out_f32 else "bf16", tile)
    return None


class FamilyTimer:
    """HIP events around every launch of one kernel family on the executor's stream."""

    def __init__(self, torch, ex, family):
        self.torch, self.ex, self.family = torch, ex, family
        self.idx = []
        self.flops = 0
        self.bytes = 0
        for lst_name in ("_fwd_train", "_bwd"):
            lst = getattr(ex, lst_name)
            for i, (name, fn, args) in enumerate(lst):
                if family_of(ex, name, args) == family:
                    self.idx.append((lst_name, i))
                    self.flops += conv_call_flops(name, args)
                    self.bytes += conv_call_bytes(ex, name, args)
        self.events = []

    def wrap(self):
        torch = self.torch
        self._saved = {}
        for lst_name, i in self.idx:
            lst = getattr(self.ex, lst_name)
            name, fn, args = lst[i]
            self._saved[(lst_name, i)] = lst[i]

            # (weight gradients run on the executor's side stream: time them there)
            on_side = bool(args) and args[-1] is getattr(self.ex, "_spv2", None)

            def timed(*a, _fn=fn, _side=on_side):
                st = self.ex._side_stream if (_side and self.ex.side_enabled) else self.ex.stream
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record(st)
                r = _fn(*a)
                e.record(st)
                self.events.append((s, e))
                return r

            lst[i] = (name, timed, args)

    def unwrap(self):
        for (lst_name, i), v in self._saved.items():
            getattr(self.ex, lst_name)[i] = v

    def result(self):
        ms = [s.elapsed_time(e) for s, e in self.events]
        return sum(ms), len(ms)


def calibrate_families(torch, ex, mod):
    """Time every MFMA-kernel launch of one step; return {family: (ms, launches, flops)}."""
    fams = {}
    for lst_name in ("_fwd_train", "_bwd"):
        for name, fn, args in getattr(ex, lst_name):
            f = family_of(ex, name, args)
            if f and f not in fams:
                fams[f] = FamilyTimer(torch, ex, f)
    for t in fams.values():
        t.wrap()
    # one serialised step (the weight gradients on the compute stream too, with the whole chip's split-M
    # grids as RN_WGRAD_STREAM=0 runs them): each family's solo launch durations, which choose the dominant
    # family and give its solo roofline fraction
    ex.side_enabled = False
    mod.forward(None, is_train=True)
    mod.backward()
    mod.update()
    torch.cuda.synchronize()
    ex.side_enabled = True
    out = {}
    for f, t in fams.items():
        ms, n = t.result()
        out[f] = (ms, n, t.flops)
        t.unwrap()
    return out


def family_roofline(family, timer, calib, model="resnet50"):
    """Roofline record of one kernel family: algorithmic FLOP and bytes per launch over the average launch
    duration from the HIP events of the timed region (`avg_launch_ms`, sharing the CUs with whatever runs
    beside it) and from the serialised calibration step (`solo_*`: the kernel alone)."""
    launches = max(1, len(timer.idx))
    fam_ms, fam_n = timer.result()
    avg_ms = fam_ms / max(fam_n, 1)
    solo_ms = calib[0] / max(calib[1], 1)
    flops = timer.flops / launches
    alg_bytes = timer.bytes / launches
    traffic, traffic_src = pmc_traffic(family, model=model)
    intensity = flops / max(alg_bytes, 1.0)  # algorithmic FLOP per byte vs the ridge: which roofline binds
    bound = "mfma" if intensity >= RIDGE else "hbm"
    tflops = flops / (avg_ms * 1e-3) / 1e12
    gbs = alg_bytes / (avg_ms * 1e-3) / 1e9
    achieved, peak, unit = (tflops, PEAK_BF16_TFLOPS, "TFLOP/s") if bound == "mfma" else (gbs, PEAK_HBM_GBS, "GB/s")
    solo_tf = flops / (solo_ms * 1e-3) / 1e12
    solo_gbs = alg_bytes / (solo_ms * 1e-3) / 1e9
    return {"bound": bound, "kernel": family, "launches_per_step": len(timer.idx),
            "achieved": round(achieved, 2), "peak": peak, "unit": unit, "frac": round(achieved / peak, 4),
            "traffic": round(traffic) if traffic else None, "traffic_unit": "HBM bytes/launch",
            "traffic_source": traffic_src, "algorithmic_bytes": round(alg_bytes), "flops_per_launch": round(flops),
            "intensity_flop_per_byte": round(intensity, 1), "ridge_flop_per_byte": round(RIDGE, 1),
            # both rooflines of the family, whichever binds
            "mfma_achieved_tflops": round(tflops, 2), "mfma_frac": round(tflops / PEAK_BF16_TFLOPS, 4),
            "hbm_achieved_gbs": round(gbs, 1), "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
            "avg_launch_ms": round(avg_ms, 4),
            # the same launches in the serialised calibration step (nothing sharing the CUs)
            "solo_avg_launch_ms": round(solo_ms, 4), "solo_mfma_frac": round(solo_tf / PEAK_BF16_TFLOPS, 4),
            "solo_hbm_frac": round(solo_gbs / PEAK_HBM_GBS, 4)}


def cpu_baseline(batch=32, steps=2, image=224):
    """SURVEY.md 8d / BASELINE.md 3: the reference's MXNet CPU executor cannot run here, so its
    closest analogue -- torch-CPU fp32 functional ops (oneDNN, MXNet's MKL-DNN counterpart) on every
    host core -- runs the identical ResNet-50 v2 graph and Solver step (oracle/torch_cpu.py) on a
    bounded sample: batch 32 at 224x224, 1 warm-up + `steps` timed steps."""
    from oracle import net as onet
    from oracle import torch_cpu
    ips, dt, cores, _ = torch_cpu.time_step(onet.resnet50_imagenet(), batch, image, 1000, steps)
    return {"value": round(ips, 3), "unit": "images/sec", "cores": cores, "kind": "port",
            "cpu_model": torch_cpu.cpu_model(),
            "sample": "torch-CPU fp32 (oneDNN) ResNet-50 v2 train step (fwd + bwd + MXNet SGD), batch %d at %dx%d, "
                      "%d timed steps after 1 warm-up (%.1f s), %d threads" % (batch, image, image, steps, dt, cores)}


def cpu_baseline_c1(batch=128, steps=20):
    """BASELINE.json configs[0]: ResNet-20 CIFAR-10 32x32, batch 128 -- the reference's own CPU case --
    as the same torch-CPU fp32 step on every host core (3 warm-up + `steps` timed)."""
    from oracle import net as onet
    from oracle import torch_cpu
    ips, dt, cores, _ = torch_cpu.time_step(onet.resnet20_cifar(), batch, 32, 10, steps, warmup=3)
    return {"value": round(ips, 3), "unit": "images/sec", "cores": cores, "kind": "port",
            "cpu_model": torch_cpu.cpu_model(),
            "sample": "torch-CPU fp32 ResNet-20 CIFAR-10 train step, batch %d at 32x32, %d timed steps (%.1f s)"
                      % (batch, steps, dt)}


def c1_module_cpu(batch=128, steps=10):
    """BASELINE.json configs[0] through the drop-in itself: train.py's Module on an mx.cpu() context
    (rn/cpu_executor.py, the product's host device), ResNet-20 CIFAR-10, batch 128, fixed synthetic
    batch, 2 warm-up + `steps` timed forward/backward/update iterations."""
    import numpy as np
    import torch
    import mxnet as mx
    from rn import graphs
    cores = torch.get_num_threads()
    mod = mx.mod.Module(graphs.resnet20_cifar(), context=mx.cpu())
    mod.bind(data_shapes=[("data", (batch, 3, 32, 32))], label_shapes=[("softmax_label", (batch,))])
    mx.random.seed(2)
    mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
    mod.init_optimizer(kvstore="local", optimizer="sgd",
                       optimizer_params={"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9})
    rng = np.random.default_rng(0)
    b = mx.io.DataBatch(data=[mx.nd.array(rng.uniform(-1, 1, (batch, 3, 32, 32)).astype(np.float32))],
                        label=[mx.nd.array(rng.integers(0, 10, batch).astype(np.float32))])

    def it():
        mod.forward(b, is_train=True)
        mod.backward()
        mod.update()
    for _ in range(2):
        it()
    t0 = time.perf_counter()
    for _ in range(steps):
        it()
    dt = time.perf_counter() - t0
    return {"value": round(batch * steps / dt, 3), "unit": "images/sec", "cores": cores,
            "sample": "mx.mod.Module(context=mx.cpu()) ResNet-20 CIFAR-10 train step, batch %d at 32x32, "
                      "%d timed steps (%.1f s)" % (batch, steps, dt)}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Interrupted(Exception):
    pass


def launch_ranks(n, argv, cmd=None):
    """`python bench.py --gpus N` without a torch.distributed launcher (how the driver runs it):
    start N fresh rank processes of this script -- one per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* set as torch.distributed.run would -- before this process touches the GPU, wait for
    them and return the exit status. The reference drives its GPUs from one `python train.py`
    (train.py:34-35, core/solver.py:58-61,121); here each GPU gets its own process and RCCL sums the
    gradients. A rank that fails takes the others down (they would block in a collective); so does
    a SIGTERM / SIGINT to this launcher (each rank runs in its own session, so a signal to the
    launcher alone would otherwise leave them holding their GPUs). `cmd`: the rank command (tests)."""
    import signal
    import subprocess
    import torch
    backend = os.environ.get("RN_DIST_BACKEND", "nccl")
    ngpu = torch.cuda.device_count()  # does not initialise the GPU on this image
    if backend == "nccl" and ngpu < n:
        print("bench.py: --gpus %d but %d GPU(s) visible (RN_DIST_BACKEND=gloo rehearses N ranks on "
              "fewer GPUs)" % (n, ngpu), file=sys.stderr)
        return 2
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + argv
    procs = []

    def stop_live():
        for pr in procs:
            if pr.poll() is None:
                try:
                    os.killpg(pr.pid, signal.SIGKILL)
                except OSError:
                    pass
        for pr in procs:
            try:
                pr.wait(timeout=30)
            except Exception:
                pass

    def on_signal(signum, frame):
        raise _Interrupted(signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    rc = 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RN_BENCH_LAUNCHED="1")
            procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
        live = list(range(n))
        while live:
            time.sleep(0.2)
            for r in list(live):
                c = procs[r].poll()
                if c is None:
                    continue
                live.remove(r)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    print("bench.py: rank %d exited with %d; stopping the other ranks" % (r, c), file=sys.stderr)
                    stop_live()
    except _Interrupted as e:
        print("bench.py: launcher got signal %d; stopping every rank" % e.args[0], file=sys.stderr)
        rc = 128 + e.args[0]
    finally:
        # a second TERM / INT during the cleanup must not abort it before every rank is killed and reaped
        for s in old:
            signal.signal(s, signal.SIG_IGN)
        stop_live()
        for s, h in old.items():
            signal.signal(s, h)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of this node (one rank each). Without a torch.distributed launcher bench.py "
                         "starts the ranks itself; under one it must equal WORLD_SIZE. Default: WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--precision", default="bfloat16")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "resnext50", "resnet50_int8"],
                    help="BASELINE.json configs: resnet50 = C2/C3 (the headline), resnext50 = C4 "
                         "(32x4d, grouped convs), resnet50_int8 = C5 (symbol/resnet_int8.py QAT graph)")
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=32)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--pcie-steps", type=int, default=None,
                    help="steps of the PCIe-inclusive leg (default: steps / 2; 0 skips it)")
    ap.add_argument("--host-input", action="store_true",
                    help="feed the pinned host batch through Module.forward every step (PCIe-inclusive "
                         "rate, the solver's own loop; not the headline value)")
    ap.add_argument("--graph", default="auto", choices=["auto", "0", "1"],
                    help="replay the captured step as one HIP graph (auto: on for a single GPU)")
    a = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (a.gpus or 1) > 1:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    if env_world is not None and a.gpus is not None and a.gpus != int(env_world):
        print("bench.py: --gpus %d disagrees with WORLD_SIZE=%s" % (a.gpus, env_world), file=sys.stderr)
        sys.exit(2)

    import numpy as np
    import torch
    from rn import dist as rdist
    from rn import graphs
    import mxnet as mx

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # (RN_DIST_BACKEND=gloo with more ranks than GPUs: a rehearsal of the N > 1 path on a one-GPU box)
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        rdist.init_from_env(os.environ.get("RN_DIST_BACKEND", "nccl"))
    import torch.distributed as dist
    # RN_BENCH_ALLREDUCE=1 at N=1: an RCCL process group of one rank and the bucketed all-reduce hooks
    # on anyway (a world-1 sum is the identity): the per-step cost of the data-parallel path itself
    force_ar = world == 1 and os.environ.get("RN_BENCH_ALLREDUCE", "0") == "1"
    if force_ar:
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%s" % os.environ.get("MASTER_PORT", "29511"),
                                rank=0, world_size=1, device_id=torch.device("cuda", local),
                                **rdist.nccl_pg_kwargs())

    sym = {"resnet50": graphs.resnet50, "resnext50": graphs.resnext50_32x4d,
           "resnet50_int8": graphs.resnet50_int8}[a.model]()
    model_name = {"resnet50": "resnet50_v2", "resnext50": "resnext50_32x4d", "resnet50_int8": "resnet50_v2_int8"}[a.model]
    workload = {"resnet50": "ResNet-50 v2 (symbol/resnet.py)", "resnext50": "ResNeXt-50 32x4d (symbol/resnext.py)",
                "resnet50_int8": "ResNet-50 v2 int8 QAT (symbol/resnet_int8.py)"}[a.model]
    mod = mx.mod.Module(sym, context=[mx.gpu(local % max(1, torch.cuda.device_count()))], precision=a.precision)
    shp = (a.batch, 3, a.image, a.image)
    mod.bind(data_shapes=[("data", shp)], label_shapes=[("softmax_label", (a.batch,))], for_training=True)
    mx.random.seed(2)
    mod.init_params(mx.init.Xavier(rnd_type="gaussian", factor_type="in", magnitude=2))
    mod.init_optimizer(kvstore="dist_sync_device" if world > 1 else "device", optimizer="sgd",
                       optimizer_params={"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9,
                                         "multi_precision": True})
    ex = mod.executor
    ex.bucket_bytes = int(a.bucket_mb * (1 << 20))
    if mod._reducer is not None or force_ar:
        from rn.dist import BucketAllReducer
        mod._reducer = BucketAllReducer(ex.grad, ex.buckets())
    data = np.random.default_rng(0 + rank).uniform(-1, 1, shp).astype(np.float32)
    label = np.random.default_rng(1 + rank).integers(0, 1000, (a.batch,)).astype(np.float32)
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    mod.forward(batch, is_train=True)  # H2D once: inputs resident from here on
    torch.cuda.synchronize()

    pinned = mx.io.DataBatch(data=[mx.nd.array(data, ctx=mx.Context("cpu_pinned", 0))],
                             label=[mx.nd.array(label, ctx=mx.Context("cpu_pinned", 0))])

    # (the data-gradient chain on a high-priority stream -- RN_MAIN_PRIORITY, rounds 3-5 -- measured slower since the
    # weight gradients' grids were sized for part of the chip, profiles/r04/priority: removed in round 6)
    def step(feed=pinned if a.host_input else None):
        mod.forward(feed, is_train=True)
        mod.backward()
        mod.update()

    for _ in range(max(a.warmup, 1)):
        step()
    torch.cuda.synchronize()
    fams = calibrate_families(torch, ex, mod)
    # roofline.kernel: the family with the most kernel time per step (serialised calibration step), as the
    # contract says -- with the side stream on that is the weight-gradient family. critical_path: the
    # compute (data-gradient) stream's largest family, which sets the step when the weight gradients
    # run overlapped beside it (rn_set_tuning 21 sizes them for part of the chip); both are timed with
    # HIP events on the stream each launch runs on, every family's time is listed
    side = bool(getattr(ex, "_side_idx", None)) and ex.side_enabled
    dom = max(fams, key=lambda f: fams[f][0])
    crit_fams = [f for f in fams if not (side and f.startswith("wgrad"))] or list(fams)
    crit = max(crit_fams, key=lambda f: fams[f][0])
    wg = next((f for f in fams if f.startswith("wgrad")), None)  # the weight-gradient family (side stream)
    timers = {dom: FamilyTimer(torch, ex, dom)}
    for f in (crit, wg):
        if f is not None and f not in timers:
            timers[f] = FamilyTimer(torch, ex, f)
    # auto: one HIP graph on a single GPU -- unless the executor runs its weight gradients on a side
    # stream: the graph replay serialises the two branches, eager launches overlap them (measured
    # 22.30 vs 22.93 ms per step for the graph with everything on one stream)
    use_graph = a.graph == "1" or (a.graph == "auto" and world == 1 and not a.host_input and
                                   getattr(ex, "_side_stream", None) is None)
    graph = None
    if use_graph:
        # the whole training step (forward, backward, SGD, weight repack) as ONE HIP graph:
        # removes the per-launch gaps between the ~580 kernels of a step; same kernels, same work
        graph = torch.cuda.CUDAGraph()
        # (a side stream joins the capture by the fork events)
        with torch.cuda.graph(graph):
            step()
        torch.cuda.synchronize()

        def replay():
            graph.replay()
        replay()  # one untimed replay
        torch.cuda.synchronize()
        run = replay
    else:
        run = step

    reducer = mod._reducer

    def instrument():
        # HIP events around every launch of the reported families (and, with RCCL, at the backward's ends and
        # each bucket: the overlap evidence) on the LAST timed step only: each event record is a packet of
        # its own between two kernels, and on every step they cost ~0.34 ms (1.7 %) of a ResNet-50 step
        # (profiles/r06/event_gaps: 19.26 ms eager without them, 19.60 with)
        for t in timers.values():
            t.wrap()
        if reducer is not None:
            reducer.timing = True
            reducer.records = []

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        if i == a.steps - 1 and not use_graph:
            instrument()
        run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    overlap = None
    if reducer is not None and reducer.timing:
        reducer.timing = False
        overlap = reducer.timing_summary(world)
        if overlap is not None and world > 1:
            t = torch.tensor([overlap["exposed_ms"], overlap["exposed_ms_max"]], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            overlap["exposed_ms_max_over_ranks"] = round(float(t[1].item()), 3)
            overlap["exposed_ms_mean_max_over_ranks"] = round(float(t[0].item()), 3)
    if use_graph:
        # graph nodes cannot carry timing events: time the family's launches in one eager step
        # run directly after the timed region (same kernels and shapes as the replayed graph)
        for t in timers.values():
            t.wrap()
        step()
        torch.cuda.synchronize()
    for t in timers.values():
        t.unwrap()
    if world > 1:
        t = torch.tensor([elapsed], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # PCIe-inclusive rate (never `value`): the solver's own loop feeds the iterator's pinned host
    # batch every step (core/solver.py:115, data/imagenet.py:17-18) -- copied H2D on the copy
    # stream, double-buffered, overlapping the previous step
    pcie = None
    psteps = a.steps // 2 if a.pcie_steps is None else a.pcie_steps
    if psteps > 0 and not a.host_input:
        for _ in range(2):
            step(pinned)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(psteps):
            step(pinned)
        torch.cuda.synchronize()
        pel = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([pel], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            pel = float(t.item())
        pcie = {"value": round(a.batch * world * psteps / pel, 2), "unit": "images/sec", "steps": psteps,
                "ms_per_step": round(pel / psteps * 1e3, 3),
                "inputs": "pinned host NCHW fp32 batch copied H2D every step (eager launches)"}
    prob = mod.get_outputs()[0].asnumpy()
    finite = bool(np.isfinite(prob).all())

    if rank == 0:
        imgs = a.batch * world * a.steps
        value = imgs / elapsed
        ms_step = elapsed / a.steps * 1e3
        flops_step = ex.plan.train_flops()
        roof = {f: family_roofline(f, t, fams[f], model=a.model) for f, t in timers.items()}
        out = {
            "metric": MODEL_METRIC[a.model], "value": round(value, 2), "unit": "images/sec", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            # the int8 graph multiplies int8 codes on int8 MFMAs forward; its backward (STE) runs in bf16
            "dtype": ("int8 fwd / bf16 bwd" if a.model == "resnet50_int8" else "bf16") if a.precision.startswith("bf")
            else "fp32",
            "data": "synthetic (seeded U(-1,1) %dx%d images, random labels; Xavier-init %s)" % (
                a.image, a.image, workload.split(" (")[0]),
            "config": {"workload": "%s train step, batch %d/GPU, %dx%d" % (
                workload, a.batch, a.image, a.image), "model": model_name, "global_batch": a.batch * world,
                "seq_len": None, "parallelism": "dp%d" % world, "per_gpu_images_per_sec": round(value / world, 2)},
            "roofline": dict(roof[dom], dominant_rule="most kernel time per step (serialised calibration step)",
                             concurrent_streams=2 if (ex._side_idx and ex.side_enabled) else 1,
                             step_tflops=round(flops_step / (ms_step * 1e-3) / 1e12, 2),
                             step_frac=round(flops_step / (ms_step * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                             families_ms_per_step={f: round(v[0], 3) for f, v in fams.items()}),
            # the compute stream's largest family: the step's critical path while the weight gradients
            # run overlapped on the side stream (the same record as roofline's; equal to it with one stream)
            "critical_path": dict(roof[crit], rule="most kernel time per step among the compute stream's "
                                                   "families" if side else "one stream: the dominant family"),
            # the weight gradients (the side stream's family: in-step with part of the chip's grids beside the
            # data-gradient chain, solo = the serialised calibration step on the whole chip)
            "weight_gradients": roof.get(wg),
            "outputs_finite": finite,
            "hip_graph": bool(use_graph),
            "family_timing": ("one eager step right after the timed region" if use_graph else
                              "HIP events on the last of the %d timed steps" % a.steps),
            "inputs":"pinned host batch copied every step (PCIe-inclusive)" if a.host_input else
                      "resident in HBM",
            "pcie_inclusive": pcie,
        }
        if force_ar or world > 1:
            nbytes = int(ex.grad.numel()) * ex.grad.element_size()
            out["allreduce"] = {"backend": dist.get_backend(), "world": world, "buckets": len(ex.buckets()),
                                "bucket_mb": a.bucket_mb, "grad_mb_per_step": round(nbytes / 2 ** 20, 2),
                                "launch": "one process per GPU (%s)" % (
                                    "bench.py --gpus" if os.environ.get("RN_BENCH_LAUNCHED") else "torch.distributed.run"),
                                "overlap": "buckets launched from the backward plan on the weight-gradient stream"}
            if overlap is not None:
                # exposed_ms: end of the backward -> last bucket summed (what the backward did not hide)
                out["allreduce"].update(overlap)
            if force_ar:
                out["allreduce"]["note"] = "RCCL bucket all-reduce hooks on at N=1 (RN_BENCH_ALLREDUCE=1)"
        if world == 1 and not a.no_cpu_baseline and a.model == "resnet50":
            try:
                out["cpu_baseline"] = cpu_baseline(a.cpu_batch, a.cpu_steps)
                out["cpu_baseline_c1"] = cpu_baseline_c1()
                out["c1_mx_cpu_module"] = c1_module_cpu()
            except Exception as e:  # baseline must not hide the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out), flush=True)
    if world > 1 or force_ar:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
