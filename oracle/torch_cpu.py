"""torch-CPU fp32 restatement of one Solver training step -- the CPU BASELINE of bench.py.

TEST / BASELINE INFRASTRUCTURE ONLY (see oracle/__init__.py): bench.py's cpu_baseline leg times it
beside the GPU number; nothing on the product path imports it.

SURVEY.md 8d / BASELINE.md 3: the reference's MXNet CPU executor cannot run here (MXNet is absent
and cannot be fetched), so the baseline is the closest analogue of MXNet's MKL-DNN CPU path:
oneDNN-backed torch functional ops in fp32 on every host core, running the identical graph
(an oracle.net Graph, restated from symbol/resnet.py / resnext.py) and the identical step of
core/solver.py:115-121 -- forward(is_train) with batch-statistics BatchNorm and moving-stat update,
SoftmaxOutput backward p - onehot (normalization 'null'), MXNet momentum SGD with rescale_grad =
1/batch and wd_mult 0 on biases / betas (train.py:186-194, oracle/ops.py).
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import ops


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class TorchStep:
    """Parameters, momenta and BN moving statistics of one graph, stepped in fp32 on the CPU."""

    def __init__(self, graph, args, aux, channels_last=True, storage=None):
        self.g = graph
        self.cl = channels_last
        # storage='bf16': conv / BN / pooling outputs and conv weights rounded to bf16 as they are
        # stored (the bf16-storage emulation of oracle.net.forward), fp32 arithmetic in between
        self.rnd = (lambda t: t.to(torch.bfloat16).to(torch.float32)) if storage == "bf16" else (lambda t: t)
        fmt = torch.channels_last if channels_last else torch.contiguous_format

        def mk(v):
            t = torch.tensor(np.asarray(v, dtype=np.float32))
            if t.dim() == 4:
                t = t.contiguous(memory_format=fmt)
            return t.requires_grad_(True)
        self.P = {k: mk(v) for k, v in args.items()}
        self.aux = {k: torch.tensor(np.asarray(v, dtype=np.float32)) for k, v in aux.items()}
        self.mom = {k: torch.zeros_like(v) for k, v in self.P.items()}
        self.wd_mult = {k: ops.wd_mult_for(k) for k in self.P}

    def grads(self, data, label):
        """Forward(is_train) + backward only: ({param: fp64 gradient of the summed CE}, probabilities)."""
        self._forward_backward(data, label)
        out = {k: (p.grad.double().numpy() if p.grad is not None else np.zeros(p.shape))
               for k, p in self.P.items()}
        for p in self.P.values():
            p.grad = None
        return out, self._prob

    def step(self, data, label, lr, momentum=0.9, wd=1e-4):
        loss = self._forward_backward(data, label)
        rescale = 1.0 / data.shape[0]
        with torch.no_grad():
            for k, p in self.P.items():
                m = self.mom[k]
                gk = p.grad if p.grad is not None else torch.zeros_like(p)  # fix_gamma: dgamma = 0
                m.mul_(momentum).sub_(lr * (rescale * gk + wd * self.wd_mult[k] * p))
                p.add_(m)
                p.grad = None
        return loss

    def _forward_backward(self, data, label):
        g = self.g
        x = torch.from_numpy(np.ascontiguousarray(data, dtype=np.float32))
        if self.cl:
            x = x.contiguous(memory_format=torch.channels_last)
        env = {"data": x}
        loss = None
        for op in g.ops:
            t = op["op"]
            if t == "conv":
                env[op["y"]] = self.rnd(F.conv2d(env[op["x"]], self.rnd(self.P[op["name"] + "_weight"]),
                                                 stride=op["stride"], padding=op["pad"], groups=op["groups"]))
            elif t == "bn":
                nm = op["name"]
                xin = env[op["x"]]
                gam = self.P[nm + "_gamma"]
                if op["fix_gamma"]:
                    gam = torch.ones_like(gam)
                env[op["y"]] = self.rnd(F.batch_norm(xin, None, None, gam, self.P[nm + "_beta"], training=True,
                                                     eps=op["eps"]))
                with torch.no_grad():  # MXNet moving stats: biased batch variance, m = 0.9 m + 0.1 batch
                    var, mean = torch.var_mean(xin, dim=(0, 2, 3), unbiased=False)
                    mm, mv = self.aux[nm + "_moving_mean"], self.aux[nm + "_moving_var"]
                    mm.mul_(op["momentum"]).add_(mean, alpha=1 - op["momentum"])
                    mv.mul_(op["momentum"]).add_(var, alpha=1 - op["momentum"])
            elif t == "relu":
                env[op["y"]] = F.relu(env[op["x"]])
            elif t == "maxpool":
                env[op["y"]] = F.max_pool2d(env[op["x"]], op["kernel"], op["stride"], op["pad"])
            elif t == "gap":
                env[op["y"]] = self.rnd(env[op["x"]].mean(dim=(2, 3), keepdim=True))
            elif t == "fc":
                env[op["y"]] = F.linear(env[op["x"]].flatten(1), self.P[op["name"] + "_weight"],
                                        self.P[op["name"] + "_bias"])
            elif t == "add":
                env[op["y"]] = self.rnd(env[op["a"]] + env[op["b"]])
            elif t == "softmax":
                # SoftmaxOutput: d logits = p - onehot per sample (sum of CE, no 1/B)
                loss = F.cross_entropy(env[op["x"]], torch.from_numpy(label.astype(np.int64)), reduction="sum")
                self._prob = F.softmax(env[op["x"]].detach(), dim=1).double().numpy()
        loss.backward()
        return float(loss.item()) / data.shape[0]


def time_step(graph, batch, image, ncls, steps, warmup=1, threads=None):
    """Seeded synthetic batch (data/imagenet.py:15-18 restated), Xavier parameters; returns
    (images/sec, seconds, threads, losses)."""
    import os
    import time
    from . import net
    nthreads = threads or int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    torch.set_num_threads(nthreads)
    args, aux = net.init_params(graph, dtype=np.float32)
    data, label = net.synthetic_batch(batch, (3, image, image), ncls, dtype=np.float32)
    st = TorchStep(graph, args, aux)
    losses = [st.step(data, label, 0.1) for _ in range(warmup)]
    t0 = time.perf_counter()
    for _ in range(steps):
        losses.append(st.step(data, label, 0.1))
    dt = time.perf_counter() - t0
    return batch * steps / dt, dt, nthreads, losses
