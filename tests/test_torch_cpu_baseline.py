"""The CPU baseline (oracle/torch_cpu.py: torch-CPU fp32 restatement of the Solver step, timed by
bench.py) computes what the numpy oracle computes: one ResNet-20 step at batch 4 -- loss, updated
parameters (MXNet SGD) and BN moving statistics -- within fp32 tolerance of the fp64 oracle."""
import numpy as np

from oracle import net as onet
from oracle import torch_cpu


def test_torch_cpu_step_matches_oracle():
    g = onet.resnet20_cifar()
    args, aux = onet.init_params(g)
    data, label = onet.synthetic_batch(4, (3, 32, 32), 10)
    st = torch_cpu.TorchStep(g, args, aux, channels_last=False)
    loss = st.step(data.astype(np.float32), label, 0.1)
    a64 = {k: v.copy() for k, v in args.items()}
    moms = {k: np.zeros_like(v) for k, v in a64.items()}
    prob, _, auxes = onet.train_step(g, a64, {k: v.copy() for k, v in aux.items()}, moms, data, label, 0.1)
    ref_loss = float(-np.log(prob[np.arange(4), label.astype(int)]).mean())
    assert abs(loss - ref_loss) < 1e-5 * max(1.0, ref_loss)
    for k, v in a64.items():
        d = st.P[k].detach().numpy().astype(np.float64)
        step = np.abs(v - args[k]).max()
        assert np.abs(d - v).max() <= 1e-3 * step + 1e-6 * np.abs(v).max() + 1e-12, k
    for k, v in auxes[0].items():
        assert np.allclose(st.aux[k].numpy(), v, rtol=1e-4, atol=1e-6), k
