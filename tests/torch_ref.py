"""Independent torch-CPU fp64 restatement used to pin the oracle (tests/test_oracle.py) and to
generate the golden fixtures (tests/golden/make_golden.py). Test infrastructure only."""
import numpy as np
import torch
import torch.nn.functional as F


def T(a, grad=False):
    # explicit dtype: never touch torch's global default (GPU tests share the session)
    return torch.tensor(np.asarray(a, dtype=np.float64), dtype=torch.float64, requires_grad=grad)


def torch_net_grads(g, args, data, label, want_loss=False):
    """Independent forward+autograd of an oracle Graph with torch fp64 functional ops."""
    P = {k: T(v, True) for k, v in args.items()}
    env = {"data": T(data)}
    for op in g.ops:
        t = op["op"]
        if t == "conv":
            env[op["y"]] = F.conv2d(env[op["x"]], P[op["name"] + "_weight"], stride=op["stride"], padding=op["pad"],
                                    groups=op["groups"])
        elif t == "bn":
            gam = torch.ones_like(P[op["name"] + "_gamma"]) if op["fix_gamma"] else P[op["name"] + "_gamma"]
            if op["fix_gamma"]:
                gam = gam + 0 * P[op["name"] + "_gamma"]
            env[op["y"]] = F.batch_norm(env[op["x"]], None, None, gam, P[op["name"] + "_beta"], training=True,
                                        eps=op["eps"])
        elif t == "relu":
            env[op["y"]] = F.relu(env[op["x"]])
        elif t == "maxpool":
            env[op["y"]] = F.max_pool2d(env[op["x"]], op["kernel"], op["stride"], op["pad"])
        elif t == "gap":
            env[op["y"]] = env[op["x"]].mean(dim=(2, 3), keepdim=True)
        elif t == "fc":
            env[op["y"]] = F.linear(env[op["x"]].flatten(1), P[op["name"] + "_weight"], P[op["name"] + "_bias"])
        elif t == "add":
            env[op["y"]] = env[op["a"]] + env[op["b"]]
        elif t == "softmax":
            loss = F.cross_entropy(env[op["x"]], torch.tensor(label.astype(np.int64)), reduction="sum")
            prob = F.softmax(env[op["x"]], dim=1)
    loss.backward()
    grads = {k: v.grad.numpy() for k, v in P.items()}
    if want_loss:
        return grads, float(loss.item()), prob.detach().numpy()
    return grads
