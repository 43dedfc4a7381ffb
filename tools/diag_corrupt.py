"""Diagnostic: run one ResNeXt fp32 training step call by call and report the first call after
which the executor's SGD tables (bound before the step) differ from their bind-time contents,
i.e. a kernel writing outside its buffers. Launches no SGD."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "resnet.mxnet_amd"), os.path.join(REPO, "tests")]


def main():
    import torch
    import mxnet as mx
    from oracle import net as onet
    from rn import graphs
    from test_step_gpu import _resnext_small, oracle_state
    cfg = _resnext_small()
    g = onet.resnext(*cfg, num_group=32)
    args, aux = oracle_state(g)
    data, label = onet.synthetic_batch(4, (3, 64, 64), 16)
    sym = graphs.resnext(*cfg, "float32", 32)
    mod = mx.mod.Module(sym, context=[mx.gpu(0)], precision="float32")
    mod.bind(data_shapes=[("data", data.shape)], label_shapes=[("softmax_label", label.shape)], for_training=True)
    mod.init_params(arg_params={k: v.astype(np.float32) for k, v in args.items()},
                    aux_params={k: v.astype(np.float32) for k, v in aux.items()}, allow_missing=True)
    mod.init_optimizer(kvstore="device", optimizer="sgd",
                       optimizer_params={"learning_rate": 0.1, "wd": 1e-4, "momentum": 0.9})
    ex = mod._exec
    torch.cuda.synchronize()
    watch = {"opt_work": ex.opt_work, "opt_packs": ex.opt_packs, "opt_offsets": ex.opt_offsets,
             "opt_numels": ex.opt_numels}
    ref = {k: v.clone() for k, v in watch.items()}
    print("watch:", {k: (hex(v.data_ptr()), v.numel() * v.element_size()) for k, v in watch.items()}, flush=True)
    batch = mx.io.DataBatch(data=[mx.nd.array(data)], label=[mx.nd.array(label)])
    # forward input staging
    ex_calls = []
    orig_run = type(ex)._run

    def changed():
        torch.cuda.synchronize()
        return [k for k in watch if not torch.equal(watch[k], ref[k])]

    def run(self, calls):
        for name, fn, a in calls:
            r = fn(*a)
            if r != 0:
                raise RuntimeError(name)
            c = changed()
            if c:
                print("CORRUPTED after", name, c, flush=True)
                for k in c:
                    d = (watch[k] != ref[k]).nonzero().flatten()[:8].tolist()
                    print("   ", k, "first differing elements", d, flush=True)
                raise SystemExit(3)
    type(ex)._run = run
    mod.forward(batch, is_train=True)
    print("forward clean:", changed(), flush=True)
    # backward without hooks goes through _run(self._bwd)
    mod.backward()
    print("backward clean:", changed(), flush=True)


if __name__ == "__main__":
    main()
