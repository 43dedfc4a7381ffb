"""CPU oracle for the ResNet/ResNeXt data-parallel training path -- TEST INFRASTRUCTURE ONLY.

This package is a plain-numpy restatement (fp64 by default) of what the reference
XiaotaoChen/resnet.mxnet computes on its hot path: the graphs of symbol/resnet.py,
symbol/resnext.py and symbol/resnet_int8.py executed by MXNet's Module (core/solver.py) with
the optimizer/scheduler of train.py and core/scheduler.py.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it, and only
as the checker (or as the timed CPU baseline). The product path (resnet.mxnet_amd) never
imports it and fails loudly if its HIP library is missing.

PARITY STATUS: **parity unpinned** against MXNet itself. The arithmetic of this path lives in
the un-vendored MXNet fork huangzehao/incubator-mxnet-bk (version not pinned by the
reference; >= 1.3-era features used at train.py:164-166). It is absent from this container
(`import mxnet` -> ModuleNotFoundError; no network), and the reference ships no tests, golden
vectors or fixtures for this path. Every MXNet-internal semantic
restated here is taken from the public MXNet 1.x code base and listed in oracle/ops.py, and
the restatement is cross-checked against an independent torch-CPU fp64 implementation in
tests/test_oracle.py. The committed fixtures under tests/golden/ pin THIS oracle from now on
(made by tests/golden/make_golden.py).
"""
