"""mx.viz.print_summary (train.py:126, commented out there): per-layer output shapes."""


def print_summary(symbol, shape=None, line_length=120, positions=(.44, .64, .74, 1.)):
    internals = symbol.get_internals()
    _, out_shapes, _ = internals.infer_shape_partial(**(shape or {}))
    for name, shp in zip(internals.list_outputs(), out_shapes or []):
        print("%-60s %s" % (name, shp))


def plot_network(*args, **kwargs):
    raise NotImplementedError("graphviz plotting is not available")
