"""Side-by-side per-layer times from several tools/conv_bench.py logs (fwd,dgrad)."""
import re
import sys


def parse(f):
    out = {}
    for l in open(f):
        m = re.match(r'(\S+)\s+(\d+)\s+(\S+ k\d s\d)\s*(\+res|g\d+)?\s+(.*)$', l)
        if m:
            t = [float(x) for x in re.findall(r'([\d.]+)us', m.group(5))]
            out[m.group(1)] = (m.group(3), int(m.group(2)), t)
    return out


logs = [parse(f) for f in sys.argv[1:]]
base = logs[0]
print("%-22s %-20s %3s " % ("layer", "shape", "n") + " | ".join("%-17s" % f.split('/')[-1][:17] for f in sys.argv[1:]))
tot = [[0.0] * 3 for _ in logs]
for k, (shape, n, _) in base.items():
    row = "%-22s %-20s %3d " % (k[:22], shape, n)
    cells = []
    for i, lg in enumerate(logs):
        t = lg.get(k, (None, 0, []))[2]
        for j, v in enumerate(t):
            tot[i][j] += v * n
        cells.append(" ".join("%8.1f" % v for v in t))
    print(row + " | ".join(cells))
print("totals (ms): " + " | ".join(" ".join("%.3f" % (v / 1e3) for v in t if v) for t in tot))
