"""Print per-kernel register / LDS usage from a hipcc -Rpass-analysis=kernel-resource-usage log.
python tools/diag/regs.py LOG [substring...]"""
import re
import sys

txt = open(sys.argv[1]).read()
pats = sys.argv[2:]
for b in re.split(r'remark: [^\n]*?Function Name: ', txt)[1:]:
    name = b.split()[0]
    if pats and not all(p in name for p in pats):
        continue
    g = lambda k: (re.search(k + r': (\d+)', b) or [None, '?'])[1]
    print("%-100s v %3s a %3s spill %3s sgpr %3s lds %6s occ %s" % (
        name[:100], g('VGPRs'), g('AGPRs'), g('VGPRs Spill'), g('SGPRs'), g(r'LDS Size \[bytes/block\]'),
        g(r'Occupancy \[waves/SIMD\]')))
