"""Instruction mix of each backward-branch loop of a kernel in a hipcc -S listing.
python tools/diag/loops.py FILE.s SYMBOL_SUBSTRING"""
import re
import sys

s = open(sys.argv[1]).read()
for m in re.finditer(r'^(\S+):\s*; @', s, re.M):
    nm = m.group(1)
    if sys.argv[2] not in nm:
        continue
    j = s.index('.Lfunc_end', m.start())
    lines = s[m.start():j].split('\n')
    labels = {}
    for k, l in enumerate(lines):
        mm = re.match(r'^(\.LBB\d+_\d+):', l)
        if mm:
            labels[mm.group(1)] = k
    print(nm, 'lines', len(lines))
    for k, l in enumerate(lines):
        mm = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < k:
            a = labels[mm.group(1)]
            seg = [x for x in lines[a:k + 1] if x.strip() and not x.strip().startswith(';')]
            cnt = lambda p: sum(1 for x in seg if re.search(p, x))
            print('  loop %6d-%6d instr %5d mfma %4d accr %4d accw %4d ds_read %4d ds_write %3d dma %3d waitcnt %3d '
                  'barrier %2d scratch %3d valu %4d salu %4d' % (
                      a, k, len(seg), cnt(r'v_mfma'), cnt('v_accvgpr_read'), cnt('v_accvgpr_write'), cnt('ds_read'),
                      cnt('ds_write'), cnt(r' lds\b'), cnt('s_waitcnt'), cnt('s_barrier'), cnt('scratch_'),
                      cnt(r'^\s*v_(?!mfma|accvgpr)'), cnt(r'^\s*s_')))
