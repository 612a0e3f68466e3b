#!/usr/bin/env python3
"""Instruction histogram of one kernel (or one loop of it) in a hipcc -S listing.
Usage: python tools/isa_hist.py FILE.s KERNEL_SUBSTR [--loop]"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split('\n')
st = [i for i, l in enumerate(L) if re.match(r'^_Z\S*:', l) and sys.argv[2] in l][0]
en = next(i for i in range(st, len(L)) if 's_endpgm' in L[i])
body = L[st:en]
blocks = {}
cur = 'entry'
for l in body:
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        cur = m.group(1)
        blocks[cur] = []
        continue
    if l.startswith('\t') and not l.strip().startswith(('.', ';')):
        blocks.setdefault(cur, []).append(l.split()[0])
for b, ins in blocks.items():
    print(b, len(ins))
biggest = max(blocks, key=lambda b: len(blocks[b]))
c = collections.Counter(blocks[biggest])
print('largest block', biggest, len(blocks[biggest]))
for k, v in c.most_common(50):
    print(f'{v:6d} {k}')
