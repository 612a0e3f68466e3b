#!/usr/bin/env python3
"""Per-basic-block instruction counts of one kernel in a hipcc -S listing (the whole function, up to
the next symbol: kernels with early returns have several s_endpgm).
Usage: python tools/isa_blocks.py FILE.s KERNEL_SUBSTR [min_instructions]"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split('\n')
st = [i for i, l in enumerate(L) if re.match(r'^_Z\S*:', l) and sys.argv[2] in l][0]
en = next((i for i in range(st + 1, len(L)) if re.match(r'^_Z\S*:', L[i]) or L[i].startswith('\t.size')), len(L))
blocks, order, cur = {}, ['entry'], 'entry'
for l in L[st:en]:
    m = re.match(r'^(\.LBB\S+):', l)
    if m:
        cur = m.group(1)
        order.append(cur)
        continue
    if l.startswith('\t') and not l.strip().startswith(('.', ';')):
        blocks.setdefault(cur, []).append(l.split()[0])
lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
tot = collections.Counter()
for b in order:
    ins = blocks.get(b, [])
    c = collections.Counter(ins)
    tot.update(c)
    if len(ins) >= lo:
        v = sum(n for k, n in c.items() if k.startswith('v_'))
        print(f"{b:12s} {len(ins):5d} valu {v:5d}  " + " ".join(f"{k}:{n}" for k, n in c.most_common(6)))
print("total", sum(tot.values()), "valu", sum(n for k, n in tot.items() if k.startswith('v_')))
