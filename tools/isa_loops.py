#!/usr/bin/env python3
"""Per-basic-block instruction histogram of one kernel in a hipcc -save-temps .s file (tool, not product)."""
import collections, re, sys
path, name = sys.argv[1], sys.argv[2]
s = open(path).read()
i = s.index(name + ':'); j = s.index('.Lfunc_end', i)
body = s[i:j].split('\n')
blocks, cur, lab = [], [], 'entry'
for l in body:
    if re.match(r'^\.LBB\d+_\d+:', l):
        blocks.append((lab, cur)); lab, cur = l.split(':')[0], []
    elif l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'):
        cur.append(l.split()[0])
blocks.append((lab, cur))
for lab, ins in blocks:
    c = collections.Counter(ins)
    if len(ins) < int(sys.argv[3]) if len(sys.argv) > 3 else 20: continue
    print(f'== {lab}: {len(ins)} instr: ' + ', '.join(f'{k}={v}' for k, v in c.most_common(12)))
