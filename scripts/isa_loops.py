#!/usr/bin/env python3
"""Per-loop instruction mix of one kernel in a hipcc -S listing (measurement helper).

  python scripts/isa_loops.py fused.s <mangled-kernel-substring>

Finds every backward branch (s_cbranch_* / s_branch to an earlier label) inside the
kernel's body and prints the instruction classes of the loop body it closes."""
import collections
import re
import sys

src, name = sys.argv[1], sys.argv[2]
lines = open(src).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(name) or (l.endswith(':') and name in l and not l.startswith('.')))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith('.Lfunc_end'))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r'^(\.LBB\w+):', l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(body):
    m = re.match(r'\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)', l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        lo = labels[m.group(2)]
        cnt = collections.Counter()
        for x in body[lo:i + 1]:
            x = x.strip()
            if not x or x.startswith(';') or x.startswith('.') or x.endswith(':'):
                continue
            op = x.split()[0]
            if op.startswith('v_') and '_dpp' in x:
                cnt['v_dpp'] += 1
            cnt[op] += 1
        tot = sum(v for k, v in cnt.items() if k != 'v_dpp')
        valu = sum(v for k, v in cnt.items() if k.startswith('v_') and k != 'v_dpp')
        print(f"loop {m.group(2)} lines {lo}-{i}: {tot} instr, {valu} VALU")
        for k, v in cnt.most_common(40):
            print(f"   {v:5d} {k}")
