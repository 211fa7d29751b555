#!/usr/bin/env python3
"""Prints the waits, loads and instruction mix of the row loop(s) of one kernel in a .s file:
python scripts/isa_loop.py /tmp/glm_u2.s <kernel-name-substring>"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
sub = sys.argv[2]
i = next(k for k, l in enumerate(L) if l.startswith("_Z") and sub in l and l.rstrip().endswith(sub.split()[-1]) or (l.startswith("_Z") and sub in l and ":" in l))
j = i
while not L[j].startswith(".Lfunc_end"):
    j += 1
body = L[i:j]
print(body[0][:120], len(body), "lines")
# loops: header label -> back-edge branch
labels = {l.split(":")[0]: k for k, l in enumerate(body) if re.match(r"^\.LBB\d+_\d+:", l)}
loops = []
for k, l in enumerate(body):
    m = re.match(r"\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < k:
        loops.append((labels[m.group(1)], k))
for a, b in loops:
    seg = body[a:b + 1]
    if not any("global_load_dwordx4" in x or "global_load_lds" in x for x in seg):
        continue
    c = collections.Counter()
    for x in seg:
        t = x.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        if op.startswith("s_waitcnt"):
            c[t] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
        else:
            c[op] += 1
    print("loop", a, "-", b, dict(c))
