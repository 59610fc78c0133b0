#!/usr/bin/env python3
"""Dependency distances inside one basic block of gfx950 assembly.

usage: tools/depdist.py block.s

For every VALU instruction, the number of instructions of the same wave issued
between it and the producer of its latest-ready VGPR source (an in-order wave
stalls on a dependent FP64 op issued fewer than ~2 VALU slots after its
producer: 9-cycle dependent latency vs ~4.6-cycle single-wave issue, profile
r03a_valu_issue.txt).  Prints the histogram of distances (in VALU instructions)
and the waitcnt positions.
"""
import collections
import re
import sys

lines = [l.strip() for l in open(sys.argv[1]) if l.strip() and not l.strip().startswith((";", "."))]


def regs(tok):
    out = []
    for m in re.finditer(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", tok):
        if m.group(3):
            out.append(int(m.group(3)))
        else:
            out.extend(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


last_write = {}
hist = collections.Counter()
nvalu = 0
close = []
for i, l in enumerate(lines):
    op = l.split()[0]
    ops = l[len(op):].split(",")
    if op.startswith("v_"):
        dst = regs(ops[0]) if ops else []
        srcs = [r for o in ops[1:] for r in regs(o)]
        if op.startswith("v_fmac"):
            srcs += dst
        d = min((nvalu - last_write[r] for r in srcs if r in last_write), default=99)
        hist[min(d, 8)] += 1
        if d <= 1:
            close.append((i, l))
        for r in dst:
            last_write[r] = nvalu
        nvalu += 1
    elif op.startswith("ds_read") or op.startswith("global_load"):
        for r in regs(ops[0]):
            last_write.pop(r, None)
print("VALU", nvalu, "distance histogram (VALU insts since producer; 8 = >=8 or none):")
for k in sorted(hist):
    print(f"  {k}: {hist[k]}")
print("distance <= 1:")
for i, l in close[:60]:
    print(f"  {i:4d} {l}")
