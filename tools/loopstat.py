#!/usr/bin/env python3
"""Static instruction counts of the innermost loop of a HIP kernel (gfx950).

usage: tools/loopstat.py file.hip kernel_regex [--rare LABEL ...]

Compiles to assembly, finds the innermost loop by the assembler's
"Depth=N" block annotations and prints per-block VALU / LDS / VMEM counts plus
the opcode histogram of the whole loop.  Blocks passed with --rare (rarely
taken branches) are listed but left out of the total.
"""
import collections
import re
import subprocess
import sys

import os
import shlex

src, kre = sys.argv[1], sys.argv[2]
rare = set(sys.argv[sys.argv.index("--rare") + 1:]) if "--rare" in sys.argv else set()
extra = shlex.split(os.environ.get("LOOPSTAT_FLAGS", ""))  # e.g. scheduler options of an A/B build
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I",
                "/root/repo/pipsort_amd/csrc", "--cuda-device-only", "-S", src, "-o", "/tmp/loopstat.s"] + extra,
               check=True, stderr=subprocess.DEVNULL)
s = open("/tmp/loopstat.s").read()
for name in re.findall(r"^(\S+):", s, re.M):
    if name.startswith(".") or not re.search(kre, name):
        continue
    lines = s[s.find(name + ":"):s.find(".Lfunc_end", s.find(name + ":"))].split("\n")
    blocks, cur = collections.OrderedDict(), None
    for l in lines:
        t = l.strip()
        m = re.match(r"^(\.LBB\S+):\s*(;.*)?$", t)
        if m:
            cur = m.group(1)
            blocks[cur] = {"ann": m.group(2) or "", "ins": []}
            continue
        if cur is None:
            continue
        if t.startswith(";"):
            if "Loop Header" in t or "Depth=" in t:
                blocks[cur]["ann"] += " " + t
            continue
        if t and not t.startswith("."):
            blocks[cur]["ins"].append(t)
    depth = max((int(x) for b in blocks.values() for x in re.findall(r"Depth=(\d+)", b["ann"])), default=0)
    tot = collections.Counter()
    print(name[:80], "innermost depth", depth)
    for lab, b in blocks.items():
        if f"Depth={depth}" not in b["ann"]:
            continue
        c = collections.Counter(i.split()[0] for i in b["ins"])
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))
        tag = " (rare, excluded)" if lab in rare else ""
        print(f"  {lab:10s} n={len(b['ins']):4d} valu={valu:4d} lds={lds:3d} vmem={vmem:3d}{tag}")
        if lab not in rare:
            tot.update(c)
    print("  loop VALU", sum(v for k, v in tot.items() if k.startswith("v_")),
          "LDS", sum(v for k, v in tot.items() if k.startswith("ds_")),
          "SALU", sum(v for k, v in tot.items() if k.startswith("s_")))
    print("  ", sorted(((v, k) for k, v in tot.items() if k.startswith("v_")), reverse=True)[:24])
