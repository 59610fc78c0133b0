#!/usr/bin/env python3
"""Schedule view of k_sweep3<true>'s pipelined step loop (its largest basic block):
VALU count per two steps and, for every vector-memory wait, how many
instructions separate it from the loads it waits for.
    python tools/hotblock.py [-D...] ...   (extra hipcc flags, e.g. A/B defines)
Diagnostics only."""
import collections
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", ROOT + "/pipsort_amd/csrc",
                "--cuda-device-only", "-S", ROOT + "/pipsort_amd/csrc/psx_sweep3.hip", "-o", "/tmp/hotblock.s"]
               + sys.argv[1:], check=True, stderr=subprocess.DEVNULL)
s = open("/tmp/hotblock.s").read()
name = next(n for n in re.findall(r"^(\S+):", s, re.M) if re.search("k_sweep3ILb1", n))
body = s[s.find(name + ":"):s.find(".Lfunc_end", s.find(name + ":"))]
blocks, cur = {}, None
for l in body.split("\n"):
    t = l.strip()
    m = re.match(r"^(\.LBB\S+):", t)
    if m:
        cur = m.group(1)
        blocks[cur] = []
    elif cur and t and not t.startswith((";", ".")):
        blocks[cur].append(t)
lab, ins = max(blocks.items(), key=lambda kv: sum(i.startswith("v_") for i in kv[1]))
c = collections.Counter(i.split()[0] for i in ins)
print(f"{lab}: {len(ins)} instructions, VALU {sum(v for k, v in c.items() if k.startswith('v_'))}, "
      f"LDS {sum(v for k, v in c.items() if k.startswith('ds_'))}, waitcnt {c['s_waitcnt']}")
loads = []  # (index, text) of outstanding vector-memory loads, in issue order (rotating: previous iteration first)
prev = [i for i, t in enumerate(ins) if t.startswith("global_load")]
order = [(i - len(ins), ins[i]) for i in prev] + [(i, ins[i]) for i in prev]
issued = [(i - len(ins)) for i in prev]
for i, t in enumerate(ins):
    if t.startswith("global_load"):
        issued.append(i)
    m = re.search(r"vmcnt\((\d+)\)", t) if t.startswith("s_waitcnt") else None
    if m:
        n = int(m.group(1))
        done = issued[:len(issued) - n]
        if done:
            print(f"  @{i:4d} vmcnt({n}): newest awaited load issued {i - done[-1]} instructions earlier")
        issued = issued[len(issued) - n:]
