"""Developer smoke run on the GPU box: engine vs oracle on the fixture loci."""
import os, sys, time, subprocess, shutil, tempfile
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from pipsort_amd import engine as E
from oracle import oracle as O
import loci

def cmp(name, a, o):
    pe, ne, se = a.pips()
    def se_(v, t):
        r = np.exp(v - t); r[v == 0] = 0; return r
    po, no, so = se_(o["post"], o["total"]), se_(o["no_causal"], o["total"]), se_(o["shared"], o["total"])
    d = max(np.abs(pe - po).max(), np.abs(ne - no).max(), np.abs(se - so).max())
    def lld(x, y):
        m = (x != 0) | (y != 0)
        return np.abs(x[m] - y[m]).max() if m.any() else 0.0
    print(f"{name}: maxPIPdiff={d:.3e} total {a.total:.10f} vs {o['total']:.10f} "
          f"sll {lld(a.shared_ll, o['shared_ll']):.2e} nsll {lld(a.notshared_ll, o['notshared_ll']):.2e} "
          f"nconf {a.n_configs} vs {o['n_configs']}", flush=True)
    return d

print("devices", E.device_count(), flush=True)
for c in (1, 2, 3):
    seam, L = loci.seam_for(loci.SMALL, c=c)
    pc = E.PostCal(seam)
    pc.run_exhaustive()
    cmp(f"small c={c}", pc.accum(), O.postcal(seam))
    pc.close()
seam, L = loci.seam_for(loci.EXAMPLE)
pc = E.PostCal(seam)
t = time.time(); pc.run_exhaustive(); dt = time.time() - t
cmp("example c=2", pc.accum(), O.postcal(seam))
print("example timing", dt, pc.timing(), flush=True)
# CLI end to end
tmp = tempfile.mkdtemp()
for f in os.listdir(L["dir"]):
    shutil.copy(os.path.join(L["dir"], f), tmp)
t = time.time()
r = subprocess.run([E.PIPSORT_BIN, "-c", "2", "-l", "ldfiles.txt", "-z", "zfiles.txt", "-m", "snp_map", "-n",
                    "334324,6771", "-p", "0.25", "-o", "pipsort_results"], cwd=tmp, capture_output=True, text=True)
print("CLI rc", r.returncode, "wall", time.time() - t, r.stdout[-600:], r.stderr[-600:], flush=True)
for f in ("study0_post", "study1_post", "study0_set", "study1_set", "nocausal", "shared_pips"):
    a = open(os.path.join(tmp, f"pipsort_results_{f}.txt")).read()
    b = open(os.path.join(tmp, f"expected_{f}.txt")).read()
    print(f, "IDENTICAL" if a == b else "DIFF", flush=True)
# configs path
seam, L = loci.seam_for(loci.CONFIGS)
rows = np.fromfile(os.path.join(L["dir"], "all_configs_int16"), dtype=np.int16).reshape(72, 5)
pc = E.PostCal(seam); pc.run_configs(rows)
cmp("configs", pc.accum(), O.postcal(seam, "configs", rows))
# SSS
seam, L = loci.seam_for(loci.SMALL)
pc = E.PostCal(seam); it = pc.run_sss()
cmp(f"sss small (it={it})", pc.accum(), O.postcal(seam, "sss"))
# synthetic
from pipsort_amd import synth
for M, c in ((100, 3), (200, 2)):
    ld, z, names, rows_, u2l = synth.syn_v1(M)
    seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=c, sharing_param=0.25)
    pc = E.PostCal(seam); t = time.time(); pc.run_exhaustive(); dt = time.time() - t
    t2 = time.time(); o = O.postcal(seam); dto = time.time() - t2
    cmp(f"syn M={M} c={c} gpu {dt:.3f}s oracle {dto:.2f}s", pc.accum(), o)
ld, z, names, rows_, u2l = synth.mixed_locus(90, 110, 60)
seam = E.seam_from_arrays(ld, z, u2l, (5000, 9000), max_causal=3, sharing_param=0.5)
pc = E.PostCal(seam); pc.run_exhaustive()
cmp("mixed c=3", pc.accum(), O.postcal(seam))
for M in (500, 1000):
    ld, z, names, rows_, u2l = synth.syn_v1(M)
    t = time.time()
    seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=3, sharing_param=0.25)
    ts = time.time() - t
    pc = E.PostCal(seam)
    for rep in range(3):
        t = time.time(); pc.run_exhaustive(); dt = time.time() - t
        tm = pc.timing()
        a = pc.accum()
        print(f"SYN M={M} c=3 setup {ts:.2f}s run {dt*1e3:.2f} ms  configs {a.n_configs} -> {a.n_configs/dt:.3e}/s  {tm}", flush=True)
