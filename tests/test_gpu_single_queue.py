"""psx_single_queue (the drop-in CLI's mode: one stream, one hardware queue per
device for the whole process).  The mode is process-wide, so the checks run in
a child process: under it the synchronous pass, back-to-back asynchronous
passes (their compute stream is the engine stream) and a world-2 sharded
exchange give the accumulators of an ordinary synchronous pass.  Marked gpu;
run on an MI355X."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
import torch  # its HIP runtime first, as the gpu fixture and bench.py load it
sys.path[:0] = [{root!r}, {tests!r}]
from pipsort_amd import engine as E
from pipsort_amd import synth
from test_gpu_parity import _sexp

lib = E.load_library()
assert lib.psx_single_queue(1) == 0
ld, z, _, _, u2l = synth.mixed_locus(300, 320, 260, seed=300)
mi = E.model_inputs(ld, z, u2l, (5000, 9000), max_causal=3, sharing_param=0.4)
F = ("post", "no_causal", "shared", "shared_ll", "notshared_ll")

ref = E.PostCal(mi)
ref.run_exhaustive()
r = ref.accum()

a = E.PostCal(mi)
for _ in range(5):
    a.run_exhaustive_async()
assert a.sync() is False
g = a.accum()
assert g.n_configs == r.n_configs and g.total == r.total
for f in F:
    assert np.array_equal(getattr(g, f), getattr(r, f)), f

world = 2
nb = ref.partials_bytes()
buf = torch.empty(nb * world, dtype=torch.uint8, device="cuda")
pcs = []
for k in range(world):
    pc = E.PostCal(mi)
    pc.set_shard(k, world)
    pcs.append(pc)
for step in range(2):
    for k, pc in enumerate(pcs):
        pc.run_exhaustive_async()
        pc.export_partials(buf.data_ptr() + k * nb)
    torch.cuda.synchronize()
    for pc in pcs:
        pc.merge_partials(buf.data_ptr(), world)
for pc in pcs:
    assert pc.sync() is False
    g = pc.accum()
    assert g.n_configs == r.n_configs
    for f in ("post", "no_causal", "shared"):
        d = np.abs(_sexp(getattr(g, f), g.total) - _sexp(getattr(r, f), r.total)).max()
        assert d <= 1e-12, f
    for f in ("shared_ll", "notshared_ll"):
        np.testing.assert_allclose(getattr(g, f), getattr(r, f), rtol=1e-12)
print("single-queue ok")
"""


def test_single_queue_passes_match(gpu):
    code = CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "single-queue ok" in p.stdout
