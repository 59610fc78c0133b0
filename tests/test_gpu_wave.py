"""The transposed wave reductions of k_sweep3 (psx_wave.h: v_permlane32_swap /
v_permlane16_swap halving the batch, then row DPP) against host sums and
maxima on one wave: exact on integer-valued doubles, batches of 4 .. 16 values
(pipsort_amd/bin/wave_red_probe, built with the engine from
tools/wave_red_probe.hip)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "pipsort_amd", "bin", "wave_red_probe")

pytestmark = pytest.mark.gpu


def test_transposed_wave_reductions_exact(gpu):
    assert os.path.exists(PROBE), "build the engine first (make -C pipsort_amd)"
    r = subprocess.run([PROBE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "wave_red_probe: ok (0 mismatches)" in r.stdout
