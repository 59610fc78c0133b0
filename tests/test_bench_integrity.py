"""bench.py's integrity gates (CPU: they fire before any GPU work).

A timing-ablation build switch has no environment form in the shipped library
any more (-DPSX_ABLATE_MERGE is compile-time only), and bench.py refuses to
print a line while any PSX_ABLATE_* variable is set."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_ablation_variables():
    env = dict(os.environ, PSX_ABLATE_MERGE="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert r.stdout == ""
    assert "PSX_ABLATE_MERGE" in r.stderr


def test_engine_has_no_ablation_environment_switch():
    """The library's sources read no PSX_ABLATE_* variable (the merge ablation
    is a separate -D build)."""
    src = os.path.join(ROOT, "pipsort_amd", "csrc")
    for f in os.listdir(src):
        with open(os.path.join(src, f)) as fh:
            text = fh.read()
        assert 'getenv("PSX_ABLATE' not in text, f
