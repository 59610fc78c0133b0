"""Multi-process sharded sweep (bench.py under torch.distributed.run).  On a
one-GPU box both ranks share cuda:0 and exchange partials over gloo
(PSX_DIST_BACKEND=gloo, host-staged); on a node the same code uses RCCL."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_bench_sharded_two_ranks(gpu, world):
    env = dict(os.environ, PSX_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--workload", "syn200c2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]  # the bench line alone on stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world
    # every rank's shard folded into rank 0's accumulators: all configurations counted once
    assert out["configs_checked"] == out["config"]["configs_per_step"] == 179_701
    # the SSS walk with its batches split across the ranks (psx_run_sss_sharded):
    # the same walk and configuration count as one GPU (bench sss line, r01x)
    assert out["sss"]["walk_iterations"] == 2 and out["sss"]["walk_configs"] == 23_993


def test_bench_rccl_path_world1(gpu):
    """The N > 1 code path with the nccl (= RCCL) backend, on the one GPU of a
    test box (PSX_FORCE_DIST=1 at world 1): RCCL communicator, all-gather of
    the partial images on the engine stream, barrier / max-over-ranks timing,
    sharded SSS walk.  RCCL prints a version banner at init; stdout must still
    hold the bench line alone."""
    env = dict(os.environ, PSX_FORCE_DIST="1")
    env.pop("PSX_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--workload", "syn200c2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    out = json.loads(lines[0])
    assert "RCCL" in out["config"]["parallelism"]
    assert out["configs_checked"] == out["config"]["configs_per_step"] == 179_701
    assert out["sss"]["walk_iterations"] == 2 and out["sss"]["walk_configs"] == 23_993
    assert "on the device" in out["sss"]["multi_gpu"]  # psx_run_sss_sharded_dev under RCCL
    assert out["single_pass_ms"] > 0  # one locus swept once, RCCL exchange included


def test_bench_gpus2_launches_its_own_ranks(gpu):
    """`python bench.py --gpus 2` with no launcher (WORLD_SIZE unset) starts two
    ranks itself (a torch.distributed.run child, before any GPU call) and the
    line reports both: n_gpus 2, a 2-rank process group, every configuration of
    the locus counted once after the exchange.  gloo lets the two ranks share
    this box's one GPU; on a node each rank gets its own GPU over RCCL."""
    env = dict(os.environ, PSX_DIST_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--workload", "syn200c2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2
    assert out["configs_checked"] == out["config"]["configs_per_step"] == 179_701


def test_bench_gpus_more_than_visible_fails(gpu):
    """With the RCCL backend, asking for more GPUs than are visible fails
    non-zero instead of silently measuring fewer."""
    import torch
    env = dict(os.environ)
    env.pop("PSX_DIST_BACKEND", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    n = torch.cuda.device_count() + 1
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1", "--warmup", "0",
           "--workload", "syn200c2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and r.stdout == ""
    assert f"--gpus {n} but only" in r.stderr


def test_bench_gpus2_rccl(gpu):
    """`bench.py --gpus 2` over RCCL, one GPU per rank: runs on a box with two
    or more GPUs (the driver's node), skipped on a one-GPU box.  The line
    reports the 2-rank RCCL world, the merged count and one plan hash."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("one device visible")
    env = dict(os.environ)
    env.pop("PSX_DIST_BACKEND", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--workload", "syn200c2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2 and "RCCL" in out["config"]["parallelism"]
    assert out["configs_checked"] == out["config"]["configs_per_step"] == 179_701
    assert len(out["plan_hash"]) == 16


def test_merge_refuses_mismatched_plans(gpu):
    """psx_merge_partials checks every image's PlanTag on the device: images of
    shards of different worlds, out of rank order, or of another locus are
    refused with an error (never folded into a wrong total)."""
    import torch
    sys.path.insert(0, ROOT)
    from pipsort_amd import engine as E
    from pipsort_amd import synth
    ld, z, _, _, u2l = synth.syn_v1(120)
    seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=2, sharing_param=0.25)
    ld2, z2, _, _, u2l2 = synth.syn_v1(125)  # same image size (ldg 128), another locus
    other = E.seam_from_arrays(ld2, z2, u2l2, (10000, 8000), max_causal=2, sharing_param=0.25)
    h = [E.PostCal(seam), E.PostCal(seam), E.PostCal(other)]
    nb = h[0].partials_bytes()
    buf = torch.empty(2 * max(nb, h[2].partials_bytes()), dtype=torch.uint8, device="cuda")

    def merge(a, ra, wa, b, rb, wb):
        a.set_shard(ra, wa)
        b.set_shard(rb, wb)
        a.run_exhaustive()
        b.run_exhaustive()
        a.export_partials(buf.data_ptr())
        b.export_partials(buf.data_ptr() + nb)
        torch.cuda.synchronize()
        m = E.PostCal(seam)
        try:
            m.merge_partials(buf.data_ptr(), 2)
            return m.accum().n_configs
        finally:
            m.close()

    assert merge(h[0], 0, 2, h[1], 1, 2) == seam.count_configs()  # the good case
    for args in ((h[0], 0, 2, h[1], 1, 3),    # another world
                 (h[0], 1, 2, h[1], 0, 2)):   # out of rank order
        with pytest.raises(E.EngineError, match="one plan"):
            merge(*args)
    if h[2].partials_bytes() == nb:  # another locus of the same image size: another hash
        with pytest.raises(E.EngineError, match="one plan"):
            merge(h[0], 0, 2, h[2], 1, 2)
    for x in h:
        x.close()


def test_refused_merge_leaves_handle_usable(gpu):
    """A refused merge writes nothing and is reported once: the same merge
    handle keeps its accumulators bitwise, and the next good merge (and the
    next psx_sync) succeed.  With a caller stream the refusal comes from
    psx_sync, after its pass bookkeeping."""
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from pipsort_amd import engine as E
    from pipsort_amd import synth
    ld, z, _, _, u2l = synth.syn_v1(120)
    seam = E.seam_from_arrays(ld, z, u2l, (10000, 8000), max_causal=2, sharing_param=0.25)
    a, b, m = E.PostCal(seam), E.PostCal(seam), E.PostCal(seam)
    nb = a.partials_bytes()
    good = torch.empty(2 * nb, dtype=torch.uint8, device="cuda")
    bad = torch.empty(2 * nb, dtype=torch.uint8, device="cuda")
    for dst, (r0, r1) in ((good, (0, 1)), (bad, (1, 0))):
        a.set_shard(r0, 2)
        b.set_shard(r1, 2)
        a.run_exhaustive()
        b.run_exhaustive()
        a.export_partials(dst.data_ptr())       # bad: rank 1's image first
        b.export_partials(dst.data_ptr() + nb)
    torch.cuda.synchronize()
    fields = ("post", "shared", "shared_ll", "notshared_ll", "no_causal")

    def snap():
        r = m.accum()
        return r.n_configs, np.float64(r.total).tobytes(), [np.asarray(getattr(r, f)).tobytes() for f in fields]

    m.merge_partials(good.data_ptr(), 2)
    ref = snap()
    assert ref[0] == seam.count_configs()
    with pytest.raises(E.EngineError, match="one plan"):
        m.merge_partials(bad.data_ptr(), 2)
    assert snap() == ref                       # nothing folded
    m.merge_partials(good.data_ptr(), 2)       # reported once: the handle merges again
    assert snap() == ref
    assert not m.sync()
    # caller's stream: no host check in merge_partials; psx_sync reports it once
    stream = torch.cuda.Stream()
    m.set_stream(stream.cuda_stream)
    m.merge_partials(bad.data_ptr(), 2)
    with pytest.raises(E.EngineError, match="one plan"):
        m.sync()
    assert not m.sync()
    assert snap() == ref
    for x in (a, b, m):
        x.close()
