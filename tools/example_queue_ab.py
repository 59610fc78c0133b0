"""A/B of the CLI on tests/example: PSX_SINGLE_QUEUE=1 (default) vs 0, phases per run.  Developer tool."""
import os, sys, json
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
import bench
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for sq, wn, lj in (("1", "0", "1"), ("1", "1", "1"), ("1", "0", "0"), ("0", "1", "0")):
        os.environ.update(PSX_SINGLE_QUEUE=sq, PSX_WARM_NULL=wn, PSX_LU_JOINT=lj)
        w, same, ph = bench.example_wall()
        print(f"queue1={sq} warm_null={wn} lu_joint={lj}", round(w, 3), same, {k: round(ph[k], 1) for k in ("hip_runtime_ms", "context_and_code_load_ms", "wait_for_gpu_ms", "gpu_setup_ms", "sweep_ms", "exit_ms")},
              flush=True)
