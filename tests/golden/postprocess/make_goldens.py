"""Generate the post-processing golden vectors (run in the build container
only: it executes the reference's own utils scripts, which never ship).

    python tests/golden/postprocess/make_goldens.py /root/reference

Inputs are the reference's expected PIPSORT outputs for tests/example
(tests/golden/example/expected_*); outputs are what the reference's
run_example.sh:3-5 post-processing steps (utils/get_global_pips.py,
utils/get_not_shared_pips.py) write from them."""
import os
import shutil
import subprocess
import sys
import tempfile

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
here = os.path.dirname(os.path.abspath(__file__))
ex = os.path.join(here, "..", "example")
with tempfile.TemporaryDirectory() as d:
    for s in ("study0_post", "study1_post", "shared_pips"):
        shutil.copy(os.path.join(ex, f"expected_{s}.txt"), os.path.join(d, f"r_{s}.txt"))
    subprocess.run([sys.executable, os.path.join(ref, "utils", "get_global_pips.py"), "r_study0_post.txt",
                    "r_study1_post.txt", "r_shared_pips.txt", "global_pips.txt"], cwd=d, check=True,
                   stdout=subprocess.DEVNULL)
    subprocess.run([sys.executable, os.path.join(ref, "utils", "get_not_shared_pips.py"), "r_shared_pips.txt",
                    "global_pips.txt", "not_shared_pips.txt"], cwd=d, check=True, stdout=subprocess.DEVNULL)
    for f in ("global_pips.txt", "not_shared_pips.txt"):
        shutil.copy(os.path.join(d, f), os.path.join(here, f"example_{f}"))
print("ok")
