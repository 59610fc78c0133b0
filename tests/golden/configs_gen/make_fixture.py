"""Generate expected_configs_int16 / expected_dims.txt by running the
reference's own generator (utils/construct_configs_all_studies.py) on the
small inputs in this directory.  Run in the build container (the reference is
not on the GPU box); the outputs are committed as test vectors:

    cd tests/golden/configs_gen && python make_fixture.py /root/reference
"""
import os
import subprocess
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
here = os.path.dirname(os.path.abspath(__file__))
subprocess.run([sys.executable, os.path.join(ref, "utils", "construct_configs_all_studies.py"), "imp_files.txt",
                "num_files.txt", "expected_configs_int16", "expected_dims.txt"], cwd=here, check=True,
               stdout=subprocess.DEVNULL)
