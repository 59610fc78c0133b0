#!/bin/bash
# r04p + r04q in one box session
bash tools/gpu_r04q.sh || exit $?
bash tools/gpu_r04p.sh || exit $?
