#!/bin/bash
# r04t: round record of the current build (GPU suite, smoke, bench line,
# rocprofv3 kernel stats, PMC passes), then the r04s plan-rounds A/B.
export TMPDIR=/tmp
TAG=r04t bash tools/gpu_final.sh || exit $?
bash tools/gpu_r04s.sh || exit $?
