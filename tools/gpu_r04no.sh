#!/bin/bash
# r04n + r04o in one box session (tools/gpu_r04n.sh, tools/gpu_r04o.sh)
bash tools/gpu_r04n.sh || exit $?
bash tools/gpu_r04o.sh || exit $?
