#!/bin/bash
bash tools/gpu_r04w.sh || exit $?
bash tools/gpu_r04v.sh || exit $?
