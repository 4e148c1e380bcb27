#!/bin/bash
# Round 6, last GPU call: the SCALE path on one box (dist tests, --one-device 2 / 4 lines), then the whole
# GPU suite, smoke() and the bench line (tools/gpu_r6_scale.sh, tools/gpu_r6_suite.sh).
R=$(pwd)
OUT=r6_scale bash tools/gpu_r6_scale.sh || exit $?
OUT=r6_suite bash tools/gpu_r6_suite.sh
