# GPU suite on the current build, then the per-rank kernel costs of C5 (1e9-node Imp3D push-sum)
# split over 8 shards on one GPU (loopback exchange), under a rocprofv3 kernel trace.
set -o pipefail
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
OUT=c5loop KT_TIMEOUT=500 KT_LINES=14 LOOP_ARGS="--world 8 --n 1000000000 --rounds 16" bash tools/gpu.sh loop
