# 8 shards of the 1e9-node C5 graph on one GPU (loopback exchange), 16 rounds, kernel trace:
# per-rank kernel costs of the 8-GPU run with the current round kernel.
set -o pipefail
OUT=c5_loopback8 KT_TIMEOUT=500 KT_LINES=10 LOOP_ARGS="--world 8 --n 1000000000 --rounds 16" bash tools/gpu.sh loop
