# Sharded engine: GPU parity tests (loopback shards on one GPU), then 8 loopback shards of 80M
# (kernel costs at a realistic remote fraction), then the shard bench at N=1 profiled
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_sharded.log 2>&1
rc=$?; echo "sharded rc=$rc"; tail -6 gpurun_out/gpu_sharded.log; [ $rc -eq 0 ] || exit $rc
ARGS="--world 8 --n 80000000 --rounds 64" bash tools/gpu_shard_ab.sh || exit 1
[ -n "$NO_PROF" ] || bash tools/gpu_shard_prof.sh
