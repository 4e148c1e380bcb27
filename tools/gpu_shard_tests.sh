# Sharded engine: GPU parity tests (loopback shards on one GPU), then the shard bench at N=1 profiled
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_sharded.log 2>&1
rc=$?; echo "sharded rc=$rc"; tail -6 gpurun_out/gpu_sharded.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_shard_prof.sh
