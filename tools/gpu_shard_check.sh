# Sharded engine on one GPU (loopback exchange) + the full GPU suite.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded.py -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_sharded.log 2>&1
rc=$?; echo "sharded rc=$rc"; tail -25 gpurun_out/gpu_sharded.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log; exit $rc
