# New GPU test: quiet waves on by default above 2^20 actors, across a reset.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "quiet" --timeout 250 --timeout-method thread > gpurun_out/quiet_tests.log 2>&1
rc=$?; tail -3 gpurun_out/quiet_tests.log; exit $rc
