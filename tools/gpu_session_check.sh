# Session start check: smoke, GPU parity tests, round-kernel timing across grid sizes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
echo "nproc $(nproc)" > gpurun_out/host.txt; lscpu | head -20 >> gpurun_out/host.txt
timeout -k 10 150 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for gsz in ${GRIDS:-0 4096 8192 16384 38832}; do
  echo -n "grid=$gsz: "; GP_GRID=$gsz timeout -k 5 60 python3 tools/prof_run.py --rounds 300 | tail -1 || exit 1
done
