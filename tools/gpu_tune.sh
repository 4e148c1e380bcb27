# tests (-m gpu), then round-kernel timing across grid sizes
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for gsz in ${GRIDS:-2048 4096 8192 16384}; do
  echo -n "grid=$gsz: "; GP_GRID=$gsz timeout -k 5 60 python3 tools/prof_run.py --rounds 300 ${PROF_ARGS} | tail -1 || exit 1
done
