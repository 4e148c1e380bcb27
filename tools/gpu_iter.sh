# Iteration loop: GPU parity tests, a bench line (no CPU baseline), kernel-trace summary.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/it
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/it/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/it/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/it/bench.json 2> gpurun_out/it/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/it/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/it/kt" -o kt -- python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-300} ${PROF_ARGS} > "$R/gpurun_out/it/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; tail -1 "$R/gpurun_out/it/kt.log"; python3 "$R/tools/kt_summary.py" "$R/gpurun_out/it/kt/kt_kernel_trace.csv" | head -5
exit $rc
