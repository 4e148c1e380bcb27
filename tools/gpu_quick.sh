# tests (-m gpu) + a timing run of the headline workload + kernel trace summary
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/q/kt" -o kt -- python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-300} ${PROF_ARGS} > "$R/gpurun_out/q_kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; grep -v "^[WE]2026" "$R/gpurun_out/q_kt.log" | tail -2; head -4 "$R/gpurun_out/q/kt/kt_kernel_stats.csv"
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/q/fetch" -o fetch -- python3 "$R/tools/prof_run.py" --rounds 60 ${PROF_ARGS} > "$R/gpurun_out/q_fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; exit $rc
