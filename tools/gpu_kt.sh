# kernel trace + stats of the headline workload (per-kernel durations)
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt" -o kt -- python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-300} ${PROF_ARGS} > "$R/gpurun_out/kt.log" 2>&1
rc=$?; grep -v "^[WE]2026" "$R/gpurun_out/kt.log" | tail -1; python3 "$R/tools/kt_summary.py" "$R/gpurun_out/kt/kt_kernel_trace.csv"; exit $rc
