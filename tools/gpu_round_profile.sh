# Round profile: bench line, rocprofv3 kernel trace/stats of the same bench command, PMC passes
# (FETCH_SIZE / WRITE_SIZE, separate runs) on the headline workload, FETCH_SIZE calibration.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${TAG:-r1}"; mkdir -p "$O"
export GP_GRID=${GP_GRID:-16384}
cd "$R"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 12 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 1800 "$O/bench.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$O/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/kt_summary.py" "$O/kt/kt_kernel_trace.csv" | head -4
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o p -- python3 "$R/tools/prof_run.py" --rounds 60 > /dev/null 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/calib_$c" -o p -- "$R/tools/microbench/membench" > /dev/null 2>&1
  rc=$?; echo "calib $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
