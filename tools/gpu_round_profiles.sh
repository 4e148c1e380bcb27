# Round profiles for profiles/<round>/: the bench line, rocprofv3 kernel trace + stats of the same
# command, PMC FETCH_SIZE / WRITE_SIZE passes (each its own run) of the round kernels, and the
# membench calibration pass for the gfx950 FETCH_SIZE correction.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/rp"; mkdir -p "$O"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 12 > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; tail -c 600 "$O/bench.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/kt_summary.py" "$O/kt/kt_kernel_trace.csv" > "$O/kt_summary.txt"; head -4 "$O/kt_summary.txt"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o p -- python3 "$R/tools/prof_run.py" --rounds 60 > "$O/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/calib_FETCH_SIZE" -o p -- "$R/tools/microbench/membench" > "$O/calib.log" 2>&1
rc=$?; echo "calib rc=$rc"; exit $rc
