# Round profile: bench line (with CPU baseline), rocprofv3 kernel trace/stats of the same bench
# command, PMC passes (FETCH_SIZE, WRITE_SIZE; one per run) on a fixed 60-round workload, and the
# FETCH_SIZE calibration pass on membench.  Output under gpurun_out/rp/.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; rm -rf gpurun_out/rp; mkdir -p gpurun_out/rp
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 12 > gpurun_out/rp/bench.json 2> gpurun_out/rp/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/rp/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/rp/kt" -o kt -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/rp/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/kt_summary.py" "$R/gpurun_out/rp/kt/kt_kernel_trace.csv" | head -6
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/rp/pmc_$c" -o p -- python3 "$R/tools/prof_run.py" --rounds 60 > "$R/gpurun_out/rp/pmc_$c.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/rp/calib_fetch" -o c -- "$R/tools/microbench/membench" > "$R/gpurun_out/rp/calib.log" 2>&1
rc=$?; echo "calib rc=$rc"; exit $rc
