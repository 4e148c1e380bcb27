# Full bench line + rocprofv3 kernel trace/stats of the same command + PMC passes (profiles/)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/bp
export GP_GRID=${GP_GRID:-16384}
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 12 > gpurun_out/bp/bench.json 2> gpurun_out/bp/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bp/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/bp/kt" -o kt -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/bp/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/kt_summary.py" "$R/gpurun_out/bp/kt/kt_kernel_trace.csv" | head -6
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  n=$(echo $c | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/bp/pmc_$n" -o p -- python3 "$R/tools/prof_run.py" --rounds 60 > /dev/null 2>&1
  echo "pmc $c rc=$?"
done
