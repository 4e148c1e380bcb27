set -o pipefail
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/prof"
rocprofv3 -L > "$R/gpurun_out/prof/counters.txt" 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof/kt" -o kt -- python3 "$R/tools/prof_run.py" --rounds 300 > "$R/gpurun_out/prof/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; tail -2 "$R/gpurun_out/prof/kt.log"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/prof/fetch" -o fetch -- python3 "$R/tools/prof_run.py" --rounds 100 > "$R/gpurun_out/prof/fetch.log" 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/prof/write" -o write -- python3 "$R/tools/prof_run.py" --rounds 100 > "$R/gpurun_out/prof/write.log" 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/prof/tcc" -o tcc -- python3 "$R/tools/prof_run.py" --rounds 100 > "$R/gpurun_out/prof/tcc.log" 2>&1
rc=$?; echo "tcc rc=$rc"
exit $rc
