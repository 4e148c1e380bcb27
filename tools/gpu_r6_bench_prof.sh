#!/bin/bash
# Round 6: the default bench line under rocprofv3 --kernel-trace --stats (the roofline's kernel average is
# checked against the trace of the same command), summarised by tools/kt_summary.py.  BENCH_ARGS=--no-cpu-baseline
# leaves out the CPU-baseline leg's same-rounds GPU run, so the trace holds the warm-up and timed steps only.
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_bench_prof}"; rm -rf "$O"; mkdir -p "$O"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 "$R/bench.py" ${BENCH_ARGS} > "$O/bench_line.json" 2> "$O/bench.err" ) || { echo "bench failed"; tail -5 "$O/bench.err"; exit 1; }
python3 tools/kt_summary.py "$O/kt/kt_kernel_trace.csv" > "$O/rocprof_kernel_summary_bench.txt" && head -5 "$O/rocprof_kernel_summary_bench.txt"
cp "$O/kt/kt_kernel_stats.csv" "$O/rocprof_kernel_stats_bench.csv" 2>/dev/null || find "$O/kt" -name '*kernel_stats.csv' -exec cp {} "$O/rocprof_kernel_stats_bench.csv" \;
find "$O/kt" -name '*kernel_trace.csv' -delete
cat "$O/bench_line.json"
