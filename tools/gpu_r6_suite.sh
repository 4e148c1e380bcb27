#!/bin/bash
# Round 6: the whole GPU suite (as the driver runs it), then smoke() and a short bench line.
R=$(pwd); O="$R/gpurun_out/${OUT:-r6_suite}"; rm -rf "$O"; mkdir -p "$O"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$O/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 "$O/smoke.txt"; [ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python -u bench.py > "$O/bench_line.json" 2> "$O/bench.err"; rc=$?; echo "bench rc=$rc"; cat "$O/bench_line.json"; exit $rc
