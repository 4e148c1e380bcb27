# One launcher for GPU-box runs (gpurun -- 'bash tools/gpu.sh MODE').  Everything lands in
# gpurun_out/<MODE>/; every GPU step has its own time limit and the script stops at the first
# failing step.
#   tests   pytest -m gpu
#   iter    tests + a bench line (no CPU baseline) + a kernel trace of 300 rounds (prof_run.py)
#   bench   the default bench.py line (with the CPU baseline) + its rocprofv3 kernel trace/stats
#   pmc     FETCH_SIZE and WRITE_SIZE passes (one run each) over 60 rounds of prof_run.py
#   loop    kernel trace of W loopback shards of one graph (tools/shard_loopback_prof.py $LOOP_ARGS)
#   ab      kernel-trace A/B of the variant libraries named in $VARIANTS (lib_<name>/, GP_LIB)
#   abpmc   one FETCH_SIZE pass per variant library of $VARIANTS over $ROUNDS (default 60) rounds
#   cli     CLI convergence times of the variant libraries of $VARIANTS on each workload of
#           $CLI_CASES ("N topo algo;N topo algo"), $REPS (default 3) interleaved runs
#   loopab  `loop` for each variant library of $VARIANTS
#   ktrun   kernel trace of one prof_run.py run ($ROUNDS, default: to convergence)
#   ktrun_bench  kernel trace of bench.py with the arguments given as the second argument
#   pmcrun  FETCH_SIZE and WRITE_SIZE passes over a whole run (prof_run.py, $ROUNDS default: to
#           convergence) -> tools/pmc_run_summary.py ($PMC_WORKLOAD, $PMC_KERNEL) into $O
#   pmcphase counters per kernel by phase of one run (tools/pmc_phase_table.py; $PMC_* below the case)
#   pmcgroup the same passes, summed over the kernels of one round ($PMC_KERNELS, comma list) and
#           divided by $PMC_ROUNDS -> tools/pmc_group_summary.py ($PMC_WORKLOAD, $PMC_GROUP)
# Extra prof_run.py arguments: $PROF_ARGS; rounds: $ROUNDS; bench.py arguments: $BENCH_ARGS;
# output directory name: $OUT (default: the mode).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
MODE=${1:-iter}
O="$R/gpurun_out/${OUT:-$MODE}"; rm -rf "$O"; mkdir -p "$O"
step() { echo "== $*"; }
tests() {
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${TEST_ARGS} > "$O/gpu_tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$O/gpu_tests.log"; return $rc
}
kt() {  # $1 = output name, rest = command
  local n=$1; shift
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 ${KT_TIMEOUT:-240} rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$n" -o kt -- "$@" > "$O/$n.log" 2>&1 )
  rc=$?; echo "kt $n rc=$rc"; tail -1 "$O/$n.log"; [ $rc -eq 0 ] || return $rc
  python3 "$R/tools/kt_summary.py" "$O/$n/kt_kernel_trace.csv" > "$O/$n.summary" && head -n ${KT_LINES:-6} "$O/$n.summary" || return $?
  # KT_POST (dev-only): the name of one post-processing script of tools/ run on the trace before it is
  # dropped (KT_DROP=1: the trace CSV is too big to travel back, gpurun merges 64 MiB at most); only
  # the names below are accepted, nothing from the environment is evaluated
  case "${KT_POST:-}" in
    "") ;;
    trace_overlap|trace_gaps|loop_phase_kernels|kt_round_series)
      python3 "$R/tools/$KT_POST.py" "$O/$n/kt_kernel_trace.csv" ${KT_POST_ARGS} > "$O/$n.post" 2>&1; cat "$O/$n.post" ;;
    *) echo "KT_POST=$KT_POST: not one of trace_overlap, trace_gaps, loop_phase_kernels, kt_round_series"; return 2 ;;
  esac
  if [ "${KT_DROP:-0}" = 1 ]; then rm -f "$O/$n/kt_kernel_trace.csv"; fi
}
case $MODE in
  tests) tests ;;
  iter)
    tests || exit $?
    timeout -k 10 240 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err"
    rc=$?; echo "bench rc=$rc"; cat "$O/bench.json"; [ $rc -eq 0 ] || exit $rc
    kt kt python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-300} ${PROF_ARGS} ;;
  bench)
    timeout -k 10 300 python3 bench.py ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err"
    rc=$?; echo "bench rc=$rc"; cat "$O/bench.json"; [ $rc -eq 0 ] || exit $rc
    kt kt python3 "$R/bench.py" --no-cpu-baseline ${BENCH_ARGS} ;;
  pmc)
    # one rocprofv3 run per pass; counters of one pass joined by commas in $PMC_EXTRA
    for c in FETCH_SIZE WRITE_SIZE ${PMC_EXTRA}; do
      n=${c%%,*}
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc ${c//,/ } --output-format csv -d "$O/pmc_$n" -o p -- python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-60} ${PROF_ARGS} > "$O/pmc_$n.log" 2>&1 )
      rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 "$R/tools/pmc_summary.py" "$O" > "$O/summary.txt" 2>&1; cat "$O/summary.txt" ;;
  loop)  # W shards of one graph on this GPU (loopback exchange) under a kernel trace
    kt kt python3 "$R/tools/shard_loopback_prof.py" ${LOOP_ARGS} ;;
  ab)
    for v in ${VARIANTS}; do
      GP_LIB=lib_$v kt "kt_$v" python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-300} ${PROF_ARGS} || exit $?
    done ;;
  abpmc)
    for v in ${VARIANTS}; do
      ( cd /tmp && export TMPDIR=/tmp && GP_LIB=lib_$v timeout -s KILL 90 rocprofv3 --pmc ${PMC_COUNTERS:-FETCH_SIZE} --output-format csv -d "$O/pmc_$v" -o p -- python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-60} ${PROF_ARGS} > "$O/pmc_$v.log" 2>&1 )
      rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
      python3 "$R/tools/pmc_summary.py" "$O/pmc_$v" k_ps_pull | sed "s/^/$v /"
    done ;;
  pmcrun)
    for c in FETCH_SIZE WRITE_SIZE; do
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o p -- python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-1000000} ${PROF_ARGS} > "$O/pmc_$c.log" 2>&1 )
      rc=$?; echo "pmc $c rc=$rc"; tail -1 "$O/pmc_$c.log"; [ $rc -eq 0 ] || exit $rc
    done
    python3 "$R/tools/pmc_run_summary.py" "$O/pmc_FETCH_SIZE" "$O/pmc_WRITE_SIZE" "$O/pmc_run.json" "${PMC_WORKLOAD:-10000000 Imp3D push-sum}" "${PMC_KERNEL:-k_ps_quiet<1>}" ;;
  pmcgroup)
    for c in FETCH_SIZE WRITE_SIZE; do
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o p -- python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-1000000} ${PROF_ARGS} > "$O/pmc_$c.log" 2>&1 )
      rc=$?; echo "pmc $c rc=$rc"; tail -1 "$O/pmc_$c.log"; [ $rc -eq 0 ] || exit $rc
    done
    python3 "$R/tools/pmc_group_summary.py" "$O/pmc_FETCH_SIZE" "$O/pmc_WRITE_SIZE" "$O/pmc_group.json" "$PMC_WORKLOAD" "$PMC_GROUP" "$PMC_ROUNDS" "$PMC_KERNELS" ;;
  cli)
    IFS=';' read -ra CASES <<< "${CLI_CASES:-10000000 Imp3D push-sum}"
    for c in "${CASES[@]}"; do
      for i in $(seq ${REPS:-3}); do
        for v in ${VARIANTS}; do
          out=$(timeout -k 10 120 "$R/cop5615-gossip_protocol_amd/lib_$v/gossip" $c < /dev/null) || { echo "cli $v $c failed"; exit 1; }
          echo "$v $c: $(echo "$out" | grep -E 'Convergence Time|Rounds' | tr '\n' ' ')" | tee -a "$O/cli.txt"
        done
      done
    done ;;
  ktrun_bench)  # kernel trace of bench.py with the arguments in $2
    kt kt python3 "$R/bench.py" $2 ;;
  ktrun)  # kernel trace of one prof_run.py run ($ROUNDS rounds, default: to convergence)
    kt kt python3 "$R/tools/prof_run.py" --rounds ${ROUNDS:-1000000} ${PROF_ARGS} ;;
  pmcphase)  # counters per kernel by phase of one run: one rocprofv3 --pmc run per pass of $PMC_PASSES
    # (";"-separated counter lists) over "python3 $PMC_CMD --series ..." -> tools/pmc_phase_table.py
    # ($PMC_RK round kernel, $PMC_WORLD, $PMC_WARMUP rounds before the run, $PMC_KERNELS comma list)
    IFS=';' read -ra PS <<< "$PMC_PASSES"
    i=0
    for c in "${PS[@]}"; do
      i=$((i+1))
      ser=""; [ $i -eq 1 ] && ser="--series $O/series.json"
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL ${PMC_TIMEOUT:-150} rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$i" -o p -- python3 $R/$PMC_CMD $ser > "$O/pmc_$i.log" 2>&1 )
      rc=$?; echo "pmc pass $i ($c) rc=$rc"; tail -1 "$O/pmc_$i.log"; [ $rc -eq 0 ] || exit $rc
    done
    python3 "$R/tools/pmc_phase_table.py" "$O/series.json" "$PMC_RK" "${PMC_WORLD:-1}" "${PMC_WARMUP:-0}" "$PMC_KERNELS" "$O/table.md" $(for j in $(seq $i); do echo "$O/pmc_$j"; done) > /dev/null && cat "$O/table.md" | head -${PMC_LINES:-40}
    [ "${PMC_DROP:-1}" = 1 ] && for j in $(seq $i); do find "$O/pmc_$j" -name '*counter_collection.csv' -size +20M -delete; done ;;
  loopab)
    for v in ${VARIANTS}; do
      GP_LIB=lib_$v kt "kt_$v" python3 "$R/tools/shard_loopback_prof.py" ${LOOP_ARGS} || exit $?
    done ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
