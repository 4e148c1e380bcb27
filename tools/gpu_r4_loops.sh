# Round 4: loopback profiles (8 shards on one GPU) of 100M Imp3D push-sum and 100M full gossip to
# convergence, each under a kernel trace with the per-phase kernel breakdown.  Optional first step:
# the shard GPU tests ($TESTS=1).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/${OUT:-r4c}"; mkdir -p "$O"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_fingerprints.py tests/test_gpu_group.py -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?; tail -4 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
loop() {  # name n topology algorithm round_kernel
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$1" -o kt -- python3 "$R/tools/shard_loopback_prof.py" --world 8 --n $2 --topology $3 --algorithm $4 --series "$O/$1.json" > "$O/$1.txt" 2>&1 ) || { echo "loop $1 failed"; tail -20 "$O/$1.txt"; return 1; }
  grep -E '"rank0_|"rank_round|tail_over|send_bytes|"rounds' "$O/$1.txt"
  python3 tools/loop_phase_kernels.py "$O/kt_$1/kt_kernel_trace.csv" "$O/$1.json" "$5" 8 > "$O/$1_phase_kernels.txt" && cat "$O/$1_phase_kernels.txt"
  rm -rf "$O/kt_$1"
}
for c in ${LOOPS:-ps gs}; do
  case $c in
    ps) loop loop100m_ps 100000000 Imp3D push-sum "k_ps_quiet_x" || exit 1 ;;
    gs) loop loop100m_gs 100000000 full gossip "${GS_KERNEL:-k_gs_full4x}" || exit 1 ;;
  esac
done
