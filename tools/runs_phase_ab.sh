# Kernel traces of a loopback shard run per variant library (lib_<v>), split by phase
# (tools/loop_phase_kernels.py), the trace itself dropped (too big to travel back).
#   VARIANTS="a b" LOOP_ARGS="--world 8 --n 100000000" RK=k_ps_quiet_x bash tools/runs_phase_ab.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-phase_ab}"; mkdir -p "$O"
for v in $VARIANTS; do
  ( cd /tmp && export TMPDIR=/tmp && GP_LIB=lib_$v timeout -k 10 ${KT_TIMEOUT:-300} rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$v" -o kt -- python3 "$R/tools/shard_loopback_prof.py" $LOOP_ARGS --series "$O/series_$v.json" > "$O/kt_$v.log" 2>&1 ) || { echo "$v failed"; tail -3 "$O/kt_$v.log"; exit 1; }
  python3 "$R/tools/loop_phase_kernels.py" "$O/kt_$v/kt_kernel_trace.csv" "$O/series_$v.json" ${RK:-k_ps_quiet_x} > "$O/phase_$v.txt" || exit 1
  rm -f "$O/kt_$v/kt_kernel_trace.csv"
  echo "== $v"; cat "$O/phase_$v.txt"
done
