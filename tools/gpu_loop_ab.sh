# Loopback A/B (8 shards on one GPU, rocprofv3 kernel trace, per-phase breakdown) of the variant
# libraries in $VARIANTS (lib_<name>/, GP_LIB) on one workload: $N $TOPO $ALGO, round kernel $RK.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/${OUT:-loopab}"; mkdir -p "$O"
i=0
for v in $VARIANTS; do
  i=$((i + 1)); tag="${v}_$i"
  ( cd /tmp && export TMPDIR=/tmp && GP_LIB=lib_$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$tag" -o kt -- python3 "$R/tools/shard_loopback_prof.py" --world 8 --n ${N:-100000000} --topology ${TOPO:-Imp3D} --algorithm ${ALGO:-push-sum} --series "$O/$tag.json" > "$O/$tag.txt" 2>&1 ) || { echo "loop $v failed"; tail -5 "$O/$tag.txt"; exit 1; }
  python3 tools/loop_phase_kernels.py "$O/kt_$tag/kt_kernel_trace.csv" "$O/$tag.json" ${RK:-k_ps_quiet_x} 8 > "$O/${tag}_phase.txt"
  echo "== $tag"; grep -E "rank0_ms_dense|rank0_ms_tail|rank0_tail_over" "$O/$tag.txt"; grep -E "^(dense|tail|whole)" "$O/${tag}_phase.txt"
  rm -rf "$O/kt_$tag"
done
