set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r4bb"; mkdir -p "$O"
for v in $VARIANTS; do
  ( cd /tmp && export TMPDIR=/tmp && GP_LIB=lib_$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$v" -o kt -- python3 "$R/tools/shard_loopback_prof.py" --world 8 --n 100000000 --topology full --algorithm gossip --series "$O/$v.json" > "$O/$v.txt" 2>&1 ) || { echo "loop $v failed"; tail -5 "$O/$v.txt"; exit 1; }
  python3 tools/loop_phase_kernels.py "$O/kt_$v/kt_kernel_trace.csv" "$O/$v.json" k_gs_full4x 8 > "$O/${v}_phase.txt"
  echo "== $v"; grep -E "send_bytes_rank0|plan_changes" "$O/$v.txt"; grep -A3 "^mid\|^whole\|^tail" "$O/${v}_phase.txt" | grep -v "__amd"
  rm -rf "$O/kt_$v"
done
