#!/bin/bash
# Round 6: 100M / 8 Imp3D push-sum loopback to convergence under a kernel trace: the rank kernels per
# phase and the tail in buckets of 100 rounds (where a tail rank-round's time goes), for each variant
# library in KT_VARIANTS (default: the in-tree lib only).
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_tail_kt}"; rm -rf "$O"; mkdir -p "$O"
for v in ${KT_VARIANTS:-lib}; do
  ( cd /tmp && export TMPDIR=/tmp && GP_LIB=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$v" -o kt -- python3 "$R/tools/shard_loopback_prof.py" --world 8 --n 100000000 --series "$O/kt_$v.json" > "$O/kt_$v.txt" 2>&1 ) || { echo "kt $v failed"; tail -5 "$O/kt_$v.txt"; exit 1; }
  python3 tools/loop_phase_kernels.py "$O/kt_$v/kt_kernel_trace.csv" "$O/kt_$v.json" k_ps_quiet_x 8 8 100 > "$O/${v}_phase.txt"
  echo "== $v"; grep -v "__amd_rocclr_fill" "$O/${v}_phase.txt"
  rm -rf "$O/kt_$v"
done
