#!/bin/bash
# Round 6: C4 x 8 loopback with and without the shards' ramp lists: kernel trace per phase (the rank
# kernels' GPU time, host issue excluded), then rank 0's rounds by events behind a GPU spin (the host
# issues all 8 ranks here; the spin gives the GPU a lead, as a node's host per rank would).
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_shardramp_kt}"; rm -rf "$O"; mkdir -p "$O"
for v in lib ${KT_VARIANTS:-lib_noshr}; do
  [ -n "$SKIP_KT" ] && break
  ( cd /tmp && export TMPDIR=/tmp && GP_LIB=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$v" -o kt -- python3 "$R/tools/shard_loopback_prof.py" --world 8 --n 100000000 --topology full --algorithm gossip --series "$O/kt_$v.json" > "$O/kt_$v.txt" 2>&1 ) || { echo "kt $v failed"; tail -5 "$O/kt_$v.txt"; exit 1; }
  PER_ROUND=${PER_ROUND:-24} python3 tools/loop_phase_kernels.py "$O/kt_$v/kt_kernel_trace.csv" "$O/kt_$v.json" k_gs_sparse_x,k_gs_bins_count,k_gs_full4x 8 9 > "$O/${v}_phase.txt"
  echo "== $v"; cat "$O/${v}_phase.txt" | grep -v "__amd_rocclr_fill"
  rm -rf "$O/kt_$v"
done
if [ -n "$SKIP_SPIN" ]; then exit 0; fi
for i in 1 2; do
  for v in lib ${KT_VARIANTS:-lib_noshr}; do
    GP_LIB=$v timeout -k 10 300 python -u tools/shard_loopback_prof.py --world 8 --n 100000000 --topology full \
      --algorithm gossip --rank0-events --spin-us 1500 --series "$O/spin_${v}_$i.json" > "$O/spin_${v}_$i.txt" 2>&1; rc=$?
    echo "spin $v $i rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$O/spin_${v}_$i.txt"; exit $rc; }
  done
done
