#!/bin/bash
# Round 6: C5 (1e9 Imp3D push-sum) on 8 loopback shards of one GPU to convergence, per variant library
# (C5_VARIANTS, default "cur pre": lib_cur, lib_pre): the per-round series and its phase summary.
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_c5loop}"; rm -rf "$O"; mkdir -p "$O"
for v in ${C5_VARIANTS:-cur pre}; do
  GP_LIB=lib_$v timeout -k 10 400 python -u tools/shard_loopback_prof.py --world 8 --n 1000000000 --topology Imp3D \
    --algorithm push-sum --series "$O/$v.json" > "$O/$v.txt" 2>&1; rc=$?
  echo "$v rc=$rc"; tail -c 1500 "$O/$v.txt"; echo; [ $rc -eq 0 ] || exit $rc
done
