# Interleaved A/B of variant libraries (lib_<v>) on loopback shard runs: the per-phase hipEvent times.
#   VARIANTS="a b" REPS=2 CASES="--world 8 --n 1000000000 --rounds 24 --no-pieces;--world 8 --n 100000000" bash tools/runs_ab_r5.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-ab}"; mkdir -p "$O"
IFS=';' read -ra CS <<< "$CASES"
for rep in $(seq ${REPS:-2}); do
  ci=0
  for c in "${CS[@]}"; do
    ci=$((ci+1))
    for v in $VARIANTS; do
      GP_LIB=lib_$v timeout -k 10 ${AB_TIMEOUT:-200} python3 tools/shard_loopback_prof.py $c --series "$O/c${ci}_${v}_${rep}.json" > "$O/c${ci}_${v}_${rep}.log" 2>&1 || { echo "$v case $ci failed"; tail -3 "$O/c${ci}_${v}_${rep}.log"; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/c${ci}_${v}_${rep}.json'))
ks=('compute_ms_dense','unpack_ms_dense','kernels_ms_dense','kernels_ms_tail','rank_round_ms_dense','host_ms')
print('case $ci $v rep $rep', {k: (round(d[k],4) if d.get(k) is not None else None) for k in ks})"
    done
  done
done
