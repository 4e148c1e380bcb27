# A/B repeat: contiguous >= 1 GiB allocations at 1e9 actors (30 rounds each, alternating).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/contig2; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  for v in base contig; do
    GP_LIB=lib_$v timeout -k 10 300 python3 tools/prof_run.py --n 1000000000 --rounds 30 2>/dev/null | sed "s/^/$v: /" >> $O/runs.txt
    rc=$?; [ $rc -eq 0 ] || exit $rc
  done
done
sort $O/runs.txt
