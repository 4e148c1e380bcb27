# Read lines (FETCH) and CLI times of the push-sum round kernel with a fully resident grid
# (6 workgroups per CU: all workgroups of an XCD sweep its span together) with and without the
# y-slab walk, against the default 16-per-CU grid (several generations of workgroups per span).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ys2; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  for v in base c6 ysc6; do
    w="10000000 Imp3D push-sum"
    timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> $O/cli.txt || exit $?
  done
done
sort $O/cli.txt
for v in c6 ysc6; do
  ( cd /tmp && export TMPDIR=/tmp && GP_LIB=lib_$v timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_$v" -o p -- python3 "$GRAFT_REPO_ROOT/tools/prof_run.py" --rounds 60 > "$O/pmc_$v.log" 2>&1 )
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$O/pmc_$v" k_ps_pull
done
