# A/B: grid cap (workgroups per CU) of the round kernels with the current push-sum kernel
# (7 resident workgroups per CU): 7 (all resident), 14, 16 (default = base), 28, 64.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/cap; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  for v in base c7 c14 c28 c64; do
    for w in "10000000 Imp3D push-sum" "100000000 Imp3D push-sum" "100000000 full gossip"; do
      timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> $O/cli.txt || exit $?
    done
  done
done
sort $O/cli.txt
