# A/B: lpos fetched at the first load level (lib_t = this tree; t7, t8: 7 / 8 waves per SIMD) vs HEAD (lib_base);
# GPU suite on this tree.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/merge; rm -rf $O; mkdir -p $O
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
for i in 1 2 3; do
  for v in base t t7 t8; do
    for w in "10000000 Imp3D push-sum" "100000000 Imp3D push-sum" "100000 3D push-sum"; do
      timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> $O/cli.txt || exit $?
    done
  done
done
sort $O/cli.txt
