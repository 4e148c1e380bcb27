# Quiet-wave skipping with its fields in a union (kernel arguments back to 344 bytes) vs HEAD
# (lib_base): full GPU suite, CLI times incl. the launch-latency-bound small graphs.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/act4; rm -rf $O; mkdir -p $O
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
for i in 1 2 3; do
  for v in base new; do
    for w in "10000000 Imp3D push-sum" "100000000 Imp3D push-sum" "100000 3D push-sum" "100000 line push-sum" "1000 full gossip"; do
      timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> $O/cli.txt || exit $?
    done
  done
done
sort $O/cli.txt
