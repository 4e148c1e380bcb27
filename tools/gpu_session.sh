# A/B: per-wave gate in the small-graph round kernels (lib_wg = this tree) vs HEAD (lib_base):
# full GPU suite, CLI times of the launch-latency-bound C2 graphs and the headline.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/wg; rm -rf $O; mkdir -p $O
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
for i in 1 2 3; do
  for v in base wg; do
    for w in "100000 3D push-sum" "100000 line push-sum" "100000 Imp3D push-sum" "10000000 Imp3D push-sum"; do
      timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> $O/cli.txt || exit $?
    done
  done
done
sort $O/cli.txt
