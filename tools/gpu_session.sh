# A/B of the full-gossip sender-side done filter (lib_gsf = this tree) against lib_base (previous
# commit): GPU suite on this tree, then CLI convergence times and a kernel trace of C4.
set -o pipefail
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
for i in 1 2 3; do
  for v in base gsf; do
    for w in "100000000 full gossip" "10000000 full gossip" "1000 full gossip"; do
      timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> $O/cli.txt || exit $?
    done
  done
done
sort $O/cli.txt
OUT=c4 BENCH_ARGS="--workload c4 --steps 3" bash tools/gpu.sh bench
