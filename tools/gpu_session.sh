# Full gossip: four actors per lane + done bitmap (lib/, this tree) against the per-actor kernel
# with the gstate sender filter (lib_base): GPU suite, CLI times, C4 bench + kernel trace.
set -o pipefail
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
for i in 1 2 3; do
  for v in base ""; do
    d=cop5615-gossip_protocol_amd/lib${v:+_$v}
    for w in "100000000 full gossip" "10000000 full gossip" "1000 full gossip"; do
      timeout -k 10 120 $d/gossip $w | grep Convergence | sed "s/^/${v:-new} $w: /" >> $O/cli.txt || exit $?
    done
  done
done
sort $O/cli.txt
OUT=c4 BENCH_ARGS="--workload c4 --steps 3" bash tools/gpu.sh bench
