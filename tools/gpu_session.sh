# k_gs_full4 filter threshold A/B: the done-bitmap filter from the first report (f1), from 1/64,
# 1/16, 1/4 (f4 = default) of the actors reported.
set -o pipefail
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
for i in 1 2 3; do
  for v in f4 f1 f16 f64; do
    for w in "100000000 full gossip" "10000000 full gossip"; do
      timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> $O/cli.txt || exit $?
    done
  done
done
sort $O/cli.txt
