# A/B of the grid cap (GP_GRID_PER_CU): convergence time of the headline run (10M Imp3D
# push-sum) and of C4 (100M full gossip) through each build's CLI.
set -o pipefail
V="g4 g6 g8 g16 g32"
for i in 1 2 3; do
  for v in $V; do
    timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip 10000000 Imp3D push-sum > gpurun_out/cli_$v.$i.txt 2>&1 || exit $?
  done
done
for v in $V; do
  timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip 100000000 full gossip > gpurun_out/cli4_$v.txt 2>&1 || exit $?
done
for v in $V; do echo "$v $(grep -h Convergence gpurun_out/cli_$v.*.txt | sed 's/Convergence Time: //' | tr '\n' ' ') | c4 $(grep -h Convergence gpurun_out/cli4_$v.txt)"; done
