# A/B of the z-march walk's planes per work item (GP_ZM_LEN; zm = planner's choice, 29 at
# 10M) against the node-range walk (base): headline convergence time through each build's CLI
# and the round kernel's EA read requests (PMC, 60 rounds).
set -o pipefail
V="base zm zm15 zm8 zm4"
for i in 1 2 3; do
  for v in $V; do
    timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip 10000000 Imp3D push-sum > gpurun_out/cli_$v.$i.txt 2>&1 || exit $?
  done
done
for v in $V; do echo "$v $(grep -h Convergence gpurun_out/cli_$v.*.txt | sed 's/Convergence Time: //' | tr '\n' ' ')"; done
for v in $V; do
  GP_LIB=lib_$v OUT=zl_$v ROUNDS=60 PMC_EXTRA="TCC_EA0_RDREQ_sum,TCC_HIT_sum,TCC_MISS_sum" bash tools/gpu.sh pmc > gpurun_out/zl_$v.txt 2>&1 || exit $?
  grep "k_ps_pull" gpurun_out/zl_$v/summary.txt | grep -E "RDREQ|HIT" | sed "s/^/$v /"
done
