# A/B of the per-workgroup contiguous-run walk (GP_WALK) against the strided node-range walk:
# headline convergence time through each build's CLI, C4 too, and read requests (PMC).
set -o pipefail
V="base walk walkg6 walkg32"
for i in 1 2 3; do
  for v in $V; do
    timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip 10000000 Imp3D push-sum > gpurun_out/cli_$v.$i.txt 2>&1 || exit $?
  done
done
for v in $V; do timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip 100000000 full gossip > gpurun_out/cli4_$v.txt 2>&1 || exit $?; done
for v in $V; do echo "$v $(grep -h Convergence gpurun_out/cli_$v.*.txt | sed 's/Convergence Time: //' | tr '\n' ' ') | c4 $(grep -h Convergence gpurun_out/cli4_$v.txt)"; done
for v in base walk walkg6; do
  GP_LIB=lib_$v OUT=wk_$v ROUNDS=60 PMC_EXTRA="TCC_EA0_RDREQ_sum,TCC_HIT_sum,TCC_MISS_sum" bash tools/gpu.sh pmc > gpurun_out/wk_$v.txt 2>&1 || exit $?
  grep -E "k_ps_pull" gpurun_out/wk_$v/summary.txt | grep -E "RDREQ|HIT|MISS" | sed "s/^/$v /"
done
