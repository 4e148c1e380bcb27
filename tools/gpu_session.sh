# A/B of the z-column walk with register reuse (GP_ZCOL) against the node-range walk: headline
# convergence time through each build's CLI, read requests (PMC), and parity of the z-column
# build (fingerprints, golden vectors, shards).
set -o pipefail
V="base zc zc5 zc8"
for i in 1 2 3; do
  for v in $V; do
    timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip 10000000 Imp3D push-sum > gpurun_out/cli_$v.$i.txt 2>&1 || exit $?
  done
done
for v in $V; do echo "$v $(grep -h Convergence gpurun_out/cli_$v.*.txt | sed 's/Convergence Time: //' | tr '\n' ' ')"; done
for v in base zc; do
  GP_LIB=lib_$v OUT=zcr_$v ROUNDS=60 PMC_EXTRA="TCC_EA0_RDREQ_sum,TCC_HIT_sum,TCC_MISS_sum" bash tools/gpu.sh pmc > gpurun_out/zcr_$v.txt 2>&1 || exit $?
  grep -E "k_ps_(pull|zcol)" gpurun_out/zcr_$v/summary.txt | grep -E "RDREQ|FETCH|WRITE" | sed "s/^/$v /"
done
GP_LIB=lib_zc timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fingerprint or golden or sharded or group" > gpurun_out/tests_zc.log 2>&1; rc=$?; echo "zc tests rc=$rc"; tail -2 gpurun_out/tests_zc.log; exit $rc
