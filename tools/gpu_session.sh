# A/B against the round-1 engine (lib_old, built from git 489ee51): convergence time of the
# headline run through each build's own CLI (3 runs each); parity of the new default build.
for v in old base nt16 fuse; do
  for i in 1 2 3; do timeout -k 10 120 cop5615-gossip_protocol_amd/lib_$v/gossip 10000000 Imp3D push-sum > gpurun_out/cli_$v.$i.txt 2>&1 || exit $?; done
  echo "$v $(grep -h Convergence gpurun_out/cli_$v.*.txt | tr '\n' ' ')"
done
GP_LIB=lib_fuse timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fingerprint or golden" > gpurun_out/tests_fuse.log 2>&1; echo "fuse tests rc=$?"; tail -1 gpurun_out/tests_fuse.log
bash tools/gpu.sh tests
