# A/B of the wave-level gate overlapped with the first actor's loads (current tree, lib/) against
# the barrier gate (lib_base, previous commit): C3, C2 line / 3D, C5w-sized Imp3D 100k; then the
# GPU suite on the current tree.
set -o pipefail
for i in 1 2 3; do
  for v in base new; do
    d=cop5615-gossip_protocol_amd/lib_$v; [ $v = new ] && d=cop5615-gossip_protocol_amd/lib
    for w in "10000000 Imp3D push-sum" "100000 line push-sum" "100000 3D push-sum" "100000 Imp3D push-sum"; do
      timeout -k 10 120 $d/gossip $w | grep Convergence | sed "s/^/$v $w: /" >> gpurun_out/gate_ab.txt || exit $?
    done
  done
done
sort gpurun_out/gate_ab.txt
TEST_TIMEOUT=800 bash tools/gpu.sh tests
