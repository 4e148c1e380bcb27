#!/bin/bash
# A/B of the gossip grid kernel's early level-1 loads on small graphs (lib_gse) against the previous tree (lib_base), after the GPU suite.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
P=$GRAFT_REPO_ROOT/cop5615-gossip_protocol_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for cfg in "100000 line gossip" "200000 2D gossip" "1000000 Imp3D gossip" "400000 3D gossip"; do
  for i in 1 2 3; do
    for v in base gse; do
      t=$(timeout -k 10 120 $P/lib_$v/gossip $cfg | grep "Convergence Time") || exit 1
      echo "$v $cfg: $t" | tee -a $O/ab_gse2.txt
    done
  done
done
