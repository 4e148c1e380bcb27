#!/bin/bash
# A/B of the tail batch rule in gp_step (lib_tb: 32-round batches once 31/32 of the nodes have reported) against GP_TAIL_BATCH=0 (lib_base), after the GPU suite.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
P=$GRAFT_REPO_ROOT/cop5615-gossip_protocol_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for cfg in "100000 Imp3D push-sum" "1000 Imp3D push-sum" "100000 Imp3D gossip" "1000 full gossip" "100000 line push-sum" "10000000 Imp3D push-sum" "100000000 full gossip"; do
  for i in 1 2 3 4; do
    for v in base tb; do
      t=$(timeout -k 10 120 $P/lib_$v/gossip $cfg | grep "Convergence Time") || exit 1
      echo "$v $cfg: $t" | tee -a $O/ab_tb.txt
    done
  done
done
