#!/bin/bash
# A/B of per-wave completion counts in the small-graph round kernels (lib_wa) against per-block (lib_base), after the GPU suite.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
P=$GRAFT_REPO_ROOT/cop5615-gossip_protocol_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for cfg in "100000 3D push-sum" "300000 3D push-sum" "100000 line push-sum" "100000 Imp3D push-sum" "100000 line gossip" "100000 2D gossip"; do
  for i in 1 2 3; do
    for v in base wa; do
      t=$(timeout -k 10 120 $P/lib_$v/gossip $cfg | grep "Convergence Time") || exit 1
      echo "$v $cfg: $t" | tee -a $O/ab_wa.txt
    done
  done
done
