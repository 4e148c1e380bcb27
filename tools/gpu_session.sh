#!/bin/bash
# A/B of the small-graph push-sum kernel loading lpos at level 1 (lib_lp) against the previous tree (lib_base), after the GPU suite.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
P=$GRAFT_REPO_ROOT/cop5615-gossip_protocol_amd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for cfg in "100000 Imp3D push-sum" "1000 Imp3D push-sum" "200000 Imp3D push-sum" "500000 Imp3D push-sum"; do
  for i in 1 2 3 4 5; do
    for v in base lp; do
      t=$(timeout -k 10 120 $P/lib_$v/gossip $cfg | grep "Convergence Time") || exit 1
      echo "$v $cfg: $t" | tee -a $O/ab_lp.txt
    done
  done
done
