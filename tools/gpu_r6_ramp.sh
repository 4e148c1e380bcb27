#!/bin/bash
# Round 6: full gossip's ramp on lists (k_gs_sparse): C4 CLI A/B (interleaved), then the gossip parity tests.
R=$(pwd); O="$R/gpurun_out/${OUT:-r6_ramp}"; rm -rf "$O"; mkdir -p "$O"
P=cop5615-gossip_protocol_amd
for i in 1 2 3; do
  for lib in lib ${VARIANTS}; do
    timeout -k 10 120 ./$P/$lib/gossip 100000000 full gossip > "$O/c4_${lib}_$i.txt" 2>&1
    rc=$?; echo "$lib rc=$rc $(grep -E 'Convergence' $O/c4_${lib}_$i.txt)"; [ $rc -eq 0 ] || { tail -5 "$O/c4_${lib}_$i.txt"; exit $rc; }
  done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fingerprints.py -x -v --timeout 600 \
  --timeout-method thread -k "ramp or full or gossip or C4" > "$O/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -8 "$O/tests.log"; exit $rc
