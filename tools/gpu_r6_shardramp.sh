#!/bin/bash
# Round 6: full gossip's ramp on lists on shards (k_gs_sparse_x): the shard gossip parity tests and the
# C4 fingerprints, then C4 x 8 loopback series with the lists (lib) and without (lib_noshr), interleaved.
R=$(pwd); O="$R/gpurun_out/${OUT:-r6_shardramp}"; rm -rf "$O"; mkdir -p "$O"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_fingerprints.py tests/test_gpu_parity.py -x -v --timeout 600 \
    --timeout-method thread -k "${TESTS_K:-gossip or C4 or ramp}" > "$O/tests.log" 2>&1; rc=$?
  echo "tests rc=$rc"; tail -6 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SKIP_LOOP" ]; then exit 0; fi
for i in 1 2; do
  for lib in lib lib_noshr; do
    GP_LIB=$lib timeout -k 10 300 python -u tools/shard_loopback_prof.py --world 8 --n 100000000 --topology full \
      --algorithm gossip --rank0-events --series "$O/series_${lib}_$i.json" > "$O/loop_${lib}_$i.txt" 2>&1; rc=$?
    echo "$lib $i rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$O/loop_${lib}_$i.txt"; exit $rc; }
  done
done
