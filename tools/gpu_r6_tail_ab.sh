#!/bin/bash
# Round 6: 100M / 8 Imp3D push-sum loopback to convergence, rank 0's rounds by hipEvents (the tail / dense
# ratio of VERDICT r5 item 8), variants interleaved; then the shard tests.
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_tail_ab}"; rm -rf "$O"; mkdir -p "$O"
for i in 1 2 3; do
  for v in ${TAIL_VARIANTS:-cur pre}; do
    GP_LIB=lib_$v timeout -k 10 300 python -u tools/shard_loopback_prof.py --world 8 --n 100000000 --topology Imp3D \
      --algorithm push-sum --rank0-events --series "$O/${v}_$i.json" > "$O/${v}_$i.txt" 2>&1; rc=$?
    echo "$v $i rc=$rc $(grep -E '"rank0_(ms_dense|ms_tail|tail_over_dense)"' $O/${v}_$i.txt | tr -d '\n ')"
    [ $rc -eq 0 ] || { tail -20 "$O/${v}_$i.txt"; exit $rc; }
  done
done
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_fingerprints.py -x -q --timeout 600 \
    --timeout-method thread -k "${TESTS_K:-push or quiet or pieces or C3 or C5}" > "$O/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 "$O/tests.log"; exit $rc
fi
