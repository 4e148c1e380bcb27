#!/bin/bash
# Round 6: C3 bench line per variant library (C3_VARIANTS, default "cur pre"), interleaved, 3 each, then the
# one-GPU fingerprint tests on the working tree's library.
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_c3_ab}"; rm -rf "$O"; mkdir -p "$O"
for i in 1 2 3; do
  for v in ${C3_VARIANTS:-cur pre}; do
    GP_LIB=lib_$v timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > "$O/c3_${v}_$i.json" 2> "$O/c3_${v}_$i.err"; rc=$?
    echo "c3 $v $i rc=$rc $(python3 -c "import json;d=json.load(open('$O/c3_${v}_$i.json'));print(round(d['ms_per_step'],2), d['roofline']['avg_kernel_ms'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_fingerprints.py tests/test_gpu_parity.py -x -q --timeout 600 \
    --timeout-method thread -k "${TESTS_K:-not shard and not group}" > "$O/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 "$O/tests.log"; exit $rc
fi
