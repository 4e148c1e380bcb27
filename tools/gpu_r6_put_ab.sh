#!/bin/bash
# Round 6: shard entry puts through an LDS peer table (put_t) vs the kernel arguments indexed per lane:
# the shard tests and fingerprints, then loopback A/B (lib_cur vs lib_pre): 100M / 8 Imp3D push-sum to
# convergence and C5 / 8 for 24 all-sending rounds (kernel trace, per-phase split).
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_put_ab}"; rm -rf "$O"; mkdir -p "$O"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_fingerprints.py -x -q --timeout 600 \
    --timeout-method thread > "$O/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do
  for v in ${PUT_VARIANTS:-cur pre}; do
    for w in ${PUT_WORK:-100000000:0 1000000000:24}; do
      n=${w%%:*}; rounds=${w#*:}; tag="${v}_${n}_$i"; ra=""; [ "$rounds" != 0 ] && ra="--rounds $rounds"
      ( cd /tmp && export TMPDIR=/tmp && GP_LIB=lib_$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$tag" -o kt -- python3 "$R/tools/shard_loopback_prof.py" --world 8 --n $n --topology Imp3D --algorithm push-sum $ra --series "$O/$tag.json" > "$O/$tag.txt" 2>&1 ) || { echo "loop $tag failed"; tail -5 "$O/$tag.txt"; exit 1; }
      python3 tools/loop_phase_kernels.py "$O/kt_$tag/kt_kernel_trace.csv" "$O/$tag.json" k_ps_quiet_x 8 > "$O/${tag}_phase.txt"
      echo "== $tag"; grep -A4 -E "^(dense|tail)" "$O/${tag}_phase.txt" | grep -E "^(dense|tail)|scatter|unpack|quiet"
      rm -rf "$O/kt_$tag"
    done
  done
done
