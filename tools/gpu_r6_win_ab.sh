#!/bin/bash
# Round 6: the tail walk reading marks a dword per lane (256-segment windows) vs HEAD: 100M / 8 loopback
# tail / dense by hipEvents (tools/gpu_r6_tail_ab.sh), then the C3 bench line per variant, interleaved.
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/${OUT:-r6_win_ab}"; mkdir -p "$O"
SKIP_TESTS=1 OUT=${OUT:-r6_win_ab}/tail bash tools/gpu_r6_tail_ab.sh || exit $?
for i in 1 2; do
  for v in ${TAIL_VARIANTS:-cur pre}; do
    GP_LIB=lib_$v timeout -k 10 300 python -u bench.py --steps 5 --no-cpu-baseline > "$O/c3_${v}_$i.json" 2> "$O/c3_${v}_$i.err"; rc=$?
    echo "c3 $v $i rc=$rc $(python3 -c "import json;d=json.load(open('$O/c3_${v}_$i.json'));print(round(d['ms_per_step'],2), d['roofline']['avg_kernel_ms'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
