# Round 4: the four-actors-per-lane dense round (k_ps_dense4): parity first (forced-quiet small
# graphs, the C3 / C5w fingerprints, the full-size properties), then C3 / 100M convergence times of
# the variant libraries ($VARIANTS, lib_<name>/) interleaved, then a 300-round kernel trace of each.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/${OUT:-r4e}"; mkdir -p "$O"
if [ -z "$NOTESTS" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fingerprints.py tests/test_gpu_full_size.py -x -q --timeout 300 --timeout-method thread -k "${TEST_K:-quiet or fingerprint or full_size or golden or sweep}" > "$O/tests.log" 2>&1; rc=$?; tail -4 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra CASES <<< "${CLI_CASES:-10000000 Imp3D push-sum;100000000 Imp3D push-sum}"
for c in "${CASES[@]}"; do
  for i in $(seq ${REPS:-3}); do
    for v in ${VARIANTS}; do
      out=$(timeout -k 10 120 "$R/cop5615-gossip_protocol_amd/lib_$v/gossip" $c < /dev/null) || { echo "cli $v $c failed"; exit 1; }
      echo "$v $c: $(echo "$out" | grep -E 'Convergence Time|Rounds' | tr '\n' ' ')" | tee -a "$O/cli.txt"
    done
  done
done
python3 tools/cli_table.py "$O/cli.txt" | tee "$O/cli_table.txt"
for v in ${KT_VARIANTS:-}; do
  ( cd /tmp && export TMPDIR=/tmp && GP_LIB=lib_$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/kt_$v" -o kt -- python3 "$R/tools/prof_run.py" --rounds 300 > "$O/kt_$v.log" 2>&1 ) || exit 1
  python3 tools/kt_summary.py "$O/kt_$v/kt_kernel_trace.csv" | head -4 | sed "s/^/$v /"
  rm -rf "$O/kt_$v"
done
