# Round 4: the whole GPU suite, then the loopback profiles (tools/gpu_r4_loops.sh) and the small-Imp3D
# A/B of the slot messages (lib_noslot vs lib_slot, CLI convergence times, interleaved).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/${OUT:-r4f}"; mkdir -p "$O"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1; rc=$?; tail -4 "$O/tests.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3 4 5; do
  for v in noslot slot; do
    for c in "100000 Imp3D push-sum" "1000000 Imp3D push-sum"; do
      out=$(timeout -k 10 60 "$R/cop5615-gossip_protocol_amd/lib_$v/gossip" $c < /dev/null) || exit 1
      echo "$v $c: $(echo "$out" | grep -E 'Convergence Time|Rounds' | tr '\n' ' ')" >> "$O/cli_small.txt"
    done
  done
done
python3 tools/cli_table.py "$O/cli_small.txt" | tee "$O/cli_small_table.txt"
OUT=${OUT:-r4f} bash tools/gpu_r4_loops.sh
