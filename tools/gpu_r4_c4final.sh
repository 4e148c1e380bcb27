# Round 4, final C4 evidence: whole-run PMC of the round bracket (k_gs_full4 + the tally passes), then
# the C4 bench line (its roofline.traffic from that PMC) and its kernel trace.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/${OUT:-r4_c4final}"; mkdir -p "$O"
PMC_WORKLOAD="100000000 full gossip" PMC_GROUP="k_gs_full4+tally" PMC_ROUNDS=69 \
  PMC_KERNELS="${PMC_KERNELS:-k_gs_full4,k_tally_rows,k_gs_tally_scatter_lds,k_gs_tally_count}" \
  PROF_ARGS="--n 100000000 --topology full --algorithm gossip" OUT=${OUT:-r4_c4final}_pmc bash tools/gpu.sh pmcgroup || exit 1
cp "$R/gpurun_out/${OUT:-r4_c4final}_pmc/pmc_group.json" "$O/pmc_group.json"
timeout -k 10 240 python3 bench.py --workload c4 --steps 5 --warmup 1 > "$O/c4_bench.json" 2> "$O/c4_bench.err" || { tail "$O/c4_bench.err"; exit 1; }
cat "$O/c4_bench.json"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c4kt" -o kt -- python3 "$R/bench.py" --workload c4 --steps 5 --warmup 1 --no-cpu-baseline > "$O/c4kt.log" 2>&1 ) || exit 1
python3 tools/kt_summary.py "$O/c4kt/kt_kernel_trace.csv" > "$O/c4kt_summary.txt"; head -8 "$O/c4kt_summary.txt"
rm -f "$O/c4kt/kt_kernel_trace.csv"
