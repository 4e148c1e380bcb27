# Round 4: (1) kernel trace of 8 loopback shards of 100M Imp3D push-sum to convergence with the
# per-round series; (2) whole-run PMC of C4 (100M full gossip: k_gs_full4 + the tally passes) and a
# C4 bench line whose roofline.traffic comes from it (+ its kernel trace).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r4b"; mkdir -p "$O"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/kt" -o kt -- python3 "$R/tools/shard_loopback_prof.py" --world 8 --n 100000000 --series "$O/loop100m.json" > "$O/loop100m.txt" 2>&1 ) || { echo "loop failed"; tail -20 "$O/loop100m.txt"; exit 1; }
tail -32 "$O/loop100m.txt"
python3 tools/loop_phase_kernels.py "$O/kt/kt_kernel_trace.csv" "$O/loop100m.json" "k_ps_quiet<2>" 8 > "$O/phase_kernels.txt" && cat "$O/phase_kernels.txt"
rm -rf "$O/kt"
PMC_WORKLOAD="100000000 full gossip" PMC_GROUP="k_gs_full4+tally" PMC_ROUNDS=69 \
  PMC_KERNELS="k_gs_full4,k_scan_reduce,k_scan_top,k_scan_apply,k_gs_tally_scatter_lds,k_gs_tally_count" \
  PROF_ARGS="--n 100000000 --topology full --algorithm gossip" OUT=r4b_c4pmc bash tools/gpu.sh pmcgroup || exit 1
cp profiles/pmc_traffic.json "$O/pmc_traffic.json"
timeout -k 10 240 python3 bench.py --workload c4 --steps 5 --warmup 1 > "$O/c4_bench.json" 2> "$O/c4_bench.err" || { tail "$O/c4_bench.err"; exit 1; }
cat "$O/c4_bench.json"
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/c4kt" -o kt -- python3 "$R/bench.py" --workload c4 --steps 5 --warmup 1 --no-cpu-baseline > "$O/c4kt.log" 2>&1 ) || exit 1
python3 tools/kt_summary.py "$O/c4kt/kt_kernel_trace.csv" > "$O/c4kt_summary.txt"; head -12 "$O/c4kt_summary.txt"
rm -f "$O/c4kt/kt_kernel_trace.csv"
