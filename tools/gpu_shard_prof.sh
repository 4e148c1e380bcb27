# Shard engine at N=1 (RCCL all-to-all to itself): bench line + rocprofv3 kernel trace, to
# attribute the per-round cost of the exchange (link scatter, pack, RCCL, unpack).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/sp
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 200 python3 bench.py --engine shard --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sp/bench.json 2> gpurun_out/sp/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 1200 gpurun_out/sp/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/sp/kt" -o kt -- python3 "$R/bench.py" --engine shard --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/sp/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/kt_summary.py" "$R/gpurun_out/sp/kt/kt_kernel_trace.csv" > "$R/gpurun_out/sp/kt_summary.txt"
head -12 "$R/gpurun_out/sp/kt_summary.txt"
