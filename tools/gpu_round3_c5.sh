# Round-3 measurement session: C5 to convergence on one GPU (bench line + kernel trace), the C5
# 50-round window, C4, and the default bench line (with the CPU baseline).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/r3meas"; rm -rf "$O"; mkdir -p "$O"
run() { local n=$1; shift; timeout -k 10 ${T:-420} python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err"; rc=$?; echo "$n rc=$rc"; cat "$O/$n.json"; return $rc; }
run c5conv --workload c5 --window 0 --steps 1 --warmup 0 --no-cpu-baseline &&
OUT=r3meas_c5kt KT_TIMEOUT=420 bash tools/gpu.sh ktrun_bench "--workload c5 --window 0 --steps 1 --warmup 0 --no-cpu-baseline" &&
run c5w --workload c5 --no-cpu-baseline &&
run c4 --workload c4 --no-cpu-baseline &&
run c3 
