# Round-3 closing measurements (one gpurun call, every GPU step under its own time limit, stops
# at the first failure): the GPU test suite, the default bench line (with the CPU baseline) and
# its rocprofv3 kernel summary, the whole-run PMC and kernel trace of C3, C4, the C5 window and
# C5 to convergence, and 8 loopback shards of C5.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
O="$R/gpurun_out/final"; rm -rf "$O"; mkdir -p "$O"
run() { local n=$1; shift; timeout -k 10 ${T:-420} python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err"; rc=$?; echo "$n rc=$rc"; head -c 400 "$O/$n.json"; echo; return $rc; }
TEST_TIMEOUT=600 OUT=final_tests bash tools/gpu.sh tests &&
run c3 &&
OUT=final_c3kt bash tools/gpu.sh ktrun_bench "--no-cpu-baseline" &&
OUT=final_c3pmc bash tools/gpu.sh pmcrun &&
OUT=final_c3run bash tools/gpu.sh ktrun &&
run c4 --workload c4 --no-cpu-baseline &&
run c5w --workload c5 --no-cpu-baseline &&
run c5conv --workload c5 --window 0 --steps 1 --warmup 0 --no-cpu-baseline &&
OUT=final_loop LOOP_ARGS="--n 1000000000 --world 8 --rounds 24" KT_LINES=8 bash tools/gpu.sh loop
