# Final measurements of the round on the final tree: smoke, default bench line (C3, CPU baseline)
# + kernel trace, C4 bench line + kernel trace, C5 one-GPU line.
set -o pipefail
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
OUT=c3 bash tools/gpu.sh bench || exit $?
OUT=c4 BENCH_ARGS="--workload c4 --steps 3" bash tools/gpu.sh bench || exit $?
mkdir -p gpurun_out/c5
timeout -k 10 400 python3 bench.py --workload c5 --steps 2 > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/c5/bench.json; exit $rc
