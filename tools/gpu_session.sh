# Final check of the round on the committed tree: GPU suite, smoke, default bench line + trace.
set -o pipefail
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
OUT=c3 bash tools/gpu.sh bench
