# Refresh of this round's measurements on the final kernels: GPU suite, C3 bench line (CPU
# baseline) + kernel trace, C4 PMC (active-round means), C5 one-GPU line.
set -o pipefail
TEST_TIMEOUT=800 bash tools/gpu.sh tests || exit $?
OUT=c3 bash tools/gpu.sh bench || exit $?
OUT=c4pmc ROUNDS=75 PROF_ARGS="--n 100000000 --topology full --algorithm gossip" PMC_EXTRA="TCC_EA0_ATOMIC_sum,TCC_EA0_WRREQ_sum" bash tools/gpu.sh pmc || exit $?
mkdir -p gpurun_out/c5
timeout -k 10 400 python3 bench.py --workload c5 --steps 2 > gpurun_out/c5/bench.json 2> gpurun_out/c5/bench.err
rc=$?; echo "c5 rc=$rc"; cat gpurun_out/c5/bench.json; exit $rc
