# Round-3 A/B session (one gpurun call): GPU tests on the default build, then CLI convergence
# times of the variant libraries and a whole-run kernel trace of the default build.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TEST_TIMEOUT=900 bash tools/gpu.sh tests &&
OUT=cli VARIANTS="${VARIANTS:-old q7 q6 seg64 seg8 seg32}" CLI_CASES="${CLI_CASES:-10000000 Imp3D push-sum;100000000 Imp3D push-sum;2000000 Imp3D push-sum}" bash tools/gpu.sh cli &&
OUT=c3 BENCH_ARGS="--no-cpu-baseline --steps 3" bash tools/gpu.sh bench
