# Tail-walk A/B session (one gpurun call): the fingerprint and quiet-wave parity tests on each
# candidate library of $CANDS, then CLI convergence times of $VARIANTS (tools/gpu.sh cli).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
for v in ${CANDS:-acc}; do
  GP_LIB=lib_$v timeout -k 10 300 python -u -m pytest tests/test_gpu_fingerprints.py tests/test_gpu_parity.py -k "single_gpu or quiet" -x -q --timeout 200 --timeout-method thread > gpurun_out/par_$v.log 2>&1; rc=$?; echo "parity $v rc=$rc"; tail -2 gpurun_out/par_$v.log; [ $rc -eq 0 ] || exit $rc
done
OUT=${OUT:-cli_tail} VARIANTS="${VARIANTS:-old acc}" CLI_CASES="${CLI_CASES:-10000000 Imp3D push-sum;100000000 Imp3D push-sum;1000000 Imp3D push-sum}" REPS=${REPS:-3} bash tools/gpu.sh cli
