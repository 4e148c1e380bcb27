# A/B of kernel variants (GP_LIB=lib_<name>) on the headline workload: 300 rounds each, twice
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
for pass in 1 2; do
  for lib in ${LIBS}; do
    echo -n "$lib: "; GP_LIB=$lib timeout -k 5 60 python3 tools/prof_run.py --rounds ${ROUNDS:-300} ${PROF_ARGS} | tail -1 || exit 1
  done
done
