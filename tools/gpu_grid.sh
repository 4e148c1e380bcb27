R="$GRAFT_REPO_ROOT"; cd "$R"
for gsz in ${GRIDS:-4096 38832 80000}; do
  echo -n "grid=$gsz: "; GP_GRID=$gsz timeout -k 5 60 python3 tools/prof_run.py --rounds 300 ${PROF_ARGS} | tail -1 || exit 1
done
