# cost attribution of the push-sum round kernel (GP_ABLATE bits; timings only)
R="$GRAFT_REPO_ROOT"; cd "$R"
for ab in 0 1 2 4 8 16 18 19 23 31; do
  echo -n "ablate=$ab: "; GP_ABLATE=$ab timeout -k 5 60 python3 tools/prof_run.py --rounds 200 ${PROF_ARGS} | tail -1 || exit 1
done
