# Timing experiments: each line of $EXPS is "ENV=.. ENV=.. -- prof_run args"; prints prof_run's summary.
R="$GRAFT_REPO_ROOT"; cd "$R"
while IFS= read -r line; do
  [ -z "$line" ] && continue
  envs="${line%%--*}"; args="${line#*--}"
  echo -n "[$envs|$args] "
  env $envs timeout -k 5 60 python3 tools/prof_run.py $args | tail -1 || exit 1
done <<< "$EXPS"
