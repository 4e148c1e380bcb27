R="$GRAFT_REPO_ROOT"; cd "$R"; timeout -k 5 120 ./tools/microbench/membench
