# FETCH_SIZE (one rocprofv3 pass each) of the round kernel under several settings; $EXPS lines as in gpu_exp.sh
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp; i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1)); envs="${line%%--*}"; args="${line#*--}"
  env $envs timeout -s KILL 90 rocprofv3 --pmc ${PMC:-FETCH_SIZE} --output-format csv -d "$R/gpurun_out/fx/$i" -o p -- python3 "$R/tools/prof_run.py" $args > "$R/gpurun_out/fx/$i.log" 2>&1 || exit 1
  echo "[$i: $envs|$args] $(python3 $R/tools/pmc_summary.py $R/gpurun_out/fx/$i k_ps_pull | tr -s ' ' | head -3)"
done <<< "$EXPS"
