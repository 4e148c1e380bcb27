# A/B of the shard round kernels at 8 loopback shards on one GPU (GP_LIB variants), kernel trace
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/ab
for lib in ${LIBS:-lib}; do
  GP_LIB=$lib timeout -k 10 150 python3 tools/shard_loopback_prof.py ${ARGS} || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ab/kt" -o kt -- python3 "$R/tools/shard_loopback_prof.py" ${ARGS} > "$R/gpurun_out/ab/kt.log" 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/kt_summary.py" "$R/gpurun_out/ab/kt/kt_kernel_trace.csv" > "$R/gpurun_out/ab/kt_summary.txt"
head -10 "$R/gpurun_out/ab/kt_summary.txt"
