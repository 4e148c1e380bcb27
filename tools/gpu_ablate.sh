# cost attribution of the push-sum round kernel (GP_ABLATE bits; timings only) + SQ counters
R="$GRAFT_REPO_ROOT"; cd "$R"
export GP_GRID=${GP_GRID:-16384}
for ab in 0 1 4 8 16 17 21 29; do
  echo -n "ablate=$ab: "; GP_ABLATE=$ab timeout -k 5 60 python3 tools/prof_run.py --rounds 200 ${PROF_ARGS} | tail -1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$R/gpurun_out/sq2/p1" -o p -- python3 "$R/tools/prof_run.py" --rounds 40 > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/sq2/p2" -o p -- python3 "$R/tools/prof_run.py" --rounds 40 > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/sq2/p3" -o p -- python3 "$R/tools/prof_run.py" --rounds 40 > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$R/gpurun_out/sq2/p4" -o p -- python3 "$R/tools/prof_run.py" --rounds 40 > /dev/null 2>&1
