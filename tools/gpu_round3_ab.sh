set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/mb
timeout -k 10 60 rocprofv3 -L > gpurun_out/mb/counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 60 ./tools/microbench/persist > gpurun_out/mb/persist.txt 2>&1 && cat gpurun_out/mb/persist.txt &&
timeout -k 10 60 ./tools/microbench/gatherpol > gpurun_out/mb/gatherpol.txt 2>&1 && cat gpurun_out/mb/gatherpol.txt &&
OUT=cli VARIANTS="base g6 s96 s96g7 s80w8 s96w7" CLI_CASES="10000000 Imp3D push-sum;100000000 Imp3D push-sum" bash tools/gpu.sh cli &&
OUT=ab ROUNDS=300 VARIANTS="base g6 s96 s96g7 s80w8 s96w7" KT_LINES=1 bash tools/gpu.sh ab
