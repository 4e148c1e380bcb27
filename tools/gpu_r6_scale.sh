#!/bin/bash
# Round 6: the driver's SCALE path on one GPU.  Run on the GPU box from the repo root:
#   gpurun --timeout 1200 -- 'bash tools/gpu_r6_scale.sh'
R=$(pwd); O="$R/gpurun_out/${OUT:-r6_scale}"; rm -rf "$O"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_dist_onebox.py -x -v --timeout 600 --timeout-method thread \
  > "$O/dist_tests.log" 2>&1; rc=$?; echo "dist tests rc=$rc"; tail -15 "$O/dist_tests.log"; [ $rc -eq 0 ] || exit $rc
for n in 2 4; do
  timeout -k 10 400 python -u bench.py --gpus $n --one-device --steps 3 --warmup 1 > "$O/bench_g${n}_onedev.json" 2> "$O/bench_g${n}_onedev.err"
  rc=$?; echo "bench g$n rc=$rc"; tail -3 "$O/bench_g${n}_onedev.err"; [ $rc -eq 0 ] || exit $rc
done
