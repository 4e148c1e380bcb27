# Headline bench line (single-GPU engine) + the shard engine through torchrun/RCCL at N=1.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 12 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --engine shard --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_shard1.json 2> gpurun_out/bench_shard1.err
rc=$?; echo "shard bench rc=$rc"; tail -c 2000 gpurun_out/bench_shard1.json; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench_shard1.err; exit $rc; }
