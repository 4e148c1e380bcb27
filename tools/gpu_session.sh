# torch.distributed.run at world 1 with the shard engine (RCCL all-to-all of empty chunks):
# C3 then C5, each under its own time limit, stage marks on stderr.
set -o pipefail
mkdir -p gpurun_out/c5shard
for w in c3 c5; do
  timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 1 --engine shard --workload $w --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c5shard/$w.json 2> gpurun_out/c5shard/$w.err
  rc=$?; echo "$w rc=$rc"; grep "^\[bench" gpurun_out/c5shard/$w.err; grep "^{" gpurun_out/c5shard/$w.json | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
