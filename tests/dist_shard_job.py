"""One rank of a multi-process shard job, launched by torch.distributed.run (one process per GPU):

    python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P tests/dist_shard_job.py --backend nccl --n-arg 100000000 --topology Imp3D \\
        --algorithm push-sum --cap 50 --out DIR

Each rank owns the node range gp_partition gives it, runs the product host loop
(gossip_amd.sharded.run) with the torch.distributed transport, and writes its part of the final
state, the completion trace and its status to DIR/rank<r>.npz; the test that launched the job
joins the parts in rank order and compares them with the single-process reference.

--backend nccl: HipShard on cuda:LOCAL_RANK, all_to_all_single over RCCL (xGMI between GPUs);
--backend gloo: the CPU oracle's shard engine (oracle.OracleShard, test infrastructure only) over
gloo, so the same script and host loop are exercised on a machine without GPUs.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cop5615-gossip_protocol_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=["nccl", "gloo"], required=True)
    ap.add_argument("--n-arg", type=int, required=True)
    ap.add_argument("--topology", required=True)
    ap.add_argument("--algorithm", required=True)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cap", type=int, default=0, help="round cap (0: to convergence)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    from gossip_amd import sharded
    from helpers import state_arrays

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    cap = a.cap or 1 << 40
    if a.backend == "nccl":
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        eng = sharded.HipShard(a.n_arg, a.topology, a.algorithm, rank=rank, world=world, seed=a.seed, device=local)
    else:
        import oracle

        dist.init_process_group("gloo")
        bounds = sharded.partition(a.n_arg, a.topology, world)
        eng = oracle.OracleShard(a.n_arg, a.topology, a.algorithm, rank=rank, world=world, bounds=bounds, seed=a.seed)
    try:
        st = sharded.run(eng, sharded.TorchTransport(), max_rounds=cap)
        arrays = state_arrays(eng, a.algorithm)
        np.savez(os.path.join(a.out, f"rank{rank}.npz"), trace=np.asarray(eng.read_trace(), np.int64),
                 status=np.array([int(st.round), int(st.completed), int(st.converged)], np.int64),
                 lo=np.int64(eng.lo), hi=np.int64(eng.hi), **arrays)
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
