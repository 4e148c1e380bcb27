"""One rank of a multi-process shard job, launched by torch.distributed.run (one process per GPU):

    python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P tests/dist_shard_job.py --backend nccl --n-arg 100000000 --topology Imp3D \\
        --algorithm push-sum --cap 50 --out DIR

Each rank owns the node range gp_partition gives it, runs the product host loop
(gossip_amd.sharded.run) with a torch.distributed transport, and writes its part of the final
state, the completion trace, its status and its shard counters to DIR/rank<r>.npz; the test that
launched the job joins the parts in rank order and compares them with the single-process reference.

--backend nccl: HipShard on cuda:LOCAL_RANK, TorchTransport (all_to_all_single over RCCL: xGMI
    between GPUs; asynchronous per piece when the round runs in pieces) — the driver's SCALE path;
--backend staged: HipShard on cuda:--device for EVERY rank (several processes on one GPU: RCCL
    refuses two ranks on one device), and StagedTransport below: the rank's device send buffer is
    copied to the host, moved by gloo's all_to_all_single, and copied into the device receive buffer.
    Test-only; it exercises HipShard's pieces, activity tiers, restore points and the two alternating
    receive buffers across processes on a one-GPU box;
--backend gloo: the CPU oracle's shard engine (oracle.OracleShard, test infrastructure only) over
    gloo, so the same script and host loop are exercised on a machine without GPUs.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cop5615-gossip_protocol_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


class StagedTransport:
    """TorchTransport's interface (exchange / exchange_piece / join) over host memory: device -> host,
    gloo all_to_all_single, host -> device, all ordered on the engine's stream (torch's current
    stream).  Synchronous per piece, so it checks the piece layout, the per-piece plans and the
    receive-buffer alternation, not the overlap (TorchTransport's job on a multi-GPU node)."""

    def __init__(self):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.calls = 0
        self.bytes = 0

    def _a2a(self, recv, send, rs, ss):
        torch = self.torch
        send_h = send.cpu()  # waits for the kernels that wrote it (same stream)
        recv_h = torch.empty(int(sum(rs)), dtype=torch.uint8)
        self.dist.all_to_all_single(recv_h, send_h, list(rs), list(ss))
        recv.copy_(recv_h)  # enqueued before the engine's next kernels on the same stream
        self.calls += 1
        self.bytes += int(sum(ss))

    def exchange(self, eng):
        ns, nr = sum(eng.send_splits), sum(eng.recv_splits)
        self._a2a(eng.recv_buf[:nr], eng.send_buf[:ns], eng.recv_splits, eng.send_splits)

    def exchange_piece(self, eng, i):
        ss, rs, so, ro = eng.piece_plans[i]
        self._a2a(eng.recv_buf[ro:ro + sum(rs)], eng.send_buf[so:so + sum(ss)], rs, ss)
        return None

    def join(self, works):
        pass


class PieceCounter:
    """Wraps a HipShard: counts the rounds run in pieces and the distinct receive buffers delivered
    (the host loop calls these methods; everything else passes through)."""

    def __init__(self, eng):
        self.e = eng
        self.piece_rounds = 0
        self.recv_ptrs = set()

    def __getattr__(self, k):
        return getattr(self.e, k)

    def round_piece(self, i):
        if i == 0:
            self.piece_rounds += 1
        return self.e.round_piece(i)

    def deliver(self):
        self.recv_ptrs.add(int(self.e.recv_buf.data_ptr()))
        return self.e.deliver()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=["nccl", "gloo", "staged"], required=True)
    ap.add_argument("--n-arg", type=int, required=True)
    ap.add_argument("--topology", required=True)
    ap.add_argument("--algorithm", required=True)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cap", type=int, default=0, help="round cap (0: to convergence)")
    ap.add_argument("--device", type=int, default=0, help="staged: the device every rank uses")
    ap.add_argument("--force-pieces", action="store_true", help="HipShard: 4 pieces at any size")
    ap.add_argument("--tight-tiers", action="store_true", help="HipShard: tiers without headroom (restores)")
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
    opts = dict(rank=rank, world=world, seed=a.seed, force_pieces=a.force_pieces, tight_tiers=a.tight_tiers)
    if a.backend == "nccl":
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        eng = sharded.HipShard(a.n_arg, a.topology, a.algorithm, device=local, **opts)
        transport = sharded.TorchTransport()
    elif a.backend == "staged":
        torch.cuda.set_device(a.device)
        dist.init_process_group("gloo")
        eng = sharded.HipShard(a.n_arg, a.topology, a.algorithm, device=a.device, **opts)
        transport = StagedTransport()
    else:
        import oracle

        dist.init_process_group("gloo")
        bounds = sharded.partition(a.n_arg, a.topology, world)
        eng = oracle.OracleShard(a.n_arg, a.topology, a.algorithm, rank=rank, world=world, bounds=bounds, seed=a.seed)
        transport = sharded.TorchTransport()
    try:
        counted = PieceCounter(eng) if a.backend != "gloo" else eng
        st = sharded.run(counted, transport, max_rounds=cap)
        arrays = state_arrays(eng, a.algorithm)
        extra = {}
        if a.backend != "gloo":
            s = eng.shard_stats()
            extra = dict(piece_rounds=np.int64(counted.piece_rounds), recv_buffers=np.int64(len(counted.recv_ptrs)),
                         plan_changes=np.int64(s["plan_changes"]), restores=np.int64(s["restores"]),
                         bytes_sent=np.int64(s["bytes_sent"]))
        np.savez(os.path.join(a.out, f"rank{rank}.npz"), trace=np.asarray(eng.read_trace(), np.int64),
                 status=np.array([int(st.round), int(st.completed), int(st.converged)], np.int64),
                 lo=np.int64(eng.lo), hi=np.int64(eng.hi), **arrays, **extra)
        dist.barrier()
    finally:
        if hasattr(eng, "close"):
            eng.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
