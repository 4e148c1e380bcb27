"""The driver's SCALE path on a ONE-GPU box: one process per rank under torch.distributed.run with
HipShard on the GPU, bit for bit against the oracle's fingerprints (tests/golden/fingerprints.json)
or the CPU oracle itself.

  * world 1, backend nccl: `bench.py --gpus N`'s exact stack (torch.distributed.run, an RCCL process
    group, HipShard, TorchTransport.exchange) on one device; a single rank exchanges nothing;
  * world 2 and 3 on the same device, host-staged (tests/dist_shard_job.py StagedTransport: device ->
    host -> gloo all_to_all_single -> host -> device; RCCL refuses two ranks on one device): HipShard's
    rounds in pieces with per-piece plans, the two receive buffers alternating across rounds (a
    push-sum round reads the previous round's remote messages where they arrived),
    the activity tiers with restore points, and full gossip's per-round plans.

The ranks are fresh child processes spawned by pytest (run_dist_job), as the driver spawns them.
What this cannot show on one GPU: RCCL moving bytes between two devices, and the asynchronous
per-piece all-to-all overlapping the next piece (test_gpu_multidevice.py, on >= 2 GPUs).
Reference: the per-round delivery replaces the mailbox tells of program.fs:116,127,143.
"""
import numpy as np
import pytest

from helpers import compare_digests, digest_arrays, fingerprints, join_parts, run_dist_job, unpack_trace

pytestmark = pytest.mark.gpu

FP = fingerprints()
PS_KEYS = ["S", "W", "flags", "msg_dst", "msg_s", "msg_w"]
GS_KEYS = ["cnt", "flags"]


def _check_fp(fp, parts, keys):
    for p in parts:
        assert tuple(int(x) for x in p["status"]) == (fp["rounds"], fp["completed"], fp["converged"])
        np.testing.assert_array_equal(p["trace"], unpack_trace(fp["trace_z"]))
    assert int(parts[0]["lo"]) == 0 and int(parts[-1]["hi"]) == fp["actors"]
    for a, b in zip(parts, parts[1:]):
        assert int(a["hi"]) == int(b["lo"])
    compare_digests(digest_arrays(join_parts(parts, keys)), fp["digests"])


@pytest.mark.parametrize("name", ["C5w_imp3d_100m_pushsum_w50", "C3_imp3d_10m_pushsum"])
def test_torchrun_nccl_world1_vs_fingerprint(name):
    """The SCALE launch form at world 1: torch.distributed.run + nccl + HipShard + TorchTransport."""
    fp = FP[name]
    parts = run_dist_job(1, "nccl", fp["n_arg"], fp["topology"], fp["algorithm"], fp["seed"], fp["cap"], 600)
    _check_fp(fp, parts, PS_KEYS)


def test_staged_world2_c5w_pieces_vs_fingerprint():
    """C5w over two processes on one GPU: 50M actors per rank >= 2^25, so every round runs in 4
    pieces (the library's own choice, as on the driver's node) with two receive buffers."""
    fp = FP["C5w_imp3d_100m_pushsum_w50"]
    parts = run_dist_job(2, "staged", fp["n_arg"], fp["topology"], fp["algorithm"], fp["seed"], fp["cap"], 900)
    _check_fp(fp, parts, PS_KEYS)
    for p in parts:
        assert int(p["piece_rounds"]) == fp["rounds"]  # every round in pieces
        assert int(p["recv_buffers"]) == 2
        assert int(p["bytes_sent"]) > 0


def _oracle_run(n, topo, algo, seed, cap):
    import oracle

    sim = oracle.OracleSim(n, topo, algo, seed=seed)
    st = sim.step(cap, threads=8)
    from helpers import state_arrays

    out = (st, np.asarray(sim.read_trace(), np.int64), state_arrays(sim, algo))
    sim.close()
    return out


@pytest.mark.parametrize("world,n,topo,algo,seed,opts", [
    (2, 300000, "Imp3D", "push-sum", 5, ["--force-pieces", "--tight-tiers"]),
    (3, 200000, "Imp3D", "push-sum", 2, ["--force-pieces"]),
    (3, 1000000, "full", "gossip", 4, ["--tight-tiers"]),
])
def test_staged_vs_oracle(world, n, topo, algo, seed, opts):
    """Host-staged ranks on one GPU to convergence against the CPU oracle: forced pieces, tight tiers
    (reduced chunks that overflow and replay from a restore point), full gossip's per-round plans."""
    cap = 5000
    parts = run_dist_job(world, "staged", n, topo, algo, seed, cap, 900, extra=opts)
    st, trace, want = _oracle_run(n, topo, algo, seed, cap)
    assert bool(st.converged)
    for p in parts:
        assert tuple(int(x) for x in p["status"]) == (int(st.round), int(st.completed), int(st.converged))
        np.testing.assert_array_equal(p["trace"], trace)
    keys = GS_KEYS if algo == "gossip" else PS_KEYS
    got = join_parts(parts, keys)
    for k in keys:
        a, b = got[k], want[k]
        if a.dtype == np.float64:
            a, b = a.view(np.uint64), b.view(np.uint64)
        np.testing.assert_array_equal(a, b, err_msg=k)
    if "--force-pieces" in opts:
        assert all(int(p["piece_rounds"]) > 0 and int(p["recv_buffers"]) == 2 for p in parts)
    if "--tight-tiers" in opts:
        assert sum(int(p["plan_changes"]) for p in parts) > 0
        assert len({int(p["restores"]) for p in parts}) == 1  # every rank replays together
