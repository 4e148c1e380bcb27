"""Multi-device parity: the multi-GPU paths across PHYSICAL GPUs, bit for bit against the CPU
oracle's full-size fingerprints (tests/golden/fingerprints.json).  They switch on when at least two
GPUs are visible (the driver's 8-GPU node) and skip with the reason on a one-GPU box, where the same
decomposition is covered on one device (test_gpu_fingerprints.py: loopback shards and the library
group with GP_FLAG_ONE_DEVICE).

  * the library's own multi-GPU engine (gp_config.num_gpus = min(8, devices): ncclCommInitAll and
    grouped ncclSend / ncclRecv between the GPUs of this process) on C3 and C4;
  * one process per GPU (torch.distributed.run, backend nccl: HipShard + TorchTransport, RCCL
    all_to_all_single over xGMI) on the C5 window, launched as freshly spawned child processes
    that touch no GPU before torch.distributed.run starts them.

The CPU analogue of the second job (the same script, gloo + the oracle's shard engine) runs in
test_sharded_gloo.py::test_dist_shard_job_script_gloo.
"""
import numpy as np
import pytest

from helpers import compare_digests, digest_arrays, fingerprints, join_parts, run_dist_job, unpack_trace

pytestmark = pytest.mark.gpu

FP = fingerprints()


def _devices():
    import torch

    return torch.cuda.device_count()  # does not initialise the GPU on this image


def _need(n):
    d = _devices()
    if d < n:
        pytest.skip(f"{d} GPU(s) visible: the cross-device RCCL path needs {n} (covered on one device by "
                    f"test_gpu_fingerprints.py)")
    return d


def _check(fp, status, trace, arrays):
    assert tuple(int(x) for x in status) == (fp["rounds"], fp["completed"], fp["converged"])
    np.testing.assert_array_equal(trace, unpack_trace(fp["trace_z"]))
    compare_digests(digest_arrays(arrays), fp["digests"])


@pytest.mark.parametrize("name", ["C3_imp3d_10m_pushsum", "C4_full_100m_gossip"])
def test_group_rccl_devices_vs_fingerprint(name):
    from gossip_amd import Simulator
    from helpers import state_arrays

    n = min(8, _need(2))
    fp = FP[name]
    sim = Simulator(fp["n_arg"], fp["topology"], fp["algorithm"], seed=fp["seed"], num_gpus=n)
    st = sim.step(fp["cap"] or 1 << 40)
    _check(fp, (st.round, st.completed, st.converged), sim.read_trace(), state_arrays(sim, fp["algorithm"]))
    assert (int(sim.layout.nodes), int(sim.layout.actors)) == (fp["nodes"], fp["actors"])
    sim.close()


def test_torchrun_nccl_shards_vs_fingerprint():
    """C5w (`100000000 Imp3D push-sum`, 50 rounds) over 2 processes, one GPU each, RCCL between them."""
    _need(2)
    fp = FP["C5w_imp3d_100m_pushsum_w50"]
    parts = run_dist_job(2, "nccl", fp["n_arg"], fp["topology"], fp["algorithm"], fp["seed"], fp["cap"], 900)
    for p in parts:
        np.testing.assert_array_equal(p["trace"], unpack_trace(fp["trace_z"]))
    assert [int(p["lo"]) for p in parts][0] == 0 and int(parts[-1]["hi"]) == fp["actors"]
    arrays = join_parts(parts, ["S", "W", "flags", "msg_dst", "msg_s", "msg_w"])
    _check(fp, parts[0]["status"], parts[0]["trace"], arrays)
