"""GPU parity of the single-process multi-GPU engine behind the C ABI (gp_config.num_gpus):
one graph split into node-range shards, each with its own stream, exchanged inside the
library.  On a one-GPU box the shards share the device (GP_FLAG_ONE_DEVICE: device copies on
one stream); with GP_FLAG_GROUP a single shard runs under an RCCL communicator of its device.
Bit-exact against the CPU oracle and the single-GPU engine."""
import numpy as np
import pytest

import oracle
from gossip_amd import GossipError, Simulator
from helpers import bits, check_same

pytestmark = pytest.mark.gpu

CASES = [
    (1000, "Imp3D", "push-sum", 1),
    (200, "3D", "push-sum", 3),
    (200, "line", "push-sum", 2),
    (1000, "full", "gossip", 1),
    (1000, "Imp3D", "gossip", 3),
    (64, "2D", "gossip", 2),
]


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[2]}-{c[1]}-{c[0]}")
def test_group_one_device_vs_oracle(case, world):
    n, topo, algo, seed = case
    try:
        gpu = Simulator(n, topo, algo, seed=seed, num_gpus=world, one_device=True)
    except GossipError as e:
        if "cannot be split" in str(e):
            pytest.skip(str(e))
        raise
    cpu = oracle.OracleSim(n, topo, algo, seed=seed)
    for chunk in (1, 6, 3000):  # batch boundaries and gossip's one-round count lag
        gs = gpu.step(chunk)
        cs = cpu.step(chunk)
        assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
        check_same(gpu, cpu, algo)
        if cs.converged:
            break
    if algo == "push-sum":
        assert gs.sum_w == pytest.approx(cs.sum_w, rel=1e-12)
    assert (gpu.nodes, gpu.actors, gpu.leader) == (cpu.layout.nodes, cpu.layout.actors, cpu.layout.leader)
    for v in (0, gpu.actors // 2, gpu.actors - 1):
        np.testing.assert_array_equal(gpu.neighbors(v), cpu.neighbors(v))
    gpu.close()
    cpu.close()


def test_group_reads_span_shards():
    gpu = Simulator(100000, "Imp3D", "push-sum", seed=4, num_gpus=4, one_device=True)
    ref = Simulator(100000, "Imp3D", "push-sum", seed=4)
    gpu.step(40)
    ref.step(40)
    first, count = 10000, 70000  # crosses three shard boundaries
    a = gpu.read_pushsum(first, count)
    b = ref.read_pushsum(first, count)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(bits(x) if x.dtype == np.float64 else x, bits(y) if y.dtype == np.float64 else y)
    gpu.reset()
    ref.reset()
    gs, rs = gpu.step(), ref.step()
    assert gs.converged and (gs.round, gs.completed) == (rs.round, rs.completed)
    check_same(gpu, ref, "push-sum")


@pytest.mark.parametrize("n,topo,algo", [(100000, "Imp3D", "push-sum"), (100000, "full", "gossip"),
                                         (20000, "line", "push-sum")])
def test_group_rccl_one_rank_vs_single_gpu(n, topo, algo):
    """GP_FLAG_GROUP at num_gpus = 1: the shard engine under an RCCL communicator of this
    device (ncclCommInitAll, grouped send/recv with no peers) against gp_step, bit for bit."""
    gpu = Simulator(n, topo, algo, seed=9, group=True)
    ref = Simulator(n, topo, algo, seed=9)
    gs, rs = gpu.step(3000), ref.step(3000)
    assert (gs.round, gs.completed, gs.converged) == (rs.round, rs.completed, rs.converged)
    check_same(gpu, ref, algo)


def test_group_needs_devices():
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU present")
    with pytest.raises(GossipError, match="device 1 not present"):
        Simulator(1000, "Imp3D", "push-sum", num_gpus=2)
    with pytest.raises(GossipError, match="GP_EINVAL"):
        Simulator(1000, "Imp3D", "push-sum", num_gpus=17, one_device=True)
