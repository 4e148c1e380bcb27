"""BASELINE config 5 at its full size on one GPU, checked through size-independent properties:
the CPU oracle cannot hold a 1e9-node run in the build container, so parity at this size rests
on the bit-exact fingerprint tests up to 1e8 nodes (test_gpu_fingerprints.py: C3 10M to
convergence, C4 100M full gossip to convergence, a 50-round window of 100M Imp3D push-sum) and
on these invariants.

  config 5: `1000000000 Imp3D push-sum` (1e9 nodes, G = 1148, 759 planes): a fixed 12-round
            window — sum(S) and sum(W) over held + in-flight messages conserved (program.fs:107-143
            only moves mass), the completion trace monotone, every estimate finite.
"""
import numpy as np
import pytest

from gossip_amd import Simulator

pytestmark = pytest.mark.gpu


def test_imp3d_1e9_pushsum_window():
    sim = Simulator(1_000_000_000, "Imp3D", "push-sum", seed=1)
    assert sim.nodes == 1_000_000_000 and sim.actors == 1_000_000_001 and sim.layout.grid == 1148
    nodes = float(sim.nodes)
    want_s = nodes * (nodes - 1.0) / 2.0
    st = sim.step(12)
    assert st.round == 12 and not st.converged
    # fp64 sums of 1e9 terms in a fixed block order: exact conservation up to summation rounding
    assert st.sum_s == pytest.approx(want_s, rel=1e-9)
    assert st.sum_w == pytest.approx(nodes, rel=1e-9)
    tr = sim.read_trace()
    assert len(tr) == 12 and (np.diff(tr) >= 0).all() and tr[-1] < sim.nodes
    # a slice in the middle and the partial last plane: finite, positive weights
    for first in (0, 500_000_000, sim.nodes - 1_000_000):
        S, W, _ = sim.read_pushsum(first, 1_000_000)
        assert np.isfinite(S).all() and (W > 0).all()
    sim.close()


def test_imp3d_1e9_pushsum_to_convergence():
    """config 5 to convergence on one GPU (program.fs:54-60: the ParentActor stops at
    count = AllNodes): every participant converged exactly once, the isolated actor `nodes` never,
    (S, W) held + in flight conserved, the trace monotone and ending at `nodes`."""
    sim = Simulator(1_000_000_000, "Imp3D", "push-sum", seed=1)
    nodes = float(sim.nodes)
    st = sim.step()
    assert st.converged and st.completed == sim.nodes, (st.round, st.completed)
    print(f"1000000000 Imp3D push-sum: {st.round} rounds, {st.device_ms:.1f} ms, "
          f"{sim.actors * st.round / (st.device_ms * 1e-3):.3e} node-updates/s", flush=True)
    assert st.sum_s == pytest.approx(nodes * (nodes - 1.0) / 2.0, rel=1e-9)
    assert st.sum_w == pytest.approx(nodes, rel=1e-9)
    tr = sim.read_trace()
    assert len(tr) == st.round and (np.diff(tr) >= 0).all() and tr[-1] == sim.nodes and tr[-2] < sim.nodes
    chunk = 100_000_000
    converged = 0
    for first in range(0, sim.actors, chunk):
        n = min(chunk, sim.actors - first)
        S, W, f = sim.read_pushsum(first, n)
        conv = (f & 16) != 0
        if first + n > sim.nodes:  # the isolated actor (program.fs:293) holds (nodes, 1)
            assert not conv[-1] and S[-1] == nodes and W[-1] == 1.0
            conv = conv[:-1]
        assert conv.all() and np.isfinite(S).all() and (W > 0).all()
        converged += int(conv.sum())
    assert converged == sim.nodes
    sim.close()
