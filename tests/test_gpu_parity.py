"""GPU parity: the HIP engine (through the C ABI) against the committed golden vectors, the CPU
oracle on the same seeded inputs, and size-independent properties at BASELINE sizes.
Bit-exact everywhere: gossip is integer work; push-sum fp64 sums run in the same canonical
ascending-source order as the oracle (tolerance 0 ulp; north star allows 1e-10 relative)."""
import numpy as np
import pytest

import oracle
from gossip_amd import GossipError, Simulator
from helpers import bits, check_same, check_state, load_golden, manifest

pytestmark = pytest.mark.gpu

MAN = manifest()
MID = MAN["mid_rounds"]
CASES = [c["name"] for c in MAN["cases"]]


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("generic", [False, True])
def test_golden(name, generic):
    g = load_golden(name)
    topo = [k for k, v in oracle.TOPOLOGIES.items() if v == int(g["topology"])][0]
    algo = "gossip" if int(g["algo"]) == 0 else "push-sum"
    sim = Simulator(int(g["n_arg"]), topo, algo, seed=int(g["seed"]), generic=generic)
    assert (sim.nodes, sim.actors, sim.leader) == (g["nodes"], g["actors"], g["leader"])
    sim.step(MID)
    check_state(sim, g, "mid_")
    st = sim.step(int(g["fin_round"]) - MID)
    assert st.round == g["fin_round"] and st.converged == g["converged"]
    np.testing.assert_array_equal(sim.read_trace(), g["trace"])
    check_state(sim, g, "fin_")
    sim.close()


def _pair(n, topo, algo, seed, **kw):
    return Simulator(n, topo, algo, seed=seed, **kw), oracle.OracleSim(n, topo, algo, seed=seed)


@pytest.mark.parametrize("n,topo,algo,rounds", [
    (100000, "Imp3D", "push-sum", None),     # to convergence (~540 rounds)
    (100000, "3D", "push-sum", 400),
    (100000, "line", "push-sum", 300),
    (100000, "2D", "push-sum", 200),
    (20000, "full", "push-sum", None),
    (100000, "Imp3D", "gossip", None),
    (100000, "3D", "gossip", None),
    (3000, "line", "gossip", None),
    (100000, "full", "gossip", None),
    (5000, "2D", "gossip", None),
    # above 2^18 actors: the gossip grid kernel's lazy-load instantiation
    (400000, "3D", "gossip", None),
    (300000, "Imp3D", "gossip", None),
    (300000, "2D", "gossip", 300),
])
def test_vs_oracle_100k(n, topo, algo, rounds):
    gpu, cpu = _pair(n, topo, algo, seed=11)
    cap = rounds if rounds else 1 << 30
    # stop at a few intermediate rounds too, so batch boundaries are exercised
    for chunk in (1, 6, 37):
        gpu.step(chunk)
        cpu.step(chunk, threads=8)
        check_same(gpu, cpu, algo)
    gs = gpu.step(cap - 44)
    cs = cpu.step(cap - 44, threads=8)
    assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
    if rounds is None:
        assert gs.converged
    check_same(gpu, cpu, algo)
    if algo == "push-sum":
        assert gs.sum_s == pytest.approx(cs.sum_s, rel=1e-12)
        assert gs.sum_w == pytest.approx(cs.sum_w, rel=1e-12)


@pytest.mark.parametrize("n,topo", [(1, "line"), (2, "line"), (1, "full"), (2, "full"), (1, "2D"),
                                    (1, "Imp3D"), (7, "Imp3D"), (8, "Imp3D"), (26, "Imp3D"),
                                    (8, "3D"), (27, "3D")])
@pytest.mark.parametrize("algo", ["gossip", "push-sum"])
def test_edge_sizes(n, topo, algo):
    gpu, cpu = _pair(n, topo, algo, seed=3)
    for v in range(gpu.actors):
        np.testing.assert_array_equal(gpu.neighbors(v), cpu.neighbors(v))
    gs = gpu.step(3000)
    cs = cpu.step(3000)
    assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
    check_same(gpu, cpu, algo)


def test_3d_single_node_never_converges():
    """N < 8 in "3D": one node with no neighbours never reports (cap the rounds)."""
    sim = Simulator(5, "3D", "push-sum")
    st = sim.step(50)
    assert st.round == 50 and not st.converged and st.completed == 0


def test_neighbors_match_oracle():
    gpu, cpu = _pair(2000, "Imp3D", "gossip", seed=9)
    for v in list(range(0, gpu.actors, 37)) + [gpu.actors - 1, gpu.nodes - 1]:
        np.testing.assert_array_equal(gpu.neighbors(v), cpu.neighbors(v))


def test_reset_is_deterministic():
    sim = Simulator(50000, "Imp3D", "push-sum", seed=2)
    a = sim.step()
    S1, W1, f1 = sim.read_pushsum()
    t1 = sim.read_trace()
    sim.reset()
    b = sim.step()
    S2, W2, f2 = sim.read_pushsum()
    assert (a.round, a.completed) == (b.round, b.completed)
    np.testing.assert_array_equal(bits(S1), bits(S2))
    np.testing.assert_array_equal(f1, f2)
    np.testing.assert_array_equal(t1, sim.read_trace())


def test_full_gossip_1m_vs_oracle():
    gpu, cpu = _pair(1_000_000, "full", "gossip", seed=4)
    gs = gpu.step()
    cs = cpu.step(threads=16)
    assert gs.converged and (gs.round, gs.completed) == (cs.round, cs.completed)
    check_same(gpu, cpu, "gossip")


@pytest.mark.parametrize("n,seed", [(20000, 5), (300000, 6), (1_500_000, 7)])
def test_full_gossip_ramp_lists_vs_oracle(n, seed):
    """Full gossip's ramp on lists (k_gs_sparse, one GPU): steps of every length, so the host extends
    its bound on the holders at syncs inside the ramp, and the switch to k_gs_full4 (with the tally from
    2^20 actors) lands at different rounds; bit-exact against the oracle after every step."""
    gpu, cpu = _pair(n, "full", "gossip", seed)
    for chunk in (1, 1, 2, 3, 5, 8, 13, 21, 1 << 20):
        gs, cs = gpu.step(chunk), cpu.step(chunk, threads=16)
        assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
        check_same(gpu, cpu, "gossip")
        if gs.converged:
            break
    assert gs.converged
    gpu.reset()  # a second run: the lists start from the leader again
    gs = gpu.step()
    assert (gs.round, gs.completed) == (cs.round, cs.completed)
    check_same(gpu, cpu, "gossip")
    gpu.close()
    cpu.close()


def test_invalid_config_errors():
    with pytest.raises(GossipError):
        Simulator(0, "line", "gossip")
    with pytest.raises(GossipError):
        Simulator(10, "line", "gossip", term_limit=0)


def test_cli_report_and_trace(tmp_path):
    """The drop-in CLI (program.fs:19-21 argv, :51-52 report) on the GPU: banner, convergence
    report and rounds, and --trace's per-round count curve equal to the oracle's."""
    import os
    import re
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "cop5615-gossip_protocol_amd", "lib", "gossip")
    out = tmp_path / "trace.csv"
    r = subprocess.run([exe, "1000", "Imp3D", "push-sum", "--seed", "3", "--trace", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    cpu = oracle.OracleSim(1000, "Imp3D", "push-sum", seed=3)
    cs = cpu.step()
    # exactly the reference's lines (program.fs:322, :51-52) plus the round count
    assert len(lines) == 4, lines
    assert lines[0] == "Push Sum Started"
    assert lines[1] == "-" * 59
    assert re.fullmatch(r"Convergence Time: \d+\.\d{6} ms", lines[2]), lines[2]
    assert lines[3] == f"Rounds: {cs.round}"
    # --verbose adds the layout line after the banner; --gpus 1 / --mode round change nothing
    r = subprocess.run([exe, "1000", "Imp3D", "push-sum", "--seed", "3", "--verbose", "--gpus", "1", "--mode", "round"],
                       capture_output=True, text=True, timeout=60)
    v = r.stdout.splitlines()
    assert r.returncode == 0 and len(v) == 5 and v[1].startswith("actors 1001 (nodes 1000), leader ")
    assert v[0] == lines[0] and v[4] == lines[3]
    rows = np.loadtxt(out, delimiter=",", skiprows=1, dtype=np.int64).reshape(-1, 2)
    np.testing.assert_array_equal(rows[:, 0], np.arange(cs.round))
    np.testing.assert_array_equal(rows[:, 1], cpu.read_trace())
    assert rows[-1, 1] == int(cpu.layout.nodes)
    cpu.close()

def _sweep_cases(count=64, seed=2026):
    """Seeded random (n, topology, algorithm, seed, generic) draws: sizes log-uniform over
    2..200000, so grid sizes that are not cubes/squares and ragged last planes all appear."""
    rng = np.random.default_rng(seed)
    topos = sorted(oracle.TOPOLOGIES)
    out = []
    for _ in range(count):
        n = int(np.exp(rng.uniform(np.log(2), np.log(200000))))
        out.append((n, topos[rng.integers(len(topos))], ("gossip", "push-sum")[rng.integers(2)],
                    int(rng.integers(1, 1 << 30)), bool(rng.integers(2))))
    return out


@pytest.mark.parametrize("n,topo,algo,seed,generic", _sweep_cases())
def test_random_sweep(n, topo, algo, seed, generic):
    """Bit-exact against the oracle over random configurations, to convergence or 2000 rounds."""
    gpu = Simulator(n, topo, algo, seed=seed, generic=generic)
    cpu = oracle.OracleSim(n, topo, algo, seed=seed)
    gs = gpu.step(2000)
    cs = cpu.step(2000, threads=8)
    assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
    np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
    check_same(gpu, cpu, algo)
    gpu.close()


# Quiet-wave skipping (once 99% of the nodes have converged, waves of 64 actors
# that the previous round did not mark skip their round) forced on small graphs, run to
# convergence (the long tail of relayed messages is where waves go quiet), bit-exact against the
# oracle in trace and state.  The 10M C3 fingerprint covers the default size gate.
@pytest.mark.parametrize("n,topo,seed", [
    (1000, "Imp3D", 1), (20000, "Imp3D", 5), (200000, "Imp3D", 3),
    (8000, "3D", 2), (2000, "line", 4), (3000, "2D", 6),
])
def test_quiet_waves_vs_oracle(n, topo, seed):
    _quiet_vs_oracle(n, topo, seed)


def _quiet_sweep_cases(count=24, seed=4242):
    """Seeded random push-sum draws for forced quiet waves, all five topologies: line and 2D up to
    3000 nodes (their convergence time grows fastest with N), the others log-uniform to 100000."""
    rng = np.random.default_rng(seed)
    topos = sorted(oracle.TOPOLOGIES)
    out = []
    for _ in range(count):
        topo = topos[rng.integers(len(topos))]
        hi = 3000 if topo in ("line", "2D") else 100000
        out.append((int(np.exp(rng.uniform(np.log(2), np.log(hi)))), topo, int(rng.integers(1, 1 << 30))))
    return out


@pytest.mark.parametrize("n,topo,seed", _quiet_sweep_cases())
def test_quiet_waves_random_sweep(n, topo, seed):
    _quiet_vs_oracle(n, topo, seed)


def _quiet_vs_oracle(n, topo, seed):
    gpu = Simulator(n, topo, "push-sum", seed=seed, quiet_waves=True)
    cpu = oracle.OracleSim(n, topo, "push-sum", seed=seed)
    gs = gpu.step(1 << 20)
    cs = cpu.step(1 << 20, threads=8)
    assert gs.converged and (gs.round, gs.completed) == (cs.round, cs.completed)
    np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
    check_same(gpu, cpu, "push-sum")
    gpu.close()
    cpu.close()


def test_quiet_waves_default_and_reset():
    """Above 2^20 actors quiet-wave skipping is on by default (the kernel reports itself as the
    marking instantiation); a run to convergence, a reset and a second run both match the
    oracle bit for bit (the marks of the first run must not leak into the second)."""
    n = 1_200_000
    gpu = Simulator(n, "Imp3D", "push-sum", seed=2, kernel_timing=True)
    assert gpu.actors >= 1 << 20
    cpu = oracle.OracleSim(n, "Imp3D", "push-sum", seed=2)
    cs = cpu.step(1 << 20, threads=8)
    for _ in range(2):
        gs = gpu.step(1 << 20)
        assert gs.converged and (gs.round, gs.completed) == (cs.round, cs.completed)
        np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
        check_same(gpu, cpu, "push-sum")
        assert gpu.kernel_stats()["kernel"] == "k_ps_quiet<1>"
        gpu.reset()
    gpu.close()
    cpu.close()


def test_quiet_work_count_vs_oracle():
    """gp_kstats.work_per_launch of the quiet kernel (bench.py's roofline units) is the exact count
    of the actors it walks: every actor in a round without marks, else every actor of each 4-actor
    segment that holds an unconverged actor or a target of the previous round's messages (the
    marks of DESIGN.md §4), recomputed here from the oracle's per-round state."""
    n, seed, seg, pct = 20000, 7, 4, 99
    gpu = Simulator(n, "Imp3D", "push-sum", seed=seed, quiet_waves=True, kernel_timing=True)
    cpu = oracle.OracleSim(n, "Imp3D", "push-sum", seed=seed)
    gs = gpu.step(1 << 20)
    ks = gpu.kernel_stats()
    actors, thr = gpu.actors, gpu.nodes * pct // 100
    trace = gpu.read_trace()
    walked = actors  # F(0)
    cpu.step(1, threads=8)
    for r in range(1, gs.round):
        dst, _, _ = cpu.read_messages()  # sent in round r - 1
        _, _, fl = cpu.read_pushsum()    # after round r - 1
        if r >= 2 and trace[r - 2] >= thr:
            act = (fl & 16) == 0
            act[gpu.nodes:] = False  # the isolated actor has no neighbours and never updates
            act[dst[dst < actors].astype(np.int64)] = True
            marked = np.zeros((actors + seg - 1) // seg, bool)
            marked[np.nonzero(act)[0] // seg] = True
            walked += int(np.minimum(seg, actors - seg * np.nonzero(marked)[0]).sum())
        else:
            walked += actors
        cpu.step(1, threads=8)
    assert ks["work_per_launch"] * gs.round == pytest.approx(walked, rel=0, abs=0.5)
    assert ks["work_per_launch"] < actors
    gpu.close()
    cpu.close()


@pytest.mark.parametrize("n,seed", [(1000, 3), (70000, 5), (300000, 2), (1_200_000, 4)])
def test_full_gossip_tally_vs_oracle(n, seed):
    """Full gossip with the receipt tally by target bucket forced in every round from round 1
    (GP_FLAG_GOSSIP_TALLY; by default it runs from 2^20 actors after a round with many chains):
    the same trace and state as the oracle, bit for bit (receipts to done targets are counted
    there and dropped by the receiver, instead of being filtered by the sender)."""
    gpu = Simulator(n, "full", "gossip", seed=seed, gossip_tally=True)
    cpu = oracle.OracleSim(n, "full", "gossip", seed=seed)
    gs = gpu.step()
    cs = cpu.step(threads=16)
    assert gs.converged and (gs.round, gs.completed) == (cs.round, cs.completed)
    np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
    check_same(gpu, cpu, "gossip")
    gpu.reset()  # a second run after a reset: the tally's ring counters start clean
    gs2 = gpu.step()
    assert (gs2.round, gs2.completed) == (cs.round, cs.completed)
    np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
    gpu.close()
    cpu.close()


@pytest.mark.parametrize("n,seed,forced", [(1_200_000, 4, True), (10_000_000, 1, False)])
def test_full_gossip_tally_fallbacks_vs_oracle(n, seed, forced):
    """The tally's live fallbacks, which a large graph reaches only at extreme counts, forced in every
    tallied round (GP_FLAG_TALLY_FALLBACKS): the counted-batch placement (a workgroup whose receipts
    outgrow its LDS; at C4 a workgroup peaks at ~24K receipts against room for 34.8K) and the 32-bit
    escape of the 16-bit receipt words (counts >= 0xFFFF), every nonzero count through it.  C4-shaped
    runs (1.2M forced from round 1; 10M with the default tally rule), bit for bit against the oracle."""
    gpu = Simulator(n, "full", "gossip", seed=seed, gossip_tally=forced, tally_fallbacks=True)
    cpu = oracle.OracleSim(n, "full", "gossip", seed=seed)
    gs = gpu.step()
    cs = cpu.step(threads=16)
    assert gs.converged and (gs.round, gs.completed) == (cs.round, cs.completed)
    np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
    check_same(gpu, cpu, "gossip")
    assert gpu.kernel_stats()["kernel"] == "k_gs_full4+tally"  # the tally was built for this graph
    gpu.close()
    cpu.close()


# Small one-GPU line grids (line, 2D) run up to 8 rounds per launch (k_ps_tile): batches
# of every length, so that launches of 1 .. 8 rounds alternate and a step can end after any round of a
# launch; segment edges, the line's ends and tiny graphs.
TILE_CASES = [
    (1, "line", 1, None), (2, "line", 1, None), (3, "line", 2, None), (9, "2D", 3, None), (253, "line", 4, None),
    (254, "2D", 5, None), (1000, "line", 6, None), (5000, "2D", 7, None), (20000, "line", 9, 1500),
    (50000, "2D", 10, 1200), (260000, "line", 12, 600),
]


@pytest.mark.parametrize("n,topo,seed,cap", TILE_CASES)
def test_tiles_vs_oracle(n, topo, seed, cap):
    gpu, cpu = _pair(n, topo, "push-sum", seed, kernel_timing=True)
    assert gpu.kernel_stats()["kernel"] == "k_ps_tile"
    done = 0
    for chunk in (1, 2, 3, 5, 8, 13, 64, 255):
        gs, cs = gpu.step(chunk), cpu.step(chunk, threads=8)
        done += chunk
        assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
        check_same(gpu, cpu, "push-sum")
        if gs.converged:
            break
    if not gs.converged:
        rest = (cap or 1 << 30) - done
        gs, cs = gpu.step(rest), cpu.step(rest, threads=8)
        assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
        check_same(gpu, cpu, "push-sum")
    if cap is None:
        assert gs.converged
    assert gs.sum_s == pytest.approx(cs.sum_s, rel=1e-12) and gs.sum_w == pytest.approx(cs.sum_w, rel=1e-12)
    gpu.reset()  # a second run: the 9 state buffers (kTileBufs) start clean
    gs2 = gpu.step(cs.round)
    assert (gs2.round, gs2.completed) == (cs.round, cs.completed)
    check_same(gpu, cpu, "push-sum")
    gpu.close()
    cpu.close()


@pytest.mark.parametrize("topo", ["line", "2D"])
def test_tiles_vs_one_round_c2(topo):
    """C2 line / 2D to convergence (1481 rounds): up to 8 rounds per launch against one round per
    launch (GP_FLAG_ONE_ROUND, pinned by the oracle above and by the fingerprints)."""
    a = Simulator(100000, topo, "push-sum", seed=1)
    b = Simulator(100000, topo, "push-sum", seed=1, one_round=True, kernel_timing=True)
    assert b.kernel_stats()["kernel"] == "k_ps_pull<0, false>"
    sa, sb = a.step(), b.step()
    assert sa.converged and (sa.round, sa.completed) == (sb.round, sb.completed)
    check_same(a, b, "push-sum")
    a.close()
    b.close()


# Gossip on tiny graphs (generic path: "full", or any topology with GP_FLAG_GENERIC; up to 8192
# actors) runs each batch of rounds in one workgroup's LDS (k_gs_tiny): steps of
# every length, so a batch can end anywhere, including past convergence.
TINY_CASES = [
    (1, "full", 1, False), (2, "full", 2, False), (3, "full", 3, False), (10, "full", 4, False),
    (100, "full", 5, False), (1000, "full", 6, False), (3000, "full", 7, False), (4095, "full", 8, False), (8191, "full", 17, False),
    (2000, "line", 9, True), (1000, "3D", 10, True), (3000, "Imp3D", 11, True), (900, "2D", 12, True),
    # (the grid topologies take it by default at this size too)
    (3000, "line", 13, False), (2700, "3D", 14, False), (2500, "Imp3D", 15, False), (2900, "2D", 16, False),
    (3900, "2D", 18, False), (4000, "3D", 19, False),
]


@pytest.mark.parametrize("n,topo,seed,generic", TINY_CASES)
def test_tiny_gossip_vs_oracle(n, topo, seed, generic):
    gpu, cpu = _pair(n, topo, "gossip", seed, generic=generic, kernel_timing=True)
    assert gpu.kernel_stats()["kernel"] == "k_gs_tiny"
    for chunk in (1, 2, 3, 5, 8, 13, 1 << 20):
        gs, cs = gpu.step(chunk), cpu.step(chunk, threads=8)
        assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
        check_same(gpu, cpu, "gossip")
        if gs.converged:
            break
    gpu.reset()
    gs = gpu.step()
    assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
    check_same(gpu, cpu, "gossip")
    gpu.close()
    cpu.close()


@pytest.mark.parametrize("n,topo", [(3000, "line"), (2000, "3D"), (3000, "Imp3D")])
def test_tiny_gossip_grid_vs_one_round(n, topo):
    """Small grid gossip: the tiny path against the grid kernels (GP_FLAG_ONE_ROUND)."""
    a = Simulator(n, topo, "gossip", seed=2)
    b = Simulator(n, topo, "gossip", seed=2, one_round=True, kernel_timing=True)
    assert b.kernel_stats()["kernel"].startswith("k_gs_pull")
    sa, sb = a.step(), b.step()
    assert sa.converged and (sa.round, sa.completed) == (sb.round, sb.completed)
    check_same(a, b, "gossip")
    a.close()
    b.close()


def test_tiny_gossip_vs_one_round_c1():
    """C1 (1000 full gossip) to convergence, one launch per batch against one per round."""
    a = Simulator(1000, "full", "gossip", seed=1)
    b = Simulator(1000, "full", "gossip", seed=1, one_round=True, kernel_timing=True)
    assert b.kernel_stats()["kernel"] != "k_gs_tiny"
    sa, sb = a.step(), b.step()
    assert sa.converged and (sa.round, sa.completed) == (sb.round, sb.completed)
    check_same(a, b, "gossip")
    a.close()
    b.close()


# Push-sum on tiny graphs through the generic path ("full", or GP_FLAG_GENERIC; up to 2048 actors):
# a batch of rounds in one workgroup's LDS, the buckets by destination rebuilt there every round
# (k_ps_tiny).
TINY_PS_CASES = [
    (1, "full", 1, False), (2, "full", 2, False), (3, "full", 3, False), (39, "full", 4, False),
    (200, "full", 5, False), (1000, "full", 6, False), (2047, "full", 7, False),
    (1000, "Imp3D", 8, True), (1000, "3D", 9, True), (500, "line", 10, True), (900, "2D", 11, True),
    (1000, "Imp3D", 12, False), (2000, "Imp3D", 13, False),  # (Imp3D takes it by default at this size)
]


@pytest.mark.parametrize("n,topo,seed,generic", TINY_PS_CASES)
def test_tiny_pushsum_vs_oracle(n, topo, seed, generic):
    gpu, cpu = _pair(n, topo, "push-sum", seed, generic=generic, kernel_timing=True)
    assert gpu.kernel_stats()["kernel"] == "k_ps_tiny"
    for chunk in (1, 2, 3, 5, 8, 13, 1 << 20):
        gs, cs = gpu.step(chunk), cpu.step(chunk, threads=8)
        assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
        check_same(gpu, cpu, "push-sum")
        if gs.converged:
            break
    assert gs.converged
    assert gs.sum_s == pytest.approx(cs.sum_s, rel=1e-12) and gs.sum_w == pytest.approx(cs.sum_w, rel=1e-12)
    gpu.reset()
    gs = gpu.step()
    assert (gs.round, gs.completed, gs.converged) == (cs.round, cs.completed, cs.converged)
    check_same(gpu, cpu, "push-sum")
    gpu.close()
    cpu.close()


def test_tiny_pushsum_vs_one_round():
    """`1000 full push-sum` to convergence, one launch per batch against the per-round passes."""
    a = Simulator(1000, "full", "push-sum", seed=3)
    b = Simulator(1000, "full", "push-sum", seed=3, one_round=True, kernel_timing=True)
    assert b.kernel_stats()["kernel"] == "k_ps_push_emit"
    sa, sb = a.step(), b.step()
    assert sa.converged and (sa.round, sa.completed) == (sb.round, sb.completed)
    check_same(a, b, "push-sum")
    a.close()
    b.close()
