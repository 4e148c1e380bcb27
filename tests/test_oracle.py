"""CPU oracle pinned against Random123 KATs, SURVEY App. B sizes and the independent
Python restatement's committed golden vectors (tests/golden/)."""
import json
import os

import numpy as np
import pytest

import oracle
import pyref

GOLD = os.path.join(os.path.dirname(__file__), "golden")
with open(os.path.join(GOLD, "manifest.json")) as _f:
    MANIFEST = json.load(_f)
CASES = [c["name"] for c in MANIFEST["cases"]]
MID = MANIFEST["mid_rounds"]

KATS = [  # Random123 kat_vectors: philox4x32_10
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_philox_kat(ctr, key, want):
    assert tuple(int(x) for x in oracle.philox(ctr, key)) == want
    got = pyref.philox(*ctr, *key)
    assert tuple(int(x) for x in got) == want


# SURVEY App. B (program.fs:26-31, :268) and the 2D rule (:228-229)
APP_B = [(20, 8, 2), (200, 125, 6), (1000, 1000, 10), (2000, 1728, 13), (100000, 97336, 50),
         (1000000, 1000000, 109), (10000000, 9938375, 239), (100000000, 99897344, 524),
         (1000000000, 1000000000, 1148), (5831, 5832, 19)]


@pytest.mark.parametrize("n,nodes,g", APP_B)
def test_imp3d_sizes(n, nodes, g):
    for topo in ("Imp3D", "3D"):
        assert oracle.sizes(n, topo) == (nodes, nodes + 1, g)


def test_other_sizes():
    assert oracle.sizes(1000, "line") == (1000, 1001, 0)
    assert oracle.sizes(1000, "full") == (1000, 1001, 0)
    assert oracle.sizes(100000, "2D") == (100489, 100490, 317)
    assert oracle.sizes(488, "2D") == (529, 530, 23)
    with pytest.raises(ValueError):
        oracle.sizes(0, "line")


def test_neighbour_order_imp3d():
    """program.fs:295-311: x-1, x+1, y-1, y+1, z-1, z+1, then ONE random link in [0, nodes-2]."""
    sim = oracle.OracleSim(200, "Imp3D", "gossip", seed=7)
    nodes, G = sim.layout.nodes, sim.layout.grid
    assert (nodes, G) == (125, 6)
    ref = pyref.neighbours(200, pyref.IMP3D, 7)
    for v in range(sim.actors):
        assert list(sim.neighbors(v)) == ref[v]
    # interior node of the 6x6 slab: 6 grid neighbours + link
    v = 1 * 36 + 1 * 6 + 1
    nb = list(sim.neighbors(v))
    assert nb[:6] == [v - 1, v + 1, v - 6, v + 6, v - 36, v + 36] and len(nb) == 7
    assert all(0 <= sim.neighbors(u)[-1] <= nodes - 2 for u in range(nodes))
    assert sim.degree(nodes) == 0  # isolated actor (program.fs:293)
    assert sim.layout.participants == nodes


def test_neighbour_order_line_full_2d():
    s = oracle.OracleSim(5, "line", "gossip")
    assert [list(s.neighbors(v)) for v in range(6)] == [[1], [0, 2], [1, 3], [2, 4], [3, 5], [4]]
    f = oracle.OracleSim(4, "full", "gossip")
    assert list(f.neighbors(2)) == [0, 1, 3, 4]
    d = oracle.OracleSim(3, "2D", "gossip")  # g = 2, nodes = 4, 5 actors: a line (Q8)
    assert [list(d.neighbors(v)) for v in range(5)] == [[1], [0, 2], [1, 3], [2, 4], [3]]


from helpers import check_state as _check_state, load_golden as _load  # noqa: E402


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("threads", [0, 4])
def test_oracle_matches_golden(name, threads):
    g = _load(name)
    sim = oracle.OracleSim(int(g["n_arg"]), int(g["topology"]), int(g["algo"]), seed=int(g["seed"]))
    assert (sim.layout.nodes, sim.layout.actors, sim.layout.grid, sim.layout.leader) == (
        g["nodes"], g["actors"], g["grid"], g["leader"])
    sim.step(MID, threads=threads)
    _check_state(sim, g, "mid_")
    st = sim.step(int(g["fin_round"]) - MID, threads=threads)
    assert st.round == g["fin_round"] and st.converged == g["converged"]
    np.testing.assert_array_equal(sim.read_trace(), g["trace"])
    _check_state(sim, g, "fin_")


@pytest.mark.parametrize("topo", ["Imp3D", "line", "full", "3D"])
def test_pushsum_conservation(topo):
    sim = oracle.OracleSim(300, topo, "push-sum", seed=5)
    part = [v for v in range(sim.actors) if sim.degree(v) > 0]
    want_s, want_w = float(sum(part)), float(len(part))
    for _ in range(6):
        st = sim.step(25)
        assert abs(st.sum_s - want_s) <= 1e-12 * want_s
        assert abs(st.sum_w - want_w) <= 1e-12 * want_w


def test_gossip_invariants():
    sim = oracle.OracleSim(500, "Imp3D", "gossip", seed=3)
    prev_cnt = np.zeros(sim.actors, np.uint32)
    prev_done = np.zeros(sim.actors, bool)
    while not sim.status.converged:
        sim.step(1)
        cnt, flags = sim.read_gossip()
        done = (flags & 4) != 0
        assert (cnt >= prev_cnt).all()
        assert (done >= prev_done).all()  # converged never reverts
        assert int(done.sum()) == sim.status.completed
        assert (cnt[done] >= 11).all() and (cnt[~done] <= 10).all()
        # done nodes are frozen
        assert (cnt[prev_done] == prev_cnt[prev_done]).all()
        prev_cnt, prev_done = cnt, done


def test_fingerprint_fixture_reproduces():
    """The full-size fixture (tests/golden/fingerprints.json) is what the oracle computes: its
    smallest case re-run here, single-thread canonical order, matches trace and every digest."""
    from helpers import compare_digests, fingerprints, state_digests, unpack_trace

    fp = fingerprints()["C2_line_100k_pushsum"]
    sim = oracle.OracleSim(fp["n_arg"], fp["topology"], fp["algorithm"], seed=fp["seed"])
    st = sim.step(fp["cap"])
    assert (st.round, st.completed, st.converged) == (fp["rounds"], fp["completed"], fp["converged"])
    np.testing.assert_array_equal(sim.read_trace(), unpack_trace(fp["trace_z"]))
    compare_digests(state_digests(sim, fp["algorithm"]), fp["digests"])
    assert st.sum_s == float.fromhex(fp["sum_s"]) and st.sum_w == float.fromhex(fp["sum_w"])
    sim.close()
