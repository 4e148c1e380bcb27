"""Statistical sanity check against the reference's ASYNCHRONOUS actor execution (SURVEY.md §4.7,
§8(f) 2; north star: "the original async actor run serves as a statistical sanity check").

oracle/gp_async.c restates program.fs:38-147 under the Akka execution model (FIFO mailboxes, a
seeded random interleaving of runnable actors) on the same neighbour lists and leader as the
round-mode oracle — which the HIP engine matches bit for bit (test_gpu_parity.py).  The two
execution models produce different trajectories by design; what must agree is the behaviour:

  * both converge on every reference topology, with the reference's report rules (11th receipt,
    termRound 1 -> 3) and push-sum mass conserved;
  * both rank the topologies the same way: full and Imp3D converge well ahead of line and "2D"
    (at N=200: round mode >2.8x in rounds, async mode >8x gossip / >60x push-sum in messages;
    report.pdf p.4-5 at N=1000: gossip full 1167.20 ms vs line 7322.90 ms; push-sum full 418.63 <
    Imp3D 541.43 < 2D 26818.37 < line 147447.74 ms).
"""
import numpy as np
import pytest

import oracle

TOPOS = ["full", "Imp3D", "line", "2D"]
SEEDS = (1, 2, 3)


@pytest.mark.parametrize("algo", ["gossip", "push-sum"])
@pytest.mark.parametrize("topo", TOPOS)
def test_async_converges_and_conserves(topo, algo):
    nodes, actors, _ = oracle.sizes(200, topo)
    st, a = oracle.async_run(200, topo, algo, seed=1)
    assert st.converged and st.completed == nodes
    if algo == "gossip":
        done = (a["flags"] & 4) != 0
        assert int(done.sum()) == nodes
        assert (a["cnt"][done] >= 11).all()  # program.fs:102: reports on the 11th receipt
        assert (a["cnt"][~done] <= 10).all()
    else:
        # program.fs:107-143 only moves mass: held + in-mailbox sums stay sum(i), #actors
        assert st.sum_s == pytest.approx(actors * (actors - 1) / 2.0, rel=1e-12)
        assert st.sum_w == pytest.approx(float(actors), rel=1e-12)
        conv = (a["flags"] & 16) != 0
        assert int(conv.sum()) == nodes
        assert np.isfinite(a["S"] / a["W"]).all()


def _round_mode(topo, algo, seed):
    sim = oracle.OracleSim(200, topo, algo, seed=seed)
    st = sim.step(100_000)
    sim.close()
    assert st.converged
    return st.round


def _async_mode(topo, algo, seed):
    st, _ = oracle.async_run(200, topo, algo, seed=seed)
    assert st.converged
    return st.steps


@pytest.mark.parametrize("algo", ["gossip", "push-sum"])
def test_topology_ranking_agrees_with_async(algo):
    for run in (_round_mode, _async_mode):
        t = {topo: np.mean([run(topo, algo, s) for s in SEEDS]) for topo in TOPOS}
        fast, slow = max(t["full"], t["Imp3D"]), min(t["line"], t["2D"])
        assert slow > 2.0 * fast, (run.__name__, t)
        if algo == "push-sum":
            assert t["full"] < t["Imp3D"] < slow, (run.__name__, t)  # report.pdf p.5 order


def test_async_is_seed_deterministic():
    a, x = oracle.async_run(100, "Imp3D", "push-sum", seed=7)
    b, y = oracle.async_run(100, "Imp3D", "push-sum", seed=7)
    assert (a.steps, a.completed) == (b.steps, b.completed)
    np.testing.assert_array_equal(x["S"].view(np.uint64), y["S"].view(np.uint64))


# ---- report.pdf p.4-5 sweeps ("compare distributions against the report.pdf
# p.4-5 sweeps").  Cost of a run in each model: the async model's processed messages and the
# round mode's node-updates (actors x rounds), each averaged over three seeds; both must rise
# with N the way the report's wall times do (rank correlation over N = 20 ... 1000).
from report_sweeps import MIN_RHO, REPORT_MS, SWEEP_N, spearman  # noqa: E402


@pytest.mark.parametrize("algo,topo", sorted(REPORT_MS))
def test_cost_over_n_follows_report_sweep(algo, topo):
    ms, asy, rnd = [], [], []
    for n, t in zip(SWEEP_N, REPORT_MS[(algo, topo)]):
        if t is None:
            continue
        a, r = [], []
        for s in SEEDS:
            st, _ = oracle.async_run(n, topo, algo, seed=s, max_steps=20_000_000)
            if st.converged:
                a.append(float(st.messages))
            sim = oracle.OracleSim(n, topo, algo, seed=s)
            rs = sim.step(1 << 22)
            assert rs.converged
            r.append(float(sim.actors) * int(rs.round))
            sim.close()
        if a:  # the async line / 2D push-sum runs at the top sizes may outlast the step cap
            ms.append(t)
            asy.append(np.mean(a))
            rnd.append(np.mean(r))
    assert len(ms) >= 8, (algo, topo, len(ms))
    rho_async, rho_round = spearman(ms, asy), spearman(ms, rnd)
    assert rho_async >= MIN_RHO[(algo, topo)], (algo, topo, rho_async, ms, asy)
    assert rho_round >= MIN_RHO[(algo, topo)], (algo, topo, rho_round, ms, rnd)
