"""The product against the reference's ASYNCHRONOUS actor execution, statistically (north star:
"the original async actor run serves as a statistical sanity check").

The HIP engine runs synchronous rounds; oracle/gp_async.c restates program.fs:38-147 under the
Akka execution model (FIFO mailboxes, a seeded random interleaving of runnable actors) on the
same neighbour lists and leader.  Trajectories differ by design, so the checks are on the
distribution of outcomes over seeds (numbers from the two models in this container, N = 300 /
1000, 8 seeds: every per-seed median error below 3e-3, the median over seeds below 1e-6;
"full" below 1e-12 in both):

  * push-sum on "full" and Imp3D: both models drive the converged estimates S/W to the mean of
    the participants' initial values (program.fs:107-108: S_i = i, W_i = 1);
  * gossip: in both models every node reports, each on its 11th receipt or later (program.fs:102),
    and the receipts a reported node holds stay in the same small range;
  * convergence cost ranks the topologies the same way in both models (rounds here, actor steps
    there): line and "2D" far behind full and Imp3D (report.pdf p.4-5).
"""
import numpy as np
import pytest

import oracle
from gossip_amd import Simulator

pytestmark = pytest.mark.gpu

SEEDS = range(1, 9)


def _target(n_arg, topo):
    nodes, actors, _ = oracle.sizes(n_arg, topo)
    # Imp3D's isolated actor `nodes` never mixes (program.fs:293): the participants are 0..nodes-1
    return (nodes - 1) / 2.0 if topo == "Imp3D" else (actors - 1) / 2.0


def _median_err(S, W, flags, mu):
    conv = (flags & 16) != 0
    assert conv.any()
    return float(np.median(np.abs(S[conv] / W[conv] - mu) / mu))


@pytest.mark.parametrize("n_arg", [300, 1000])
@pytest.mark.parametrize("topo", ["full", "Imp3D"])
def test_pushsum_estimates_agree_with_async(topo, n_arg):
    mu = _target(n_arg, topo)
    gpu, asy = [], []
    for s in SEEDS:
        sim = Simulator(n_arg, topo, "push-sum", seed=s)
        st = sim.step(1 << 20)
        assert st.converged
        gpu.append(_median_err(*sim.read_pushsum(), mu))
        sim.close()
        ast, a = oracle.async_run(n_arg, topo, "push-sum", seed=s)
        assert ast.converged
        asy.append(_median_err(a["S"], a["W"], a["flags"], mu))
    for name, e in (("round (HIP)", gpu), ("async", asy)):
        assert max(e) < 1e-2, (name, e)
        assert float(np.median(e)) < 1e-4, (name, e)
        if topo == "full":
            assert max(e) < 1e-11, (name, e)


@pytest.mark.parametrize("topo", ["full", "Imp3D", "line", "2D"])
def test_gossip_reports_agree_with_async(topo):
    n_arg = 300
    nodes, _, _ = oracle.sizes(n_arg, topo)
    for s in (1, 2, 3):
        sim = Simulator(n_arg, topo, "gossip", seed=s)
        st = sim.step(1 << 20)
        assert st.converged and st.completed == nodes
        cnt, flags = sim.read_gossip()
        sim.close()
        ast, a = oracle.async_run(n_arg, topo, "gossip", seed=s)
        assert ast.converged and ast.completed == nodes
        for c, f in ((cnt, flags), (a["cnt"], a["flags"])):
            done = (f & 4) != 0
            assert int(done.sum()) == nodes
            assert (c[done] >= 11).all()
            assert 11.0 <= float(c[done].mean()) <= 20.0


@pytest.mark.parametrize("algo", ["gossip", "push-sum"])
def test_topology_cost_ranking_agrees_with_async(algo):
    topos = ["full", "Imp3D", "line", "2D"]
    rounds, steps = {}, {}
    for t in topos:
        r, q = [], []
        for s in (1, 2, 3):
            sim = Simulator(200, t, algo, seed=s)
            st = sim.step(1 << 20)
            assert st.converged
            r.append(int(st.round))
            sim.close()
            ast, _ = oracle.async_run(200, t, algo, seed=s)
            q.append(int(ast.steps))
        rounds[t], steps[t] = np.mean(r), np.mean(q)
    for cost in (rounds, steps):
        assert min(cost["line"], cost["2D"]) > 2.0 * max(cost["full"], cost["Imp3D"]), (rounds, steps)


# The HIP round engine's cost (node-updates to convergence, three seeds) over report.pdf's
# sweep sizes rises with N the way the reference's published wall times do (tests/report_sweeps.py).
from report_sweeps import MIN_RHO, REPORT_MS, SWEEP_N, spearman  # noqa: E402


@pytest.mark.parametrize("algo,topo", sorted(REPORT_MS))
def test_engine_cost_over_n_follows_report_sweep(algo, topo):
    ms, cost = [], []
    for n, t in zip(SWEEP_N, REPORT_MS[(algo, topo)]):
        if t is None:
            continue
        c = []
        for s in (1, 2, 3):
            sim = Simulator(n, topo, algo, seed=s)
            st = sim.step(1 << 22)
            assert st.converged
            c.append(float(sim.actors) * int(st.round))
            sim.close()
        ms.append(t)
        cost.append(np.mean(c))
    rho = spearman(ms, cost)
    assert rho >= MIN_RHO[(algo, topo)], (algo, topo, rho, ms, cost)
