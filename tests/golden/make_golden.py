"""Regenerate tests/golden/*.npz from the independent Python restatement (pyref.py).

    python tests/golden/make_golden.py

Each case stores the layout, the per-round completion trace, the state after a few rounds
(``mid_*``) and the state at convergence or at the round cap (``fin_*``).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import pyref  # noqa: E402

MID = 5
# (n_arg, topology, algo, seed, round cap)
CASES = [
    (20, "full", "gossip", 1, 4000),
    (100, "full", "gossip", 2, 4000),
    (1000, "full", "gossip", 1, 4000),
    (64, "line", "gossip", 1, 20000),
    (200, "line", "gossip", 3, 20000),
    (64, "2D", "gossip", 2, 20000),
    (20, "Imp3D", "gossip", 1, 4000),
    (133, "Imp3D", "gossip", 2, 4000),
    (1000, "Imp3D", "gossip", 3, 4000),
    (200, "3D", "gossip", 1, 4000),
    (20, "full", "push-sum", 1, 4000),
    (39, "full", "push-sum", 2, 4000),
    (1000, "full", "push-sum", 3, 4000),
    (20, "line", "push-sum", 1, 600),
    (200, "line", "push-sum", 2, 300),
    (50, "2D", "push-sum", 3, 400),
    (20, "Imp3D", "push-sum", 1, 4000),
    (200, "Imp3D", "push-sum", 2, 4000),
    (789, "Imp3D", "push-sum", 3, 4000),
    (1000, "Imp3D", "push-sum", 1, 4000),
    (200, "3D", "push-sum", 3, 4000),
    (1000, "3D", "push-sum", 2, 4000),
]


def case_name(n, topo, algo, seed):
    return f"{algo}_{topo}_{n}_s{seed}"


def run_case(n, topo, algo, seed, cap):
    t = pyref.TOPO_NAMES[topo]
    a = pyref.GOSSIP if algo == "gossip" else pyref.PUSHSUM
    sim = pyref.Sim(n, t, a, seed)
    out = {
        "n_arg": np.int64(n),
        "topology": np.int32(t),
        "algo": np.int32(a),
        "seed": np.uint64(seed),
        "nodes": np.int64(sim.nodes),
        "actors": np.int64(sim.A),
        "grid": np.int64(sim.grid),
        "leader": np.int64(sim.leader),
    }
    sim.step(MID)
    for k, v in sim.state().items():
        out["mid_" + k] = v
    out["mid_round"] = np.int64(sim.round)
    sim.step(cap - MID)
    for k, v in sim.state().items():
        out["fin_" + k] = v
    out["fin_round"] = np.int64(sim.round)
    out["converged"] = np.int32(sim.converged)
    out["trace"] = np.array(sim.trace, np.int64)
    return out


def main():
    manifest = []
    for n, topo, algo, seed, cap in CASES:
        name = case_name(n, topo, algo, seed)
        out = run_case(n, topo, algo, seed, cap)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        manifest.append({"name": name, "n_arg": n, "topology": topo, "algo": algo, "seed": seed,
                         "cap": cap, "rounds": int(out["fin_round"]), "converged": int(out["converged"])})
        print(name, "rounds", int(out["fin_round"]), "converged", int(out["converged"]), flush=True)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"mid_rounds": MID, "cases": manifest}, f, indent=1)


if __name__ == "__main__":
    main()
