"""Full-size oracle fingerprints of the BASELINE.json configurations (tests/golden/fingerprints.json).

    python tests/golden/make_fingerprints.py [--only NAME ...] [--threads 8]

The CPU oracle (oracle/gp_oracle.c, OpenMP pull mode: bit-identical to its canonical
single-thread order) runs each workload at the size BASELINE.json quotes it on, and the
fixture keeps what the GPU tests need to compare the HIP engine with it bit for bit without
running the oracle on the GPU box:

  * the layout (nodes, actors, grid, leader), the rounds executed and whether they converged;
  * the per-round ParentActor count (program.fs:44-63), the whole trace (int64, zlib +
    base64: helpers.unpack_trace);
  * SHA-256 digests of the final state, per array, over the whole actor range and over 16
    equal chunks of it (a mismatch names the chunk):
      push-sum: S, W (fp64 bits), flags, and the last round's messages dst / s / w
                (program.fs:119-143);
      gossip:   cnt (messageCount), flags (tok | done) (program.fs:89-105);
  * sum_s / sum_w (held + in-flight mass) as hex floats.

Cases:
  C3  `10000000 Imp3D push-sum` seed 1, to convergence (the headline workload)
  C2  `100000 line push-sum` seed 1 (5000-round cap; it converges in 1481 rounds) and
      `100000 3D push-sum` seed 1 to convergence (62125 rounds)
  C4  `100000000 full gossip` seed 1, to convergence
  C5w `100000000 Imp3D push-sum` seed 1 over a 50-round window: the largest Imp3D push-sum
      window whose oracle run fits this container's memory (C5 itself is 1e9 nodes)

The oracle is test infrastructure; this script only writes fixtures.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))

import oracle  # noqa: E402
from helpers import pack_trace, state_digests  # noqa: E402

OUT = os.path.join(HERE, "fingerprints.json")

# name: (n_arg, topology, algorithm, seed, rounds cap or None = to convergence)
CASES = {
    "C3_imp3d_10m_pushsum": (10_000_000, "Imp3D", "push-sum", 1, None),
    "C2_line_100k_pushsum": (100_000, "line", "push-sum", 1, 5000),
    "C2_3d_100k_pushsum": (100_000, "3D", "push-sum", 1, None),
    "C4_full_100m_gossip": (100_000_000, "full", "gossip", 1, None),
    "C5w_imp3d_100m_pushsum_w50": (100_000_000, "Imp3D", "push-sum", 1, 50),
}


def run(name, threads):
    n, topo, algo, seed, cap = CASES[name]
    t0 = time.time()
    sim = oracle.OracleSim(n, topo, algo, seed=seed)
    st = sim.step(cap if cap else 1 << 40, threads=threads)
    el = time.time() - t0
    rec = {
        "n_arg": n, "topology": topo, "algorithm": algo, "seed": seed, "cap": cap,
        "nodes": int(sim.layout.nodes), "actors": int(sim.layout.actors), "grid": int(sim.layout.grid),
        "leader": int(sim.layout.leader), "rounds": int(st.round), "completed": int(st.completed),
        "converged": int(st.converged), "sum_s": float(st.sum_s).hex(), "sum_w": float(st.sum_w).hex(),
        "trace_z": pack_trace(sim.read_trace()),
        "digests": state_digests(sim, algo),
        "oracle_seconds": round(el, 1), "oracle_threads": threads,
    }
    sim.close()
    print(f"{name}: rounds {rec['rounds']} converged {rec['converged']} ({el:.1f} s)", flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    args = ap.parse_args()
    data = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            data = json.load(f)
    for name in args.only or list(CASES):
        data[name] = run(name, args.threads)
        with open(OUT, "w") as f:
            json.dump(data, f, indent=1)


if __name__ == "__main__":
    main()
