"""Fixed-size workload for rocprofv3 runs: create a simulator and run R rounds (no CPU work).

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/prof_run.py --rounds 300
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cop5615-gossip_protocol_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--topology", default="Imp3D")
ap.add_argument("--algorithm", default="push-sum")
ap.add_argument("--rounds", type=int, default=300)
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--generic", action="store_true")
ap.add_argument("--series", default=None, help="write the run's per-round completion counts (JSON) here")
a = ap.parse_args()

from gossip_amd import Simulator  # noqa: E402

sim = Simulator(a.n, a.topology, a.algorithm, seed=a.seed, generic=a.generic)
t0 = time.perf_counter()
st = sim.step(a.rounds)
el = time.perf_counter() - t0
print(f"{a.n} {a.topology} {a.algorithm}: {st.round} rounds, converged={st.converged}, "
      f"{el * 1e3:.1f} ms host, {st.device_ms:.1f} ms device, "
      f"{sim.actors * st.round / el / 1e9:.2f} G node-updates/s", flush=True)
if a.series:
    import json

    with open(a.series, "w") as f:
        json.dump({"workload": f"{a.n} {a.topology} {a.algorithm}", "world": 1, "nodes": int(sim.layout.nodes),
                   "rounds": int(st.round), "trace": [int(x) for x in sim.read_trace()]}, f)
sim.close()
