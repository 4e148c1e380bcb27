"""Find the first round where the HIP engine and the CPU oracle disagree (state or messages),
and print the differing actors with their neighbourhood.  Diagnostic only.

    python tools/diag_compare.py --n 10000000 --topology Imp3D --algorithm push-sum --chunk 64
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cop5615-gossip_protocol_amd"), os.path.join(ROOT, "oracle")]

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10_000_000)
ap.add_argument("--topology", default="Imp3D")
ap.add_argument("--algorithm", default="push-sum")
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--chunk", type=int, default=64)
ap.add_argument("--threads", type=int, default=16)
ap.add_argument("--max-rounds", type=int, default=1 << 30)
a = ap.parse_args()

import oracle  # noqa: E402
from gossip_amd import Simulator  # noqa: E402

gpu = Simulator(a.n, a.topology, a.algorithm, seed=a.seed)
cpu = oracle.OracleSim(a.n, a.topology, a.algorithm, seed=a.seed)


def arrays(s):
    if a.algorithm == "gossip":
        c, f = s.read_gossip()
        return {"cnt": c, "flags": f}
    S, W, f = s.read_pushsum()
    d, ms, mw = s.read_messages()
    return {"S": S.view(np.uint64), "W": W.view(np.uint64), "flags": f, "dst": d, "ms": ms.view(np.uint64),
            "mw": mw.view(np.uint64)}


done = 0
while done < a.max_rounds:
    step = min(a.chunk, a.max_rounds - done)
    gs = gpu.step(step)
    cs = cpu.step(step, threads=a.threads)
    done = int(cs.round)
    ga, ca = arrays(gpu), arrays(cpu)
    bad = {k: np.nonzero(ga[k] != ca[k])[0] for k in ga}
    nbad = sum(len(v) for v in bad.values())
    print(f"round {gs.round}/{cs.round} completed {gs.completed}/{cs.completed} mismatches "
          + " ".join(f"{k}:{len(v)}" for k, v in bad.items()), flush=True)
    if nbad or gs.round != cs.round:
        # narrow down to the exact round: rerun both to the chunk start, then step one by one
        lo = done - step
        gpu.reset()
        cpu.close()
        cpu = oracle.OracleSim(a.n, a.topology, a.algorithm, seed=a.seed)
        if lo:
            gpu.step(lo)
            cpu.step(lo, threads=a.threads)
        for r in range(lo, done):
            gpu.step(1)
            cpu.step(1, threads=a.threads)
            ga, ca = arrays(gpu), arrays(cpu)
            bad = {k: np.nonzero(ga[k] != ca[k])[0] for k in ga}
            if any(len(v) for v in bad.values()):
                print(f"first difference after round {r} (state after {r + 1} rounds):", flush=True)
                for k, v in bad.items():
                    if len(v):
                        print(f"  {k}: {len(v)} actors, first {v[:12].tolist()}")
                        for i in v[:6]:
                            print(f"    v={i} gpu={ga[k][i]} cpu={ca[k][i]} nbrs={cpu.neighbors(int(i)).tolist()}")
                break
        break
    if cs.converged:
        print("converged, no difference", flush=True)
        break
