"""Stage timing of one shard's setup and first rounds (no collective: world 1 needs no
exchange), to locate slow or stuck stages at large sizes.

    python3 tools/diag_shard_setup.py --n 1000000000 [--world 1 --rank 0 --rounds 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cop5615-gossip_protocol_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000_000)
ap.add_argument("--topology", default="Imp3D")
ap.add_argument("--algorithm", default="push-sum")
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
t0 = time.perf_counter()


def say(msg):
    print(f"{time.perf_counter() - t0:8.2f} s  {msg}", flush=True)


import torch  # noqa: E402

from gossip_amd import sharded  # noqa: E402

torch.cuda.set_device(0)
say("torch ready")
e = sharded.HipShard(a.n, a.topology, a.algorithm, rank=a.rank, world=a.world, seed=1)
say(f"created: actors {e.actors}, own [{e.lo}, {e.hi}), send {sum(e.send_splits)} B, recv {sum(e.recv_splits)} B")
st = e.sync()
say(f"sync: round {st.round}")
for i in range(a.rounds):
    e.round()
    e.deliver()
    torch.cuda.synchronize()
    say(f"round {i} done")
st = e.sync()
say(f"sync: round {st.round} completed {st.completed}")
e.reset()
say("reset")
e.close()
say("closed")
