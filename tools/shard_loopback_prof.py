"""W shards of one graph on ONE GPU (loopback exchange): per-kernel cost of the shard round at a
realistic remote fraction (e.g. 8 ranks -> 7/8 of the extra links remote), for A/B builds.

    python3 tools/shard_loopback_prof.py --world 8 --n 80000000 --rounds 64
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cop5615-gossip_protocol_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=80_000_000)
ap.add_argument("--world", type=int, default=8)
ap.add_argument("--topology", default="Imp3D")
ap.add_argument("--algorithm", default="push-sum")
ap.add_argument("--rounds", type=int, default=64)
a = ap.parse_args()

import torch  # noqa: E402

from gossip_amd import sharded  # noqa: E402

torch.cuda.set_device(0)
shards = [sharded.HipShard(a.n, a.topology, a.algorithm, rank=r, world=a.world, seed=1, kernel_timing=True)
          for r in range(a.world)]
sharded.run_local(shards, max_rounds=8)
torch.cuda.synchronize()
t0 = time.perf_counter()
sts = sharded.run_local(shards, max_rounds=a.rounds)
torch.cuda.synchronize()
el = time.perf_counter() - t0
ks = shards[0].kernel_stats()
print(f"{a.world} shards of {a.n} {a.topology} {a.algorithm}: {a.rounds} rounds in {el * 1e3:.1f} ms "
      f"(all shards serialised on one GPU); rank 0 {ks['kernel']} {ks['avg_ms'] * 1e3:.1f} us, "
      f"{ks['aux_kernel']} {ks['aux_avg_ms'] * 1e3:.1f} us", flush=True)
for e in shards:
    e.close()
