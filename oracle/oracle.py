"""ctypes wrapper for oracle/libgp_oracle.so (the CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker or the timed CPU baseline — never as the product.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgp_oracle.so")

TOPOLOGIES = {"line": 0, "full": 1, "2D": 2, "Imp3D": 3, "3D": 4}
ALGOS = {"gossip": 0, "push-sum": 1}


class Config(C.Structure):
    _fields_ = [("n_arg", C.c_int64), ("topology", C.c_int32), ("algo", C.c_int32),
                ("seed", C.c_uint64), ("delta", C.c_double), ("gossip_threshold", C.c_int32),
                ("term_init", C.c_int32), ("term_limit", C.c_int32)]


class Layout(C.Structure):
    _fields_ = [("nodes", C.c_int64), ("actors", C.c_int64), ("grid", C.c_int64),
                ("leader", C.c_int64), ("participants", C.c_int64)]


class Status(C.Structure):
    _fields_ = [("round", C.c_int64), ("completed", C.c_int64), ("converged", C.c_int32),
                ("pad", C.c_int32), ("sum_s", C.c_double), ("sum_w", C.c_double)]


class AsyncStatus(C.Structure):
    _fields_ = [("steps", C.c_int64), ("completed", C.c_int64), ("converged", C.c_int32), ("pad", C.c_int32),
                ("messages", C.c_int64), ("sum_s", C.c_double), ("sum_w", C.c_double)]


_lib = None


def build():
    """Compile the oracle with its Makefile (gcc, no GPU needed)."""
    import subprocess
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.gpo_create.restype = P
        L.gpo_create.argtypes = [C.POINTER(Config), C.POINTER(Layout)]
        L.gpo_step.argtypes = [P, C.c_int64, C.c_int32, C.POINTER(Status)]
        L.gpo_degree.argtypes = [P, C.c_int64]
        L.gpo_neighbors.argtypes = [P, C.c_int64, P, C.c_int32]
        L.gpo_read_gossip.argtypes = [P, C.c_int64, C.c_int64, P, P]
        L.gpo_read_pushsum.argtypes = [P, C.c_int64, C.c_int64, P, P, P]
        L.gpo_read_messages.argtypes = [P, C.c_int64, C.c_int64, P, P, P]
        L.gpo_read_trace.argtypes = [P, C.c_int64, C.c_int64, P]
        L.gpo_destroy.argtypes = [P]
        L.gpo_sizes.argtypes = [C.c_int64, C.c_int32, P, P, P]
        L.gpo_philox4x32_10.argtypes = [P, P, P]
        L.gpo_shard_create.restype = P
        L.gpo_shard_create.argtypes = [C.POINTER(Config), C.c_int32, C.c_int32, P, C.POINTER(Layout)]
        L.gpo_shard_plan.argtypes = [P, P, P]
        L.gpo_shard_round.argtypes = [P, P]
        L.gpo_shard_deliver.argtypes = [P, P]
        L.gpo_shard_sync.argtypes = [P, C.POINTER(Status)]
        L.gpo_async_run.argtypes = [C.POINTER(Config), C.c_int64, C.POINTER(AsyncStatus), P, P, P, P]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def philox(ctr, key):
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().gpo_philox4x32_10(_ptr(c), _ptr(k), _ptr(out))
    return out


def sizes(n_arg, topology):
    t = TOPOLOGIES[topology] if isinstance(topology, str) else topology
    v = np.zeros(3, np.int64)
    rc = lib().gpo_sizes(n_arg, t, _ptr(v[0:1]), _ptr(v[1:2]), _ptr(v[2:3]))
    if rc:
        raise ValueError(f"invalid size {n_arg} {topology}")
    return int(v[0]), int(v[1]), int(v[2])


class OracleSim:
    """One simulation in the CPU restatement; mirrors the product's Simulator API."""

    def __init__(self, n_arg, topology, algo, seed=1, delta=1e-10, gossip_threshold=10,
                 term_init=1, term_limit=3):
        t = TOPOLOGIES[topology] if isinstance(topology, str) else topology
        a = ALGOS[algo] if isinstance(algo, str) else algo
        self.cfg = Config(n_arg, t, a, seed, delta, gossip_threshold, term_init, term_limit)
        self.layout = Layout()
        self.algo = a
        h = lib().gpo_create(C.byref(self.cfg), C.byref(self.layout))
        if not h:
            raise ValueError(f"gpo_create failed for {n_arg} {topology} {algo}")
        self.h = C.c_void_p(h)
        self.status = Status()

    @property
    def actors(self):
        return int(self.layout.actors)

    def step(self, max_rounds=1 << 40, threads=0):
        rc = lib().gpo_step(self.h, max_rounds, threads, C.byref(self.status))
        if rc:
            raise RuntimeError(f"gpo_step rc={rc}")
        return self.status

    def degree(self, v):
        return lib().gpo_degree(self.h, v)

    def neighbors(self, v):
        out = np.zeros(max(1, self.degree(v)), np.uint32)
        d = lib().gpo_neighbors(self.h, v, _ptr(out), len(out))
        return out[:d]

    def read_gossip(self):
        n = self.actors
        cnt = np.zeros(n, np.uint32)
        flags = np.zeros(n, np.uint8)
        if lib().gpo_read_gossip(self.h, 0, n, _ptr(cnt), _ptr(flags)):
            raise RuntimeError("read_gossip")
        return cnt, flags

    def read_pushsum(self):
        n = self.actors
        S = np.zeros(n, np.float64)
        W = np.zeros(n, np.float64)
        flags = np.zeros(n, np.uint8)
        if lib().gpo_read_pushsum(self.h, 0, n, _ptr(S), _ptr(W), _ptr(flags)):
            raise RuntimeError("read_pushsum")
        return S, W, flags

    def read_messages(self):
        n = self.actors
        d = np.zeros(n, np.uint32)
        s = np.zeros(n, np.float64)
        w = np.zeros(n, np.float64)
        if lib().gpo_read_messages(self.h, 0, n, _ptr(d), _ptr(s), _ptr(w)):
            raise RuntimeError("read_messages")
        return d, s, w

    def read_trace(self):
        r = int(self.status.round)
        out = np.zeros(r, np.int64)
        if r and lib().gpo_read_trace(self.h, 0, r, _ptr(out)):
            raise RuntimeError("read_trace")
        return out

    def close(self):
        if self.h:
            lib().gpo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OracleShard(OracleSim):
    """Rank `rank` of a sharded CPU run (gpo_shard_*): the checker of the multi-GPU
    decomposition.  Same engine interface as gossip_amd.sharded.HipShard (round / deliver /
    sync, send_buf / recv_buf with per-peer splits), with CPU torch tensors as buffers, so
    the product's host loop and torch.distributed transport drive it unchanged (gloo)."""

    def __init__(self, n_arg, topology, algo, *, rank, world, bounds, seed=1, **kw):
        import torch

        t = TOPOLOGIES[topology] if isinstance(topology, str) else topology
        a = ALGOS[algo] if isinstance(algo, str) else algo
        self.cfg = Config(n_arg, t, a, seed, kw.get("delta", 1e-10), kw.get("gossip_threshold", 10),
                          kw.get("term_init", 1), kw.get("term_limit", 3))
        self.layout = Layout()
        self.algo = a
        b = np.asarray(bounds, np.int64)
        h = lib().gpo_shard_create(C.byref(self.cfg), rank, world, _ptr(b), C.byref(self.layout))
        if not h:
            raise ValueError(f"gpo_shard_create failed for {n_arg} {topology} {algo} rank {rank}/{world}")
        self.h = C.c_void_p(h)
        self.status = Status()
        self.rank, self.world = rank, world
        self.lo, self.hi = int(b[rank]), int(b[rank + 1])
        sb = np.zeros(world, np.int64)
        rb = np.zeros(world, np.int64)
        lib().gpo_shard_plan(self.h, _ptr(sb), _ptr(rb))
        self.send_splits, self.recv_splits = [int(x) for x in sb], [int(x) for x in rb]
        self.send_buf = torch.zeros(int(sb.sum()), dtype=torch.uint8)
        self.recv_buf = torch.zeros(int(rb.sum()), dtype=torch.uint8)

    def round(self):
        if lib().gpo_shard_round(self.h, C.c_void_p(self.send_buf.data_ptr())):
            raise RuntimeError("gpo_shard_round")

    def deliver(self):
        if lib().gpo_shard_deliver(self.h, C.c_void_p(self.recv_buf.data_ptr())):
            raise RuntimeError("gpo_shard_deliver")

    def sync(self):
        if lib().gpo_shard_sync(self.h, C.byref(self.status)):
            raise RuntimeError("gpo_shard_sync")
        return self.status

    def _own(self, arrays):
        return tuple(a[self.lo:self.hi] for a in arrays)

    def read_gossip(self):
        return self._own(super().read_gossip())

    def read_pushsum(self):
        return self._own(super().read_pushsum())

    def read_messages(self):
        return self._own(super().read_messages())


def async_run(n_arg, topology, algo, seed=1, max_steps=50_000_000, delta=1e-10, gossip_threshold=10,
              term_init=1, term_limit=3):
    """The reference's asynchronous actor execution (gp_async.c) on the same neighbour lists and
    leader: a statistical sanity check of the round engine, not a parity oracle.  Returns
    (status, per-actor arrays {cnt, S, W, flags})."""
    t = TOPOLOGIES[topology] if isinstance(topology, str) else topology
    a = ALGOS[algo] if isinstance(algo, str) else algo
    cfg = Config(n_arg, t, a, seed, delta, gossip_threshold, term_init, term_limit)
    _, actors, _ = sizes(n_arg, t)
    cnt = np.zeros(actors, np.uint32)
    S = np.zeros(actors, np.float64)
    W = np.zeros(actors, np.float64)
    flags = np.zeros(actors, np.uint8)
    st = AsyncStatus()
    rc = lib().gpo_async_run(C.byref(cfg), max_steps, C.byref(st), _ptr(cnt), _ptr(S), _ptr(W), _ptr(flags))
    if rc:
        raise RuntimeError(f"gpo_async_run failed ({rc})")
    return st, {"cnt": cnt, "S": S, "W": W, "flags": flags}
