"""Shared comparison helpers for oracle / golden / HIP parity tests."""
import base64
import hashlib
import json
import os
import socket
import subprocess
import sys
import tempfile
import zlib

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLD, "manifest.json")) as f:
        return json.load(f)


def load_golden(name):
    with np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def bits(a):
    return np.ascontiguousarray(a, np.float64).view(np.uint64)


def check_state(sim, g, prefix):
    """sim: oracle.OracleSim or gossip_amd.Simulator; g: golden dict; bit-exact comparison."""
    if int(g["algo"]) == 0:
        cnt, flags = sim.read_gossip()
        np.testing.assert_array_equal(cnt, g[prefix + "cnt"])
        np.testing.assert_array_equal(flags, g[prefix + "flags"])
    else:
        S, W, flags = sim.read_pushsum()
        np.testing.assert_array_equal(bits(S), bits(g[prefix + "S"]))
        np.testing.assert_array_equal(bits(W), bits(g[prefix + "W"]))
        np.testing.assert_array_equal(flags, g[prefix + "flags"])
        d, s, w = sim.read_messages()
        np.testing.assert_array_equal(d, g[prefix + "msg_dst"])
        np.testing.assert_array_equal(bits(s), bits(g[prefix + "msg_s"]))
        np.testing.assert_array_equal(bits(w), bits(g[prefix + "msg_w"]))


DIGEST_CHUNKS = 16


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def digest_arrays(arrays):
    """{name: {"all": sha256, "chunks": [16 x sha256]}} of full-range state arrays (little
    endian; fp64 compared as bits)."""
    out = {}
    for k, a in arrays.items():
        if a.dtype == np.float64:
            a = a.view(np.uint64)
        out[k] = {"all": _sha(a), "chunks": [_sha(c) for c in np.array_split(a, DIGEST_CHUNKS)]}
    return out


def state_arrays(sim, algo):
    """Full-range state of any engine with the read_* API (oracle.OracleSim, gossip_amd.Simulator)."""
    if algo in (0, "gossip"):
        cnt, flags = sim.read_gossip()
        return {"cnt": cnt, "flags": flags}
    S, W, flags = sim.read_pushsum()
    d, s, w = sim.read_messages()
    return {"S": S, "W": W, "flags": flags, "msg_dst": d, "msg_s": s, "msg_w": w}


def state_digests(sim, algo):
    return digest_arrays(state_arrays(sim, algo))


def compare_digests(got, want):
    """Assert two digest dicts are equal; on a mismatch name the array and the first chunk."""
    assert set(got) == set(want), (sorted(got), sorted(want))
    for k in want:
        if got[k]["all"] != want[k]["all"]:
            bad = [i for i, (a, b) in enumerate(zip(got[k]["chunks"], want[k]["chunks"])) if a != b]
            raise AssertionError(f"state array {k!r} differs from the oracle fingerprint in chunks {bad} "
                                 f"(of {DIGEST_CHUNKS})")


def pack_trace(trace):
    return base64.b64encode(zlib.compress(np.asarray(trace, np.int64).tobytes(), 9)).decode()


def unpack_trace(z):
    return np.frombuffer(zlib.decompress(base64.b64decode(z)), np.int64)


def fingerprints():
    with open(os.path.join(GOLD, "fingerprints.json")) as f:
        return json.load(f)


def check_same(a, b, algo):
    """Two simulators (any engines) hold bit-identical state."""
    if algo in (0, "gossip"):
        ca, fa = a.read_gossip()
        cb, fb = b.read_gossip()
        np.testing.assert_array_equal(ca, cb)
        np.testing.assert_array_equal(fa, fb)
    else:
        Sa, Wa, fa = a.read_pushsum()
        Sb, Wb, fb = b.read_pushsum()
        np.testing.assert_array_equal(fa, fb)
        np.testing.assert_array_equal(bits(Sa), bits(Sb))
        np.testing.assert_array_equal(bits(Wa), bits(Wb))
        da, sa, wa = a.read_messages()
        db, sb, wb = b.read_messages()
        np.testing.assert_array_equal(da, db)
        np.testing.assert_array_equal(bits(sa), bits(sb))
        np.testing.assert_array_equal(bits(wa), bits(wb))
    np.testing.assert_array_equal(a.read_trace(), b.read_trace())


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_dist_job(world, backend, n, topology, algorithm, seed, cap, timeout, extra=()):
    """Launch tests/dist_shard_job.py under torch.distributed.run with `world` ranks (extra: more job
    options, e.g. --force-pieces); returns the rank parts (status, trace, state arrays, shard counters)
    in rank order."""
    out = tempfile.mkdtemp(prefix="gp_dist_")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_shard_job.py"), "--backend", backend, "--n-arg", str(n),
           "--topology", topology, "--algorithm", algorithm, "--seed", str(seed), "--cap", str(cap or 0), "--out", out,
           *extra]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    parts = []
    for q in range(world):
        with np.load(os.path.join(out, f"rank{q}.npz"), allow_pickle=False) as z:
            parts.append({k: z[k] for k in z.files})
    return parts


def join_parts(parts, keys):
    return {k: np.concatenate([p[k] for p in parts]) for k in keys}
