"""Shared comparison helpers for oracle / golden / HIP parity tests."""
import json
import os

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
