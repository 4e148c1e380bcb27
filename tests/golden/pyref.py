"""Independent Python restatement of the reference's hot path (golden-vector generator).

TEST INFRASTRUCTURE ONLY.  Written directly from /root/reference/program.fs and the
synchronous-round semantics of DESIGN.md §2, without looking at either
oracle/gp_oracle.c or the HIP product, so the committed vectors it produces are a second,
independent opinion.  Pure-Python loops (small N only); Philox is vectorised with numpy.

Parity against the reference itself is UNPINNED (the reference is an unseeded async
Akka.NET program with no tests, and cannot run here); see DESIGN.md §4.
"""
from __future__ import annotations

import math

import numpy as np

LINE, FULL, TWO_D, IMP3D, THREE_D = 0, 1, 2, 3, 4
GOSSIP, PUSHSUM = 0, 1
TOPO_NAMES = {"line": LINE, "full": FULL, "2D": TWO_D, "Imp3D": IMP3D, "3D": THREE_D}

_M32 = np.uint64(0xFFFFFFFF)
_MUL = (np.uint64(0xD2511F53), np.uint64(0xCD9E8D57))
_WEYL = (np.uint64(0x9E3779B9), np.uint64(0xBB67AE85))
STREAM = {"leader": 0x4C454144, "topo": 0x544F504F, "gossip": 0x474F5353, "push": 0x50555348}
NONE = 0xFFFFFFFF


def philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Random123).  Arguments: uint64 arrays/scalars holding 32-bit values."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint64) for x in (c0, c1, c2, c3))
    k0 = np.uint64(k0)
    k1 = np.uint64(k1)
    s32 = np.uint64(32)
    for i in range(10):
        if i:
            k0 = (k0 + _WEYL[0]) & _M32
            k1 = (k1 + _WEYL[1]) & _M32
        p0 = _MUL[0] * c0
        p1 = _MUL[1] * c2
        c0, c1, c2, c3 = ((p1 >> s32) ^ c1 ^ k0) & _M32, p1 & _M32, ((p0 >> s32) ^ c3 ^ k1) & _M32, p0 & _M32
    return c0, c1, c2, c3


def draw_words(seed: int, stream: str, r: int, vs):
    """All four Philox words for counters {v, r, 0, stream}, v in vs."""
    vs = np.asarray(vs, dtype=np.uint64)
    z = np.zeros_like(vs)
    return philox(vs, z + np.uint64(r), z, z + np.uint64(STREAM[stream]), seed & 0xFFFFFFFF, seed >> 32)


def scale(x, n):
    """Random().Next(0, n) replacement: floor(x * n / 2^32)."""
    return int((int(x) * int(n)) >> 32)


def sizes(n_arg: int, topology: int):
    """(nodes, actors, grid) — program.fs:26-31, :228-229, :268."""
    if topology in (LINE, FULL):
        return n_arg, n_arg + 1, 0
    if topology == TWO_D:
        g = int(math.ceil(math.sqrt(float(n_arg))))
        return g * g, g * g + 1, g
    c = math.floor(float(n_arg) ** 0.33334)
    nodes = int(float(c) ** 3.0)
    g = int(math.floor(float(n_arg) ** 0.34))
    return nodes, nodes + 1, g


def neighbours(n_arg: int, topology: int, seed: int):
    """Neighbour arrays in the reference's order, one Python list per actor."""
    nodes, actors, g = sizes(n_arg, topology)
    if topology == FULL:  # program.fs:201-206
        return None
    nb = [[] for _ in range(actors)]
    if topology == LINE:  # program.fs:162-171
        for i in range(actors):
            if i == 0:
                nb[i] = [1]
            elif i == nodes:
                nb[i] = [nodes - 1]
            else:
                nb[i] = [i - 1, i + 1]
    elif topology == TWO_D:  # program.fs:242-248
        for i in range(actors):
            if i > 0:
                nb[i].append(i - 1)
            if i < nodes:
                nb[i].append(i + 1)
    else:  # program.fs:281-313
        links = None
        if topology == IMP3D:
            w0 = draw_words(seed, "topo", 0, range(nodes))[0]
            links = [scale(w0[i], nodes - 1) for i in range(nodes)]
        zm, ym, lim = g * g, g, g - 1
        for z in range(g):
            for y in range(g):
                for x in range(g):
                    i = z * zm + y * ym + x
                    if i >= nodes:
                        continue
                    lst = []
                    if x > 0:
                        lst.append(i - 1)
                    if x < lim and i + 1 < nodes:
                        lst.append(i + 1)
                    if y > 0:
                        lst.append(i - ym)
                    if y < lim and i + ym < nodes:
                        lst.append(i + ym)
                    if z > 0:
                        lst.append(i - zm)
                    if z < lim and i + zm < nodes:
                        lst.append(i + zm)
                    if links is not None:
                        lst.append(links[i])
                    nb[i] = lst
    return nb


class Sim:
    def __init__(self, n_arg, topology, algo, seed, delta=1e-10, threshold=10, term_init=1, term_limit=3):
        self.topology, self.algo, self.seed = topology, algo, seed
        self.delta, self.thr, self.term_limit = delta, threshold, term_limit
        self.nodes, self.A, self.grid = sizes(n_arg, topology)
        self.nb = neighbours(n_arg, topology, seed)
        self.leader = scale(draw_words(seed, "leader", 0, [0])[0][0], self.nodes)
        self.round = 0
        self.completed = 0
        self.converged = False
        self.trace = []
        A = self.A
        if algo == GOSSIP:
            self.cnt = [0] * A
            self.tok = [0] * A
            self.done = [False] * A
            if topology == FULL:  # CallChildActor to the leader (program.fs:218)
                self.cnt[self.leader] = 1
            self.tok[self.leader] = 1  # first receipt or ActivateChildActor (:181, :258, :323)
        else:
            self.S = [float(v) for v in range(A)]  # InitializeVariables (:107-108)
            self.W = [1.0] * A  # :78
            self.term = [term_init if self.deg(v) > 0 else 0 for v in range(A)]  # :79
            self.conv = [False] * A
            self.Sin = [0.0] * A
            self.Win = [0.0] * A
            self.cin = [0] * A
            self.msg = [None] * A

    def deg(self, v):
        return self.nodes if self.topology == FULL else len(self.nb[v])

    def nbr(self, v, k):
        return k + (1 if k >= v else 0) if self.topology == FULL else self.nb[v][k]

    def _gossip_round(self):
        r, A = self.round, self.A
        words = draw_words(self.seed, "gossip", r, range(A))
        inc = [0] * A
        for v in range(A):
            d = self.deg(v)
            for k in range(self.tok[v]):
                if d == 0:
                    break
                t = self.nbr(v, scale(words[k][v], d))
                if not self.done[t]:  # program.fs:92 (round-start flags)
                    inc[t] += 1
        newly = 0
        for v in range(A):
            c0 = self.cnt[v]
            c1 = c0 + inc[v]
            self.cnt[v] = c1
            if c0 == 0 and c1 > 0:  # :99-100
                self.tok[v] += 1
            if c0 <= self.thr < c1:  # :102-104 (report on receipt number thr+1)
                self.done[v] = True
                newly += 1
        return newly

    def _pushsum_round(self):
        r, A = self.round, self.A
        w0 = draw_words(self.seed, "push", r, range(A))[0]
        newly = 0
        msgs = [None] * A
        for v in range(A):
            d = self.deg(v)
            if d == 0:
                continue
            if self.conv[v]:  # :125-127 relay
                if self.cin[v] > 0:
                    msgs[v] = (self.nbr(v, scale(w0[v], d)), self.Sin[v], self.Win[v])
                continue
            S, W = self.S[v], self.W[v]
            nS, nW = S + self.Sin[v], W + self.Win[v]
            if self.cin[v] > 0:
                cal = abs(S / W - nS / nW)  # :123
                self.term[v] = 0 if cal > self.delta else self.term[v] + 1
                if self.term[v] == self.term_limit:  # :135-138
                    self.term[v] = 0
                    self.conv[v] = True
                    newly += 1
            self.S[v], self.W[v] = nS / 2.0, nW / 2.0
            msgs[v] = (self.nbr(v, scale(w0[v], d)), self.S[v], self.W[v])
        Sin, Win, cin = [0.0] * A, [0.0] * A, [0] * A
        for u in range(A):  # ascending source id, accumulated from +0.0
            if msgs[u] is not None:
                t, s, w = msgs[u]
                Sin[t] += s
                Win[t] += w
                cin[t] += 1
        self.Sin, self.Win, self.cin, self.msg = Sin, Win, cin, msgs
        return newly

    def step(self, max_rounds):
        for _ in range(max_rounds):
            if self.converged:
                break
            newly = self._gossip_round() if self.algo == GOSSIP else self._pushsum_round()
            self.completed += newly
            self.trace.append(self.completed)
            self.round += 1
            if self.completed >= self.nodes:  # ParentActor :49, :56
                self.converged = True

    def state(self):
        if self.algo == GOSSIP:
            flags = [(t & 3) | (4 if d else 0) for t, d in zip(self.tok, self.done)]
            return {"cnt": np.array(self.cnt, np.uint32), "flags": np.array(flags, np.uint8)}
        flags = [(t & 15) | (16 if c else 0) for t, c in zip(self.term, self.conv)]
        dst = [NONE if m is None else m[0] for m in self.msg]
        ms = [0.0 if m is None else m[1] for m in self.msg]
        mw = [0.0 if m is None else m[2] for m in self.msg]
        return {
            "S": np.array(self.S, np.float64),
            "W": np.array(self.W, np.float64),
            "flags": np.array(flags, np.uint8),
            "msg_dst": np.array(dst, np.uint32),
            "msg_s": np.array(ms, np.float64),
            "msg_w": np.array(mw, np.float64),
        }
