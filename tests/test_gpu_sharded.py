"""GPU parity of the multi-GPU engine: several HIP shards of one graph (gp_create_shard) on
one MI355X, exchanging through the in-process LoopbackTransport (the same chunks RCCL carries
between GPUs), against the single-process CPU oracle and the single-GPU engine — bit-exact
(completion trace, convergence round, every actor's state and last-round messages)."""
import numpy as np
import pytest

import oracle
from gossip_amd import GossipError, Simulator, sharded
from helpers import bits

pytestmark = pytest.mark.gpu


def _shards(n, topo, algo, world, seed, **kw):
    return [sharded.HipShard(n, topo, algo, rank=r, world=world, seed=seed, **kw) for r in range(world)]


def _check_vs(ref, engines, algo):
    """ref: OracleSim or Simulator over the whole graph; engines: the shards."""
    rt = ref.read_trace()
    if algo == "gossip":
        cnt, flags = ref.read_gossip()
    else:
        S, W, flags = ref.read_pushsum()
        d, s, w = ref.read_messages()
    for e in engines:
        np.testing.assert_array_equal(e.read_trace(), rt)
        lo, hi = e.lo, e.hi
        if algo == "gossip":
            c, f = e.read_gossip()
            np.testing.assert_array_equal(c, cnt[lo:hi])
            np.testing.assert_array_equal(f, flags[lo:hi])
        else:
            eS, eW, ef = e.read_pushsum()
            np.testing.assert_array_equal(ef, flags[lo:hi])
            np.testing.assert_array_equal(bits(eS), bits(S[lo:hi]))
            np.testing.assert_array_equal(bits(eW), bits(W[lo:hi]))
            ed, es, ew = e.read_messages()
            np.testing.assert_array_equal(ed, d[lo:hi])
            np.testing.assert_array_equal(bits(es), bits(s[lo:hi]))
            np.testing.assert_array_equal(bits(ew), bits(w[lo:hi]))


CASES = [
    (1000, "Imp3D", "push-sum", 1, None),
    (200, "Imp3D", "push-sum", 2, None),
    (200, "3D", "push-sum", 3, None),
    (200, "line", "push-sum", 2, 300),
    (50, "2D", "push-sum", 3, 400),
    (1000, "full", "gossip", 1, None),
    (1000, "Imp3D", "gossip", 3, None),
    (133, "Imp3D", "gossip", 2, None),
    (200, "line", "gossip", 3, None),
    (64, "2D", "gossip", 2, None),
    (200, "3D", "gossip", 1, None),
]


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[2]}-{c[1]}-{c[0]}")
def test_shards_vs_oracle(case, world):
    n, topo, algo, seed, cap = case
    try:
        bounds = sharded.partition(n, topo, world)
    except GossipError as e:
        if "cannot be split" not in str(e):
            raise
        pytest.skip(str(e))
    cap = cap or 1 << 30
    ref = oracle.OracleSim(n, topo, algo, seed=seed)
    engines = _shards(n, topo, algo, world, seed)
    assert [e.lo for e in engines] + [engines[-1].hi] == bounds
    # stop at intermediate rounds too (batch boundaries, gossip's one-round count lag)
    for chunk in (1, 5, cap):
        rs = ref.step(chunk)
        sts = sharded.run_local(engines, max_rounds=int(rs.round) - int(engines[0].status.round))
        for st in sts:
            assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
        _check_vs(ref, engines, algo)
        if rs.converged:
            break
    if algo == "push-sum":  # conservation over the shards: sum w = participants
        sw = sum(st.sum_w for st in sts)
        assert sw == pytest.approx(ref.layout.participants, rel=1e-12)
    for e in engines:
        e.close()


@pytest.mark.parametrize("n,topo,algo,world,rounds", [
    (100000, "Imp3D", "push-sum", 4, None),
    (100000, "3D", "push-sum", 3, 300),
    (100000, "full", "gossip", 3, None),
    (100000, "Imp3D", "gossip", 2, None),
])
def test_shards_vs_single_gpu_100k(n, topo, algo, world, rounds):
    cap = rounds or 1 << 30
    ref = Simulator(n, topo, algo, seed=5)
    rs = ref.step(cap)
    engines = _shards(n, topo, algo, world, seed=5)
    sts = sharded.run_local(engines, max_rounds=cap)
    assert (sts[0].round, sts[0].completed, sts[0].converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, algo)


@pytest.mark.parametrize("n,topo,algo,rounds", [
    (2_000_000, "Imp3D", "push-sum", None),   # 7/8 of the links remote, both halo sides
    (1_000_000, "3D", "push-sum", 400),
    (1_000_000, "full", "gossip", None),      # every receipt an entry, 7 peers
    (1_000_000, "Imp3D", "gossip", None),
])
def test_shards_vs_single_gpu_world8(n, topo, algo, rounds):
    """The driver's 8-rank layout (8 shards on one GPU, loopback exchange): every peer's
    sub-segments, the owner() search over 8 bounds and the middle ranks' two halo faces, bit
    for bit against the single-GPU engine."""
    cap = rounds or 1 << 30
    ref = Simulator(n, topo, algo, seed=7)
    rs = ref.step(cap)
    engines = _shards(n, topo, algo, 8, seed=7)
    sts = sharded.run_local(engines, max_rounds=cap)
    assert (sts[0].round, sts[0].completed, sts[0].converged) == (rs.round, rs.completed, rs.converged)
    np.testing.assert_array_equal(engines[0].read_trace(), ref.read_trace())
    _check_vs(ref, engines, algo)


# The quiet-tail walk on shards: once 99% of the nodes have converged, a rank
# walks only the 4-actor segments marked by its own round kernel (its own actors still updating,
# the targets of its own local messages) and by its unpack (the targets of the halo and link
# messages other ranks sent it).  Forced at small sizes, run to convergence, bit-exact against the
# oracle; the C3 x8 fingerprint covers the default size gate (2^20 actors per rank).
QUIET_SHARD_CASES = [
    (1000, "Imp3D", 2, 1), (20000, "Imp3D", 3, 5), (200000, "Imp3D", 4, 3), (300000, "Imp3D", 8, 11),
    (8000, "3D", 3, 2), (2000, "line", 3, 4), (3000, "2D", 2, 6), (64000, "3D", 5, 8),
]


@pytest.mark.parametrize("tiers", ["default", "tight"])
@pytest.mark.parametrize("n,topo,world,seed", QUIET_SHARD_CASES)
def test_shards_quiet_tail_vs_oracle(n, topo, world, seed, tiers):
    """tight: activity tiers from the first batch with no headroom (GP_FLAG_TIGHT_TIERS), so reduced
    chunks overflow and batches are discarded and replayed from restore points over and over: the
    run must still be exact."""
    ref = oracle.OracleSim(n, topo, "push-sum", seed=seed)
    rs = ref.step(1 << 20, threads=8)
    engines = _shards(n, topo, "push-sum", world, seed, quiet_waves=True, tight_tiers=tiers == "tight")
    sts = sharded.run_local(engines, max_rounds=1 << 20)
    if tiers == "tight" and n >= 200000:
        ss = [e.shard_stats() for e in engines]
        assert all(x["plan_changes"] > 0 for x in ss), ss
        assert sum(x["restores"] for x in ss) > 0, ss
    assert rs.converged
    for st in sts:
        assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, "push-sum")
    # a second run after a reset: no mark of the first run may leak into it
    for e in engines:
        e.reset()
    sts = sharded.run_local(engines, max_rounds=1 << 20)
    assert (sts[0].round, sts[0].completed) == (rs.round, rs.completed)
    _check_vs(ref, engines, "push-sum")
    for e in engines:
        e.close()


def _quiet_shard_sweep(count=16, seed=99):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(count):
        topo = ("Imp3D", "3D", "line", "2D", "Imp3D")[rng.integers(5)]
        hi = 3000 if topo in ("line", "2D") else 150000
        out.append((int(np.exp(rng.uniform(np.log(64), np.log(hi)))), topo, int(rng.integers(2, 9)),
                    int(rng.integers(1, 1 << 30))))
    return out


@pytest.mark.parametrize("n,topo,world,seed", _quiet_shard_sweep())
def test_shards_quiet_tail_random_sweep(n, topo, world, seed):
    _quiet_sweep_case(n, topo, world, seed, tight=False)


@pytest.mark.parametrize("n,topo,world,seed", _quiet_shard_sweep(count=12, seed=1234))
def test_shards_tight_tiers_random_sweep(n, topo, world, seed):
    _quiet_sweep_case(n, topo, world, seed, tight=True)


def _quiet_sweep_case(n, topo, world, seed, tight):
    try:
        sharded.partition(n, topo, world)
    except GossipError as e:
        if "cannot be split" not in str(e):
            raise
        pytest.skip(str(e))
    ref = oracle.OracleSim(n, topo, "push-sum", seed=seed)
    rs = ref.step(1 << 20, threads=8)
    engines = _shards(n, topo, "push-sum", world, seed, quiet_waves=True, tight_tiers=tight)
    sts = sharded.run_local(engines, max_rounds=int(rs.round))
    for st in sts:
        assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, "push-sum")
    for e in engines:
        e.close()


def test_shards_quiet_default_and_work_count():
    """Shards of 2^20 actors or more run the quiet kernel by default (k_ps_quiet_x), which routes
    every round's link messages itself (no k_ps_link_scatter_x: no aux kernel), and count the actors
    it walks in their timed rounds only, so work_per_launch averages over the same launches as the
    kernel time: below the shard's actor count (the tail walks a few per cent of it)."""
    n, world = 4_500_000, 2
    ref = Simulator(n, "Imp3D", "push-sum", seed=3)
    rs = ref.step()
    engines = _shards(n, "Imp3D", "push-sum", world, seed=3, kernel_timing=True)
    sts = sharded.run_local(engines)
    assert (sts[0].round, sts[0].completed, sts[0].converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, "push-sum")
    for e in engines:
        ks = e.kernel_stats()
        assert ks["kernel"] == "k_ps_quiet_x", ks
        assert ks["aux_kernel"] == "", ks  # (no link pass: the round kernel routes the links)
        assert ks["launches"] == (int(rs.round) + 7) // 8, ks  # every 8th round is timed
        assert 0 < ks["work_per_launch"] < e.hi - e.lo, ks
        e.close()


def test_shards_activity_tiers_default():
    """Default activity tiers on an 8-rank run to convergence (2M Imp3D, 7/8 of the links remote):
    once half the nodes have converged, each batch's chunks are sized from the last batch's counts,
    so the tail ships a fraction of the full plan; bit-exact against the single-GPU engine and
    against the same shards with the full plan."""
    n, seed = 2_000_000, 7
    ref = Simulator(n, "Imp3D", "push-sum", seed=seed)
    rs = ref.step()
    engines = _shards(n, "Imp3D", "push-sum", 8, seed)
    full_bytes = engines[0].bytes_per_round()[0]
    t = sharded.LoopbackTransport()
    sts = [e.sync() for e in engines]
    least, batch = full_bytes, 8
    while not sts[0].converged:
        for _ in range(batch):
            for e in engines:
                e.round()
            t.exchange_all(engines)
            for e in engines:
                e.deliver()
        sts = [e.sync() for e in engines]
        least = min(least, engines[0].bytes_per_round()[0])
        batch = min(batch * 2, 64)
    assert (sts[0].round, sts[0].completed) == (rs.round, rs.completed)
    _check_vs(ref, engines, "push-sum")
    ss = [e.shard_stats() for e in engines]
    assert all(x["plan_changes"] > 0 for x in ss), ss
    assert least * 2 < full_bytes, (least, full_bytes)  # the fixed halo part and the 64-entry floor remain
    for e in engines:
        e.close()


@pytest.mark.parametrize("n,world,seed", [(1000, 2, 1), (20000, 3, 4), (100000, 5, 2), (300000, 8, 6), (2000000, 8, 3)])
def test_full_gossip_tight_tiers_vs_oracle(n, world, seed):
    """Full gossip on shards with tight activity tiers: the senders filter remote receipts on the
    replicated done bitmap, the chunks shrink with the receipts still sent, overflowed batches are
    replayed from restore points (cnt, states, receipts, the replica) — bit-exact against the oracle,
    twice (after a reset)."""
    ref = oracle.OracleSim(n, "full", "gossip", seed=seed)
    rs = ref.step(threads=8)
    engines = _shards(n, "full", "gossip", world, seed, tight_tiers=True)
    for _ in range(2):
        sts = sharded.run_local(engines)
        for st in sts:
            assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
        _check_vs(ref, engines, "gossip")
        for e in engines:
            e.reset()
    if n >= 100000:
        # sized plans overflow under tight tiers and the batches replay from restore points (the
        # counts, states, pending receipts, the replica and the shipped done words)
        ss = [e.shard_stats() for e in engines]
        assert all(x["plan_changes"] > 0 for x in ss), ss
        assert sum(x["restores"] for x in ss) > 0, ss
    for e in engines:
        e.close()


@pytest.mark.parametrize("n,world,seed", [(300000, 8, 6), (2000000, 8, 3), (1000000, 3, 9)])
def test_full_gossip_round_plans(n, world, seed):
    """Full gossip on shards sizes every round's chunks: through the ramp from the
    chain bound (chains at most double per round), after it from the last round's counts, and the
    done words as lazily shipped (index, word) pairs.  The run ships a fraction of the full plan's
    bytes, replays nothing, and is bit-exact against the single-GPU engine and the full-plan shards."""
    ref = Simulator(n, "full", "gossip", seed=seed)
    rs = ref.step()
    engines = _shards(n, "full", "gossip", world, seed)
    full_bytes = int(engines[0].shard.send_total)
    t = sharded.LoopbackTransport()
    sts = [e.sync() for e in engines]
    per_round, batch = [], 8
    while not sts[0].converged:
        for _ in range(batch):
            for e in engines:
                e.round()
            per_round.append(sum(engines[0].send_splits))
            t.exchange_all(engines)
            for e in engines:
                e.deliver()
        sts = [e.sync() for e in engines]
    assert (sts[0].round, sts[0].completed) == (rs.round, rs.completed)
    _check_vs(ref, engines, "gossip")
    ss = [e.shard_stats() for e in engines]
    assert sum(x["restores"] for x in ss) == 0, ss
    assert ss[0]["bytes_sent"] == sum(per_round)
    assert per_round[0] < full_bytes / 20 and per_round[1] <= 2 * per_round[0] + 8192, per_round[:4]  # the ramp
    assert sum(per_round) * 2 < len(per_round) * full_bytes, (sum(per_round), len(per_round), full_bytes)
    # the same run with the full plan every round: the same counts
    fp = _shards(n, "full", "gossip", world, seed, full_plan=True)
    sharded.run_local(fp)
    for a, b in zip(engines, fp):
        np.testing.assert_array_equal(a.read_gossip()[0], b.read_gossip()[0])
        np.testing.assert_array_equal(a.read_trace(), b.read_trace())
        assert b.shard_stats()["bytes_sent"] > a.shard_stats()["bytes_sent"]
    for e in engines + fp:
        e.close()


@pytest.mark.parametrize("n,world,seed", [(1000, 2, 1), (20000, 3, 4), (300000, 8, 6), (1_500_000, 5, 7)])
def test_full_gossip_shard_ramp_lists_vs_oracle(n, world, seed):
    """Full gossip's ramp on shards (k_gs_sparse_x): while every rank's chain holders
    stay within the lists' bound (1/256 of the actors, at least 64), each rank walks its own lists —
    the targets of the last round, its own receipts and the ones the peers sent (listed by the
    unpack), and its holders — then every actor.  Stopped at every round of the ramp and the switch,
    bit-exact against the oracle each time, and again after a reset."""
    ref = oracle.OracleSim(n, "full", "gossip", seed=seed)
    engines = _shards(n, "full", "gossip", world, seed)
    for rep in range(2):
        if rep:
            ref = oracle.OracleSim(n, "full", "gossip", seed=seed)
            for e in engines:
                e.reset()
        for chunk in (1, 1, 1, 2, 3, 5, 8, 13, 21, 1 << 20):
            rs = ref.step(chunk, threads=8)
            sts = sharded.run_local(engines, max_rounds=int(rs.round) - int(engines[0].status.round))
            for st in sts:
                assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
            _check_vs(ref, engines, "gossip")
            if rs.converged:
                break
        assert rs.converged
        lists = [e.shard_stats()["list_rounds"] for e in engines]
        # the ramp ran on lists on every rank (the same rounds: the bound is global), not the whole run
        assert len(set(lists)) == 1 and 4 <= lists[0] < int(rs.round), (lists, int(rs.round))
    for e in engines:
        e.close()


@pytest.mark.parametrize("tiers", ["default", "tight", "full"])
@pytest.mark.parametrize("n,world,seed", [(1000, 2, 2), (20000, 3, 4), (100000, 8, 5), (300000, 5, 8)])
def test_full_gossip_shard_bins_vs_oracle(n, world, seed, tiers):
    """Full gossip's receipts in bins on shards (k_gs_bins_count / k_gs_bins_place / k_shard_unpack_bins,
    DESIGN.md §6.15), forced in every round after the ramp's lists: the sender counts each (peer, bin)
    per workgroup, places u16 offsets after a scan, and the receiver counts a bin per workgroup and adds
    to its receipt words.  No sender-side filter in these rounds.  With the three plans (per-round,
    tight: overflowed batches replay from restore points, full), stopped at several rounds, bit-exact
    against the oracle, twice (after a reset)."""
    kw = {"tight_tiers": True} if tiers == "tight" else {"full_plan": True} if tiers == "full" else {}
    engines = _shards(n, "full", "gossip", world, seed, force_bins=True, **kw)
    for rep in range(2):
        ref = oracle.OracleSim(n, "full", "gossip", seed=seed)
        if rep:
            for e in engines:
                e.reset()
        for chunk in (3, 5, 8, 13, 1 << 20):
            rs = ref.step(chunk, threads=8)
            sts = sharded.run_local(engines, max_rounds=int(rs.round) - int(engines[0].status.round))
            for st in sts:
                assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
            _check_vs(ref, engines, "gossip")
            if rs.converged:
                break
        assert rs.converged
        ss = [e.shard_stats() for e in engines]
        assert all(x["bin_rounds"] > 0 for x in ss), ss
    for e in engines:
        e.close()


def test_full_gossip_shard_bins_default_wave():
    """Without the test hook the receipt wave runs in bins (the chain bound times the share of nodes not
    done at least actors / GP_BIN_DIV), the ramp on lists before it and entries with the sender filter
    after it: all three kinds of rounds in one run at 16M actors on 8 ranks, bit-exact against the
    single-GPU engine (the C4 x 8 fingerprint test checks the same at 100M)."""
    n, world, seed = 16_000_000, 8, 3
    ref = Simulator(n, "full", "gossip", seed=seed)
    rs = ref.step()
    engines = _shards(n, "full", "gossip", world, seed)
    sts = sharded.run_local(engines)
    assert (sts[0].round, sts[0].completed, sts[0].converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, "gossip")
    ss = [e.shard_stats() for e in engines]
    assert len({(x["bin_rounds"], x["list_rounds"]) for x in ss}) == 1, ss
    lr, br = ss[0]["list_rounds"], ss[0]["bin_rounds"]
    assert lr > 0 and br > 0 and lr + br + 1 < int(rs.round), (lr, br, int(rs.round))
    for e in engines:
        e.close()


@pytest.mark.parametrize("n,topo,world,seed", [(20000, "Imp3D", 3, 5), (300000, "Imp3D", 8, 11)])
def test_group_tight_tiers_vs_oracle(n, topo, world, seed):
    """The library's multi-GPU engine (gp_step over num_gpus shards, here on one device) with
    tight tiers: its own exchange follows the plans and replays overflowed batches."""
    gpu = Simulator(n, topo, "push-sum", seed=seed, num_gpus=world, one_device=True, quiet_waves=True,
                    tight_tiers=True)
    cpu = oracle.OracleSim(n, topo, "push-sum", seed=seed)
    gs, cs = gpu.step(), cpu.step(1 << 20, threads=8)
    assert gs.converged and (gs.round, gs.completed) == (cs.round, cs.completed)
    S, W, f = gpu.read_pushsum()
    rS, rW, rf = cpu.read_pushsum()
    np.testing.assert_array_equal(f, rf)
    np.testing.assert_array_equal(bits(S), bits(rS))
    np.testing.assert_array_equal(bits(W), bits(rW))
    np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
    gpu.close()
    cpu.close()


# Rounds in pieces, forced at small sizes: each piece's round kernel and link pass
# over its own actors, the halo faces in the end pieces, its headers and chunks, exchanged piece by
# piece on the loopback transport's own stream; the quiet tail walks each piece's segments.
PIECE_CASES = [(1000, "Imp3D", 2, 1, None), (20000, "Imp3D", 3, 5, None), (300000, "Imp3D", 8, 11, None),
               (8000, "3D", 4, 2, None), (20000, "line", 3, 4, 400), (40000, "2D", 2, 6, 400)]


@pytest.mark.parametrize("tiers", ["default", "tight"])
@pytest.mark.parametrize("n,topo,world,seed,cap", PIECE_CASES)
def test_shards_pieces_vs_oracle(n, topo, world, seed, cap, tiers):
    """tight: the per-(piece, peer) activity tiers overflow and replay from restore points."""
    ref = oracle.OracleSim(n, topo, "push-sum", seed=seed)
    rs = ref.step(cap or 1 << 20, threads=8)
    engines = _shards(n, topo, "push-sum", world, seed, quiet_waves=True, force_pieces=True,
                      tight_tiers=tiers == "tight")
    assert all(e.npieces == 4 for e in engines), [e.npieces for e in engines]
    sts = sharded.run_local(engines, max_rounds=int(rs.round))
    for st in sts:
        assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, "push-sum")
    if tiers == "tight" and n >= 20000 and cap is None:
        assert sum(e.shard_stats()["restores"] for e in engines) > 0
    for e in engines:
        e.close()


def test_group_pieces_vs_oracle():
    """The library's multi-GPU engine in pieces: each piece's exchange on the group's own stream
    (one device: copies), joined before the unpacks."""
    n, world, seed = 100000, 4, 3
    gpu = Simulator(n, "Imp3D", "push-sum", seed=seed, num_gpus=world, one_device=True, quiet_waves=True,
                    force_pieces=True)
    cpu = oracle.OracleSim(n, "Imp3D", "push-sum", seed=seed)
    gs, cs = gpu.step(), cpu.step(1 << 20, threads=8)
    assert gs.converged and (gs.round, gs.completed) == (cs.round, cs.completed)
    S, W, f = gpu.read_pushsum()
    rS, rW, rf = cpu.read_pushsum()
    np.testing.assert_array_equal(f, rf)
    np.testing.assert_array_equal(bits(S), bits(rS))
    np.testing.assert_array_equal(bits(W), bits(rW))
    np.testing.assert_array_equal(gpu.read_trace(), cpu.read_trace())
    gpu.close()
    cpu.close()


def test_shards_imp3d_10m_two_ranks():
    """BASELINE config 3 split over 2 shards (in 4 pieces each, forced: the library runs 5M-actor ranks
    in one piece): the same run as the single-GPU engine."""
    ref = Simulator(10_000_000, "Imp3D", "push-sum", seed=1)
    rs = ref.step()
    one = sharded.HipShard(10_000_000, "Imp3D", "push-sum", rank=0, world=2, seed=1)
    assert one.npieces == 1  # below 2^25 actors per rank
    one.close()
    engines = _shards(10_000_000, "Imp3D", "push-sum", 2, seed=1, force_pieces=True)
    assert all(e.npieces == 4 for e in engines)
    sts = sharded.run_local(engines)
    assert rs.converged and (sts[0].round, sts[0].completed) == (rs.round, rs.completed)
    np.testing.assert_array_equal(engines[0].read_trace(), ref.read_trace())
    for e in engines:
        S, W, f = e.read_pushsum()
        rS, rW, rf = ref.read_pushsum(e.lo, e.hi - e.lo)
        np.testing.assert_array_equal(bits(S), bits(rS))
        np.testing.assert_array_equal(bits(W), bits(rW))
        np.testing.assert_array_equal(f, rf)
    assert sum(st.sum_w for st in sts) == pytest.approx(ref.layout.participants, rel=1e-12)


def test_shard_errors():
    with pytest.raises(GossipError):
        sharded.HipShard(1000, "full", "push-sum", rank=0, world=2)  # single-GPU only
    with pytest.raises(GossipError):
        sharded.HipShard(20, "Imp3D", "push-sum", rank=0, world=4)  # 2 planes for 4 ranks
    e = sharded.HipShard(1000, "Imp3D", "push-sum", rank=0, world=2)
    with pytest.raises(GossipError):
        e.deliver()  # deliver before round
    buf = np.zeros(4, np.float64)
    p = buf.ctypes.data_as(sharded.C.c_void_p)
    assert e.lib.gp_read_pushsum(e.h, e.hi, 1, p, p, None) == -1  # another rank's actor
    assert e.lib.gp_step(e.h, 1, None) == -4  # a shard advances with gp_shard_round
    e.close()


def _sweep_cases(count=40, seed=7):
    """Seeded random (n, topology, algorithm, seed, world) draws for the shard engine: sizes
    log-uniform over 64..200000, 2..8 ranks (push-sum on "full" is single-GPU only)."""
    rng = np.random.default_rng(seed)
    topos = sorted(oracle.TOPOLOGIES)
    out = []
    while len(out) < count:
        n = int(np.exp(rng.uniform(np.log(64), np.log(200000))))
        topo, algo = topos[rng.integers(len(topos))], ("gossip", "push-sum")[rng.integers(2)]
        case = (n, topo, algo, int(rng.integers(1, 1 << 30)), int(rng.integers(2, 9)))
        if not (topo == "full" and algo == "push-sum"):
            out.append(case)
    return out


@pytest.mark.parametrize("n,topo,algo,seed,world", _sweep_cases())
def test_shards_random_sweep(n, topo, algo, seed, world):
    """Loopback shards bit-exact against the oracle over random configurations (2000 rounds max)."""
    try:
        sharded.partition(n, topo, world)
    except GossipError as e:
        if "cannot be split" not in str(e):
            raise
        pytest.skip(str(e))
    ref = oracle.OracleSim(n, topo, algo, seed=seed)
    engines = _shards(n, topo, algo, world, seed)
    rs = ref.step(2000, threads=8)
    sts = sharded.run_local(engines, max_rounds=int(rs.round))
    for st in sts:
        assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, algo)
    for e in engines:
        e.close()


def _full_gossip_sweep(count=24, seed=2026):
    """Seeded random full-gossip shard jobs: sizes log-uniform over 64..1.5M, 2..8 ranks, one of the
    plans and the bins' test hook drawn per case."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(count):
        n = int(np.exp(rng.uniform(np.log(64), np.log(1_500_000))))
        out.append((n, int(rng.integers(1, 1 << 30)), int(rng.integers(2, 9)),
                    ("default", "tight", "full")[rng.integers(3)], bool(rng.integers(2))))
    return out


@pytest.mark.parametrize("n,seed,world,plan,bins", _full_gossip_sweep())
def test_full_gossip_shards_random_sweep(n, seed, world, plan, bins):
    """Full gossip on shards over random jobs, every kind of round the engine has (the ramp on lists, the
    receipt wave in bins — forced in every round past the lists when `bins` — and entries with the
    sender filter) under a random plan, bit-exact against the oracle to convergence."""
    try:
        sharded.partition(n, "full", world)
    except GossipError as e:
        if "cannot be split" not in str(e):
            raise
        pytest.skip(str(e))
    kw = {"tight_tiers": True} if plan == "tight" else {"full_plan": True} if plan == "full" else {}
    ref = oracle.OracleSim(n, "full", "gossip", seed=seed)
    rs = ref.step(threads=8)
    engines = _shards(n, "full", "gossip", world, seed, force_bins=bins, **kw)
    sts = sharded.run_local(engines)
    for st in sts:
        assert (st.round, st.completed, st.converged) == (rs.round, rs.completed, rs.converged)
    _check_vs(ref, engines, "gossip")
    ss = engines[0].shard_stats()
    assert ss["list_rounds"] > 0, ss
    if bins:
        assert ss["bin_rounds"] > 0, ss
    for e in engines:
        e.close()


def test_shard_tables_scale_with_rank_count():
    """Per-rank link tables: a rank holds the CSR of its own receivers and the
    `lpos` of its own senders, not the global tables, so its device memory is its share of the
    graph (+ two halo planes, the slot-indexed remote messages and the chunks), and the total
    over 8 ranks stays within a small factor of one GPU's.  (Round 1 kept every global link
    table on every rank: 16 B per global actor each.)"""
    n = 8_000_000
    one = Simulator(n, "Imp3D", "push-sum")
    d1 = int(one.layout.device_bytes)
    actors = one.actors
    one.close()
    ranks = [sharded.HipShard(n, "Imp3D", "push-sum", rank=r, world=8) for r in range(8)]
    per = [int(e.layout.device_bytes) for e in ranks]
    own = [e.hi - e.lo for e in ranks]
    for e in ranks:
        e.close()
    for b, o in zip(per, own):
        # own share of the single-GPU bytes, x2.5 for rmsg / halos / chunks and the activity tiers'
        # restore point (allocated at creation: ~35 B per own actor), and far below a global table of
        # 16 B per actor
        assert b < 2.5 * d1 * o / actors, (b, d1, o, actors)
        assert b < d1 / 2, (b, d1)
    assert sum(per) < 2.5 * d1, (per, d1)
