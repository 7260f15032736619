"""GPU parity of ad_max_conflicts (CommandStore.preaccept's witnessedAt proposal, local/CommandStore.java:322-347)
against the oracle (oracle.cpp Oracle::max_conflict), bit-exact: per view and txn the rank holding
maxConflicts.get(keys) and the fast-path flag.  Full sizes: a txn's answer depends only on txns with a smaller
TxnId, so the oracle on a prefix must equal the GPU's first rows of the full batch.
"""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, engine, workload
from batchkit import T, make_batch

pytestmark = pytest.mark.gpu


def _slice(b, m):
    """The first m txns of a key batch (TxnId order = arrival order)."""
    ko = b["key_off"][:m + 1]
    out = {"n": m, "key_off": ko.copy(), "keys": b["keys"][:int(ko[-1])].copy(),
           "range_off": None, "range_start": None, "range_end": None}
    for f in ("txn_msb", "txn_lsb", "txn_node", "exec_msb", "exec_lsb", "exec_node", "status"):
        out[f] = b[f][:m].copy()
    return out


def check(engine_factory, b, window=32, replicas=3, drop_p=0.1, seed=0xACC0D1, prefix=None, eng=None):
    cfg = abi.make_config(window, replicas, drop_p, seed)
    if eng is None:
        eng = engine_factory(window=window, replicas=replicas, drop_p=drop_p, seed=seed)
    eng.load(b)
    eng.preaccept_deps()
    rank, fast = eng.max_conflicts()
    m = b["n"] if prefix is None else min(prefix, b["n"])
    want_rank, want_fast = O.max_conflicts(_slice(b, m) if m < b["n"] else b, cfg)
    bad = np.nonzero((rank[:, :m] != want_rank).any(axis=0))[0]
    assert len(bad) == 0, "max_rank differs at txns %s: gpu %s cpu %s" % (bad[:8], rank[:, bad[:4]], want_rank[:, bad[:4]])
    assert np.array_equal(fast[:, :m], want_fast)
    return eng, rank, fast


@pytest.mark.parametrize("name,n", [("C2", 20000), ("C3", 20000), ("C2", 200000)])
def test_configs(engine_factory, name, n):
    _, rank, fast = check(engine_factory, workload.config(name, n=n))
    assert (rank != abi.AD_RANK_NONE).any()
    if name == "C3":
        assert fast.min() == 0          # Zipf hot keys: slow-path bumps above later TxnIds (594 rows at 20k)


@pytest.mark.parametrize("window,replicas,drop_p", [(0, 1, 0.0), (32, 1, 0.0), (32, 5, 0.3), (200, 8, 0.5)])
def test_window_views_drops(engine_factory, window, replicas, drop_p):
    b = workload.generate(30000, keys_per_txn=4, keyspace=20000, slow_frac=0.3, bump_max=200, seed=window + replicas)
    check(engine_factory, b, window=window, replicas=replicas, drop_p=drop_p)


def test_kinds_statuses_and_wide_txns(engine_factory):
    rng = np.random.default_rng(5)
    n = 20000
    kinds = rng.integers(0, 5, size=n)                  # Read, Write, EphemeralRead, SyncPoint, ExclusiveSyncPoint
    status = rng.integers(0, 8, size=n).astype(np.uint8)  # every InternalStatus
    b = workload.generate(n, keys_per_txn=20, keyspace=30000, kinds=kinds, status=status, slow_frac=0.4,
                          bump_max=100, seed=6)             # 20 keys > KMAX: the large-txn pairs as well
    check(engine_factory, b)


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 4097])
def test_edge_sizes(engine_factory, n):
    check(engine_factory, workload.generate(n, keys_per_txn=2, keyspace=5, seed=n))


def test_after_merge_and_levels(engine_factory):
    # the sorted entries the kernels read survive Deps.merge and the level stage
    b = workload.config("C3", n=20000, seed=11)
    eng = engine_factory()
    eng.load(b)
    eng.preaccept_deps()
    r0, f0 = eng.max_conflicts()
    r0, f0 = r0.copy(), f0.copy()
    eng.merge()
    eng.exec_levels()
    r1, f1 = eng.max_conflicts()
    assert np.array_equal(r0, r1) and np.array_equal(f0, f1)


def test_call_order_and_carry_validation(engine_factory):
    eng = engine_factory()
    b = workload.generate(2000, range_frac=0.1, seed=3)
    eng.load(b)
    with pytest.raises(engine.IllegalStateException):
        eng.max_conflicts()                            # before ad_preaccept_deps
    eng.preaccept_deps()
    with pytest.raises(engine.IllegalStateException):
        eng.max_conflicts_export_ranges()              # before ad_max_conflicts(_ts)
    eng.max_conflicts()
    eng.max_conflicts_ts()                             # range txns: the carried map covers ranges too
    one = np.ones(2, np.uint64)
    for s_, e_ in (([5, 3], [6, 9]), ([1, 4], [5, 8]), ([4, 9], [4, 12])):   # unsorted, overlapping, empty
        with pytest.raises(engine.AccordDepsError) as e:
            eng.max_conflicts_carry_ranges((np.array(s_, np.uint64), np.array(e_, np.uint64), one, one,
                                            np.ones(2, np.int32)))
        assert e.value.rc == abi.AD_ERR_ARGUMENT


@pytest.mark.parametrize("n,keyspace,rf,width,window,replicas,drop", [(3000, 3000, 0.2, 200, 16, 3, 0.2),
                                                                      (20000, 40000, 0.1, 400, 32, 2, 0.1),
                                                                      (4000, 500, 0.3, 50, 0, 1, 0.0)])
def test_range_footprints(engine_factory, n, keyspace, rf, width, window, replicas, drop):
    # MaxConflicts as a ReducingRangeMap: key txns vs range txns covering their keys, range txns vs the keys inside
    # and the ranges crossing them (k_mc_range_keys / k_mc_range_entries) — vs Oracle::max_conflict
    b = workload.generate(n, 3, keyspace, "uniform", range_frac=rf, range_width_max=width, slow_frac=0.3, bump_max=40,
                          seed=n + keyspace)
    eng = engine_factory(window=window, replicas=replicas, drop_p=drop, seed=0xC0DE)
    eng.load(b)
    eng.preaccept_deps()
    rank, fast = eng.max_conflicts()
    orank, ofast = O.max_conflicts(b, abi.make_config(window, replicas, drop, 0xC0DE))
    bad = np.nonzero((rank != orank).any(axis=0) | (fast != ofast).any(axis=0))[0]
    assert len(bad) == 0, "txns %s: gpu %s oracle %s" % (bad[:6], rank[:, bad[:6]], orank[:, bad[:6]])
    is_range = (b["txn_lsb"] & np.uint64(1)).astype(bool)
    assert (rank[:, is_range] != abi.AD_RANK_NONE).any()


@pytest.mark.parametrize("name", ["C2", "C3"])
def test_full_size_prefix(engine_factory, name):
    b = workload.config(name)                          # 1,048,576 txns
    _, rank, fast = check(engine_factory, b, prefix=60000)
    # whole batch: the named txn precedes the query; fast == TxnId >= its executeAt
    n = b["n"]
    has = rank != abi.AD_RANK_NONE
    for v in range(rank.shape[0]):
        i = np.nonzero(has[v])[0]
        j = rank[v, i].astype(np.int64)
        assert (j < i).all()
        # Timestamp.compareTo (Timestamp.java:208-217): msb unsigned, lowHlc, identity flags, node signed
        fa = (b["txn_msb"][i], b["txn_lsb"][i] >> 16, b["txn_lsb"][i] & 0x1E, b["txn_node"][i])
        fb = (b["exec_msb"][j], b["exec_lsb"][j] >> 16, b["exec_lsb"][j] & 0x1E, b["exec_node"][j])
        gt, eq = np.zeros(len(i), bool), np.ones(len(i), bool)
        for x, y in zip(fa, fb):
            gt |= eq & (x > y)
            eq &= x == y
        assert np.array_equal(fast[v, i].astype(bool), gt | eq)
        assert fast[v, ~has[v]].all()
    assert n == 1 << 20


# ---- MaxConflicts carried across batches (ad_max_conflicts_carry / _ts / _export) -------------------------------
def _engine_store(engine_factory, batches, window, replicas, drop_p, seed):
    eng = engine_factory(window=window, replicas=replicas, drop_p=drop_p, seed=seed)
    carry = None
    out = []
    for b in batches:
        eng.load(b)
        eng.preaccept_deps()
        if carry is not None:
            eng.max_conflicts_carry(carry)
        else:
            eng.max_conflicts_carry(O.EMPTY_CARRY)
        out.append(eng.max_conflicts_ts())
        carry = eng.max_conflicts_export()
        out[-1] = out[-1] + (carry,)
    return out


def test_gpu_preaccept_kat_multi_key(engine_factory):
    # PreAcceptTest.multiKeyTimestampUpdate through the engine: the later-arriving smaller TxnId sees (1, 100, ID2)
    from accord_amd import witness as Wt
    first = make_batch([T(100, abi.KIND_WRITE, [10], node=2)])
    second = make_batch([T(50, abi.KIND_WRITE, [10, 11], node=3)])
    (m1, l1, n1, f1, c1), (m2, l2, n2, f2, c2) = _engine_store(engine_factory, [first, second], 0, 1, 0.0, 1)
    assert f1[0, 0] == 1 and f2[0, 0] == 0
    assert (int(m2[0, 0]), int(l2[0, 0]), int(n2[0, 0])) == Wt.from_values(1, 100, abi.KIND_WRITE << 1, 2)
    # the node clock as PreAcceptTest builds it (test_oracle_preaccept_kats.test_multi_key_timestamp_update): Node.now
    # made at epoch 0, the HLC 10 ahead, so nowAtLeast takes the max conflict's bits, flags included
    clock = Wt.NodeClock(1, 1, 100, now_epoch=0)
    clock.clock += 10
    w = Wt.preaccept_witnessed_at(Wt.from_values(1, 50, abi.KIND_WRITE << 1, 3), (int(m2[0, 0]), int(l2[0, 0]), int(n2[0, 0])), clock)
    assert (Wt.epoch(w), Wt.hlc(w), w[2]) == (1, 110, 1)
    # PreAcceptOk.equals -> Timestamp.equals (Timestamp.java:244-249): the identity flags (kind, domain) included
    assert Wt.equals(w, Wt.from_values(1, 110, abi.KIND_WRITE << 1, 1))
    assert not Wt.equals(w, Wt.from_values(1, 110, 0, 1))


@pytest.mark.parametrize("keyspace,window,replicas,drop", [(40, 0, 1, 0.0), (300, 16, 3, 0.2), (5000, 32, 2, 0.1)])
def test_gpu_carry_chain_equals_oracle(engine_factory, keyspace, window, replicas, drop):
    # five consecutive batches of one store: every batch's maxConflicts timestamps / fast flags and the carried map
    # after it equal the oracle's, bit for bit
    batches = [workload.generate(3000, keys_per_txn=3, keyspace=keyspace, seed=100 + k, slow_frac=0.3, bump_max=50,
                                 hlc_start=1_000_000 + 40_000 * k) for k in range(5)]
    got = _engine_store(engine_factory, batches, window, replicas, drop, 0xC0FFEE)
    cfg = abi.make_config(window, replicas, drop, 0xC0FFEE)
    carry = None
    for b, (m, l, n_, f, exp) in zip(batches, got):
        om, ol, on, fast = O.max_conflicts_ts(b, cfg, carry)
        assert np.array_equal(m, om) and np.array_equal(l, ol) and np.array_equal(n_, on) and np.array_equal(f, fast)
        carry = O.max_conflicts_export(b, carry)
        assert all(np.array_equal(x, y) for x, y in zip(exp, carry))
    assert carry[0].size > 0


@pytest.mark.parametrize("name,window,drop", [("C3", 32, 0.2), ("C2", 32, 0.1), ("C3", 0, 0.0)])
def test_gpu_fast_path_merge(engine_factory, name, window, drop):
    # CoordinateTransaction.onPreAccepted :75 — the fast-path merge folds only the replies with witnessedAt == TxnId:
    # ad_merge_deps_fast with the fast flags of ad_max_conflicts equals the oracle's merge under the same mask
    b = workload.config(name, n=20000)
    R = 3
    eng = engine_factory(window=window, replicas=R, drop_p=drop, seed=0x51DE)
    eng.load(b)
    eng.preaccept_deps()
    _, fast = eng.max_conflicts()
    eng.merge_fast()
    ref = O.OracleResult(b, abi.make_config(window, R, drop, 0x51DE), O.FLAG_MERGE, view_mask=fast)
    for c in range(abi.NUM_CLASSES):
        assert eng.fetch_merged(c).equal(ref.merged(c)), "class %d" % c
    if name == "C3":
        assert fast.min() == 0 and fast.max() == 1        # both outcomes exercised
    # the slow path (all replies) on the same handle afterwards
    eng.merge()
    full = O.OracleResult(b, abi.make_config(window, R, drop, 0x51DE), O.FLAG_MERGE)
    assert eng.fetch_merged(abi.CLASS_KEY).equal(full.merged(abi.CLASS_KEY))


# ---- the carried map's range part: intervals (s, e] from range txns (ad_max_conflicts_carry_ranges / _export_ranges)
def _store_chain(engine_factory, batches, cfg_args, carry_k=None, carry_r=None):
    eng = engine_factory(window=cfg_args[0], replicas=cfg_args[1], drop_p=cfg_args[2], seed=cfg_args[3])
    out = []
    for b in batches:
        eng.load(b)
        eng.preaccept_deps()
        eng.max_conflicts_carry(O.EMPTY_CARRY if carry_k is None else carry_k)
        eng.max_conflicts_carry_ranges(O.EMPTY_CARRY_RANGES if carry_r is None else carry_r)
        ts = tuple(a.copy() for a in eng.max_conflicts_ts())
        carry_k = tuple(a.copy() for a in eng.max_conflicts_export())
        carry_r = tuple(a.copy() for a in eng.max_conflicts_export_ranges())
        out.append((ts, carry_k, carry_r))
    return out


def _mixed_batch(n, keyspace, width, seed, hlc_start):
    rng = np.random.default_rng(seed)
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT,
                        abi.KIND_EXCLUSIVE_SYNC_POINT], p=[0.35, 0.35, 0.1, 0.1, 0.1], size=n)
    status = rng.integers(0, 8, size=n).astype(np.uint8)
    return workload.generate(n, keys_per_txn=3, keyspace=keyspace, range_frac=0.2, range_width_max=width, seed=seed,
                             slow_frac=0.3, bump_max=400, kinds=kinds, status=status, hlc_start=hlc_start)


@pytest.mark.parametrize("n,keyspace,width,window,replicas,drop", [(3000, 2000, 100, 16, 3, 0.2),
                                                                   (6000, 50000, 3000, 32, 2, 0.1),
                                                                   (2000, 1 << 44, 1 << 38, 0, 1, 0.0)])
def test_gpu_range_carry_chain_equals_oracle(engine_factory, n, keyspace, width, window, replicas, drop):
    # four batches of one store with key AND range txns: every batch's maxConflicts timestamps / fast flags and
    # both tables after it equal the oracle's (the last case spreads the breakpoints beyond 32 bits: two LSD passes)
    batches = [_mixed_batch(n, keyspace, width, 300 + k, 1_000_000 + 80_000 * k) for k in range(4)]
    cfg_args = (window, replicas, drop, 0xCAFE)
    got = _store_chain(engine_factory, batches, cfg_args)
    cfg = abi.make_config(*cfg_args)
    ck = cr = None
    for k, (b, (ts, gk, gr)) in enumerate(zip(batches, got)):
        want = O.max_conflicts_ts(b, cfg, ck, cr)
        for x, y, name in zip(ts, want, ("msb", "lsb", "node", "fast")):
            bad = np.nonzero((x != y).any(axis=0))[0]
            assert len(bad) == 0, "batch %d %s differs at txns %s" % (k, name, bad[:8])
        ck = O.max_conflicts_export(b, ck)
        cr = O.max_conflicts_export_ranges(b, cr)
        assert all(np.array_equal(x, y) for x, y in zip(gk, ck)), "batch %d key table" % k
        assert len(gr[0]) == len(cr[0]), "batch %d: %d pieces vs oracle %d" % (k, len(gr[0]), len(cr[0]))
        assert all(np.array_equal(x, y) for x, y in zip(gr, cr)), "batch %d intervals" % k
    assert cr[0].size > 0 and ck[0].size > 0
    is_range = (batches[-1]["txn_lsb"] & np.uint64(1)).astype(bool)
    assert (got[-1][0][3][:, is_range] == 0).any()     # range txns pushed off the fast path by the carry


def test_gpu_range_carry_seeded_and_empty(engine_factory):
    # a host-seeded interval table (no range txns in the batch) passes through the export unchanged but normalised;
    # a batch of key txns stabs it; an empty map exports nothing
    rng = np.random.default_rng(9)
    cuts = np.unique(rng.integers(0, 5000, size=400)).astype(np.uint64)
    s_, e_ = cuts[0:-1:2], cuts[1::2]
    k = min(len(s_), len(e_))
    s_, e_ = s_[:k], e_[:k]
    h = (1_000_000 + rng.integers(0, 3, size=k)).astype(np.uint64)     # few values: equal neighbours coalesce
    msb = np.full(k, 1 << 16, np.uint64)
    lsb = (h << np.uint64(16)) | np.uint64(abi.KIND_WRITE << 1 | 1)
    node = np.ones(k, np.int32)
    carry_r = (s_, e_, msb, lsb, node)
    b = workload.generate(3000, keys_per_txn=2, keyspace=5000, seed=10, hlc_start=900_000)
    got = _store_chain(engine_factory, [b], (0, 1, 0.0, 1), None, carry_r)
    cfg = abi.make_config(0, 1, 0.0, 1)
    want = O.max_conflicts_ts(b, cfg, None, carry_r)
    assert all(np.array_equal(x, y) for x, y in zip(got[0][0], want))
    assert (got[0][0][3] == 0).any()
    wr = O.max_conflicts_export_ranges(b, carry_r)
    assert all(np.array_equal(x, y) for x, y in zip(got[0][2], wr))
    empty = _store_chain(engine_factory, [b], (0, 1, 0.0, 1))
    assert empty[0][2][0].size == 0
