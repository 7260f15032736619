"""Oracle known answers for the witnessedAt proposal (CommandStore.preaccept, local/CommandStore.java:322-347).

maxConflicts.get(keys) (local/MaxConflicts.java:46-59) folds Timestamp::max over the executeAt of every
globally visible txn the store recorded on the keys (CommandStore.updateMaxConflicts :282-291 —
SafeCommandStore.updateMaxConflicts :210-222 skips kinds that are not globally visible); the replica answers
witnessedAt = TxnId when TxnId.compareTo(maxConflict) >= 0 (:343), else a fresh timestamp above it.
The cases below pin the oracle (oracle.cpp Oracle::max_conflict) against those rules, and an independent
pure-Python restatement on random batches.
"""
import numpy as np

import oracle as O
from accord_amd import abi, workload

from batchkit import T, make_batch

NONE = abi.AD_RANK_NONE
R, W = abi.KIND_READ, abi.KIND_WRITE


def run(txns, window=0, replicas=1, drop_p=0.0):
    b = make_batch(txns)
    return O.max_conflicts(b, abi.make_config(window, replicas, drop_p, 7))


def test_first_txn_has_no_conflict():
    rank, fast = run([T(10, W, [1]), T(20, R, [2])])
    assert list(rank[0]) == [NONE, NONE] and list(fast[0]) == [1, 1]


def test_fast_path_below_and_slow_path_above():
    # A committed at its TxnId: B (later TxnId) takes the fast path; C committed at a later executeAt (slow path
    # bump beyond D's TxnId) forces D off the fast path (TxnId < maxConflict)
    rank, fast = run([T(10, W, [1]), T(20, R, [1]), T(30, W, [2], exec_hlc=50), T(40, R, [2])])
    assert list(rank[0]) == [NONE, 0, NONE, 2]
    assert list(fast[0]) == [1, 1, 1, 0]


def test_every_globally_visible_kind_counts_not_ephemeral_reads():
    # Reads conflict with Reads for MaxConflicts (no witness filter, CommandStore.java:341 TODO); an
    # EphemeralRead is not globally visible (SafeCommandStore.java:218-219) and never recorded
    rank, fast = run([T(10, R, [1], exec_hlc=90), T(20, abi.KIND_EPHEMERAL_READ, [1], exec_hlc=95),
                      T(30, abi.KIND_SYNC_POINT, [1]), T(40, R, [1])])
    assert list(rank[0]) == [NONE, 0, 0, 0]
    assert list(fast[0]) == [1, 0, 0, 0]


def test_unrecorded_statuses_are_skipped():
    # TRANSITIVELY_KNOWN (no local definition: keysOrRanges null, CommandStore.java:286-287) and INVALID
    # entries do not raise maxConflicts
    rank, _ = run([T(10, W, [1], exec_hlc=90, status=abi.ST_TRANSITIVELY_KNOWN),
                   T(20, W, [1], exec_hlc=80, status=abi.ST_INVALID), T(30, W, [1], exec_hlc=35), T(40, R, [1])])
    assert list(rank[0]) == [NONE, NONE, NONE, 2]


def test_max_over_all_keys_and_ties_to_larger_rank():
    txns = [T(10, W, [1], exec_hlc=60), T(12, W, [2], exec_hlc=60), T(14, W, [3], exec_hlc=99), T(20, R, [1, 2])]
    rank, fast = run(txns)
    assert rank[0][3] == 1 and fast[0][3] == 0       # equal executeAt (Timestamp.equals): the larger rank
    rank, _ = run(txns[:3] + [T(20, R, [1, 3])])
    assert rank[0][3] == 2


def test_in_flight_window_and_drops():
    # j in [i - W, i) is PreAccepted from i's viewpoint whatever its final status: recorded by every view that
    # did not drop it; drop_p = 1 drops every in-flight txn, leaving only the out-of-window prefix (j = 0 for i = 2)
    txns = [T(10, W, [1], exec_hlc=70), T(20, W, [1], exec_hlc=80, status=abi.ST_INVALID), T(30, R, [1])]
    rank, _ = run(txns, window=1, replicas=1)
    assert list(rank[0]) == [NONE, 0, 1]             # j = 1 in flight for i = 2: counted despite INVALID
    rank, _ = run(txns, window=1, replicas=2, drop_p=1.0)
    assert list(rank[0]) == [NONE, NONE, 0] and list(rank[1]) == [NONE, NONE, 0]


M64 = (1 << 64) - 1


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _drop_hash(seed, view, i, j):   # include/accord_deps.h ad_drop_hash
    return _mix64(seed ^ _mix64(((view << 56) ^ (i << 28) ^ j) & M64)) >> 32


def _drop_threshold(p):              # include/accord_deps.h ad_drop_threshold
    if p <= 0.0:
        return 0
    if p >= 1.0:
        return 0xFFFFFFFF
    return int(float(np.float32(p)) * 4294967296.0)


def _model(b, cfg):
    """Independent restatement straight from the rules above (no CFK structures)."""
    n = b["n"]
    ts = lambda m, l, node: (int(m), int(l) >> 16, int(l) & 0x1E, int(node))
    tx = [ts(b["txn_msb"][i], b["txn_lsb"][i], b["txn_node"][i]) for i in range(n)]
    ex = [ts(b["exec_msb"][i], b["exec_lsb"][i], b["exec_node"][i]) for i in range(n)]
    kind = [(int(b["txn_lsb"][i]) >> 1) & 7 for i in range(n)]
    keys = [set(int(k) for k in b["keys"][b["key_off"][i]:b["key_off"][i + 1]]) for i in range(n)]
    ranges = [[] for _ in range(n)]
    if b.get("range_off") is not None:
        ro = b["range_off"]
        ranges = [[(int(b["range_start"][q]), int(b["range_end"][q])) for q in range(ro[i], ro[i + 1])] for i in range(n)]

    def overlaps(i, j):
        # MaxConflicts is a ReducingRangeMap: keys are points, ranges (start, end] intervals
        if keys[i] & keys[j]:
            return True
        if any(s < k <= e for (s, e) in ranges[j] for k in keys[i]):
            return True
        if any(s < k <= e for (s, e) in ranges[i] for k in keys[j]):
            return True
        return any(not (a1 >= b2 or b1 <= a2) for (a1, b1) in ranges[i] for (a2, b2) in ranges[j])
    thresh = _drop_threshold(cfg.drop_p)
    R_ = cfg.replicas
    rank = np.full((R_, n), NONE, np.uint32)
    fast = np.ones((R_, n), np.uint8)
    for v in range(R_):
        for i in range(n):
            best = None
            for j in range(i):
                if kind[j] not in (abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT):
                    continue
                if not overlaps(i, j):
                    continue
                in_flight = cfg.window > 0 and j + cfg.window >= i
                if in_flight:
                    if thresh and _drop_hash(cfg.seed, v, i, j) < thresh:
                        continue
                elif int(b["status"][j]) in (abi.ST_TRANSITIVELY_KNOWN, abi.ST_INVALID):
                    continue
                if best is None or (ex[j], j) > (ex[best], best):
                    best = j
            if best is not None:
                rank[v, i] = best
                fast[v, i] = 1 if tx[i] >= ex[best] else 0
    return rank, fast


def test_oracle_equals_independent_model():
    for seed, keyspace in ((3, 50), (4, 200), (5, 20)):
        b = workload.generate(300, keys_per_txn=3, keyspace=keyspace, seed=seed, slow_frac=0.3, bump_max=40)
        cfg = abi.make_config(8, 2, 0.3, 0xBEEF + seed)
        rank, fast = O.max_conflicts(b, cfg)
        mr, mf = _model(b, cfg)
        assert np.array_equal(rank, mr) and np.array_equal(fast, mf)
        assert fast.min() == 0 and (rank != NONE).any()     # both outcomes exercised


def test_oracle_equals_independent_model_with_ranges():
    # range footprints: key txns vs range txns covering their keys, range txns vs keys inside / ranges crossing
    for seed in (6, 7):
        b = workload.generate(300, keys_per_txn=2, keyspace=400, range_frac=0.25, range_width_max=60, seed=seed,
                              slow_frac=0.3, bump_max=40)
        cfg = abi.make_config(8, 2, 0.3, 0xBEEF + seed)
        rank, fast = O.max_conflicts(b, cfg)
        mr, mf = _model(b, cfg)
        assert np.array_equal(rank, mr) and np.array_equal(fast, mf)
        is_range = (b["txn_lsb"] & np.uint64(1)).astype(bool)
        assert (rank[:, is_range] != NONE).any() and fast.min() == 0


def test_reduce_witnessed_across_stores():
    # PreAccept.reduce (messages/PreAccept.java:141-156) of per-store answers: with the snapshot model (W = 0, no
    # drops) each store's answer depends only on its own keys, so the oracle per key-range slice, folded by
    # sharding.reduce_witnessed, must equal the oracle on the whole batch
    from accord_amd import sharding
    b = workload.generate(3000, keys_per_txn=4, keyspace=400, seed=8, slow_frac=0.4, bump_max=300)
    cfg = abi.make_config(0, 2, 0.0, 1)
    want_rank, want_fast = O.max_conflicts(b, cfg)
    for shards in (2, 3, 5):
        bounds = sharding.even_bounds(0, 400, shards)
        parts = []
        for k in range(shards):
            local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            rank, fast = O.max_conflicts(local, cfg)
            g = np.where(rank != NONE, gid[np.where(rank != NONE, rank, 0)], NONE).astype(np.uint32)
            parts.append((gid, g, fast))
        got_rank, got_fast, _ = sharding.reduce_witnessed(b, parts)
        assert np.array_equal(got_rank, want_rank) and np.array_equal(got_fast, want_fast)
    assert want_fast.min() == 0


# ---- the carried map's range part (ad_max_conflicts_carry_ranges / _export_ranges) -------------------------------
def _order(msb, lsb, node):
    """Timestamp.compareTo key (Timestamp.java:208-217), then raw lsb: the tie rule of the carried map."""
    return (int(msb), int(lsb) >> 16, int(lsb) & 0x1E, int(node), int(lsb))


def _recorded_ranges(b):
    """(start, end, ts) of every range the batch's recorded range txns cover (globally visible kinds, status not
    TRANSITIVELY_KNOWN / INVALID)."""
    out = []
    if b["range_off"] is None:
        return out
    for i in range(b["n"]):
        lsb = int(b["txn_lsb"][i])
        kind, dom, st = (lsb >> 1) & 0xF, lsb & 1, int(b["status"][i])
        if dom != 1 or kind not in (R, W, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT):
            continue
        if st in (abi.ST_TRANSITIVELY_KNOWN, abi.ST_INVALID):
            continue
        ts = (int(b["exec_msb"][i]), int(b["exec_lsb"][i]), int(b["exec_node"][i]))
        for q in range(int(b["range_off"][i]), int(b["range_off"][i + 1])):
            out.append((int(b["range_start"][q]), int(b["range_end"][q]), ts))
    return out


def _sweep_export(b, carry_ranges):
    """Independent restatement of the interval export: every breakpoint, the max over what contains each elementary
    gap, maximal runs of one value (the oracle merges txn by txn instead)."""
    pieces = [(int(s), int(e), (int(m), int(l), int(n))) for s, e, m, l, n in zip(*carry_ranges)]
    pieces += _recorded_ranges(b)
    xs = sorted({p for s, e, _ in pieces for p in (s, e)})
    vals = []
    for g in range(len(xs) - 1):
        y = xs[g + 1]
        best = None
        for s, e, t in pieces:
            if s < y <= e and (best is None or _order(*t) > _order(*best)):
                best = t
        vals.append(best)
    out = []
    for g, v in enumerate(vals):
        if v is None:
            continue
        if out and out[-1][1] == xs[g] and out[-1][2] == v:
            out[-1] = (out[-1][0], xs[g + 1], v)
        else:
            out.append((xs[g], xs[g + 1], v))
    return out


def _random_carry_ranges(rng, keyspace, hlc, count):
    cuts = np.unique(rng.integers(0, keyspace, size=2 * count))
    s, e = cuts[0:-1:2], cuts[1::2]
    k = min(len(s), len(e))
    s, e = s[:k].astype(np.uint64), e[:k].astype(np.uint64)
    epoch = np.ones(k, np.uint64)
    h = hlc + rng.integers(0, 400, size=k)
    msb = (epoch << np.uint64(16)) | (np.asarray(h, np.uint64) >> np.uint64(48))
    lsb = (np.asarray(h, np.uint64) << np.uint64(16)) | (np.uint64(abi.KIND_WRITE << 1) | np.uint64(1))
    node = rng.integers(1, 9, size=k).astype(np.int32)
    return s, e, msb, lsb, node


def _range_batch(seed, n=400, keyspace=600):
    rng = np.random.default_rng(seed)
    kinds = rng.choice([R, W, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT],
                       p=[0.35, 0.35, 0.1, 0.1, 0.1], size=n)
    status = rng.integers(0, 8, size=n).astype(np.uint8)
    return workload.generate(n, keys_per_txn=2, keyspace=keyspace, range_frac=0.3, range_width_max=80, seed=seed,
                             slow_frac=0.3, bump_max=300, kinds=kinds, status=status)


def test_export_ranges_equals_sweep():
    for seed in (11, 12, 13):
        b = _range_batch(seed)
        rng = np.random.default_rng(seed)
        carry = _random_carry_ranges(rng, 600, 1_000_000, 40) if seed != 11 else O.EMPTY_CARRY_RANGES
        got = O.max_conflicts_export_ranges(b, carry)
        want = _sweep_export(b, carry)
        assert [(int(s), int(e), (int(m), int(l), int(n))) for s, e, m, l, n in zip(*got)] == want
        assert len(want) > 10
        # normal form: sorted, disjoint, no two touching pieces of one value
        assert all(got[1][k] <= got[0][k + 1] for k in range(len(want) - 1))


def test_ts_folds_carried_points_and_intervals():
    for seed in (21, 22):
        b = _range_batch(seed)
        rng = np.random.default_rng(seed)
        carry_r = _random_carry_ranges(rng, 600, 1_000_500, 30)
        keys = np.unique(rng.integers(0, 600, size=80)).astype(np.uint64)
        kh = 1_000_000 + rng.integers(0, 900, size=len(keys))
        kmsb = (np.uint64(1) << np.uint64(16)) | (kh.astype(np.uint64) >> np.uint64(48))
        klsb = kh.astype(np.uint64) << np.uint64(16) | np.uint64(abi.KIND_WRITE << 1)
        carry_k = (keys, kmsb, klsb, rng.integers(1, 9, size=len(keys)).astype(np.int32))
        cfg = abi.make_config(8, 2, 0.2, 0xF00 + seed)
        om, ol, on, fast = O.max_conflicts_ts(b, cfg, carry_k, carry_r)
        rank, _ = O.max_conflicts(b, cfg)
        is_range = (b["txn_lsb"] & np.uint64(1)).astype(bool)
        for i in range(b["n"]):
            best = None
            def fold(t):
                nonlocal best
                if best is None or _order(*t) > _order(*best):
                    best = t
            if not is_range[i]:
                for p in range(int(b["key_off"][i]), int(b["key_off"][i + 1])):
                    k = int(b["keys"][p])
                    for x in range(len(keys)):
                        if int(keys[x]) == k:
                            fold((int(carry_k[1][x]), int(carry_k[2][x]), int(carry_k[3][x])))
                    for s, e, m, l, n in zip(*carry_r):
                        if int(s) < k <= int(e):
                            fold((int(m), int(l), int(n)))
            else:
                for q in range(int(b["range_off"][i]), int(b["range_off"][i + 1])):
                    qs, qe = int(b["range_start"][q]), int(b["range_end"][q])
                    for x in range(len(keys)):
                        if qs < int(keys[x]) <= qe:
                            fold((int(carry_k[1][x]), int(carry_k[2][x]), int(carry_k[3][x])))
                    for s, e, m, l, n in zip(*carry_r):
                        if int(s) < qe and int(e) > qs:
                            fold((int(m), int(l), int(n)))
            for v in range(2):
                t = best
                r = int(rank[v, i])
                if r != NONE:
                    bt = (int(b["exec_msb"][r]), int(b["exec_lsb"][r]), int(b["exec_node"][r]))
                    if t is None or _order(*bt)[:4] > _order(*t)[:4]:
                        t = bt
                assert (int(om[v, i]), int(ol[v, i]), int(on[v, i])) == (t if t is not None else (0, 0, 0)), (v, i)
                me = (int(b["txn_msb"][i]), int(b["txn_lsb"][i]), int(b["txn_node"][i]))
                esp = (int(b["txn_lsb"][i]) >> 1) & 7 == abi.KIND_EXCLUSIVE_SYNC_POINT   # CommandStore.java:333-337
                assert int(fast[v, i]) == int(esp or t is None or _order(*me)[:4] >= _order(*t)[:4])
        assert fast.min() == 0 and fast.max() == 1


def test_export_ranges_chain_is_one_merge():
    # carrying the interval map through two batches equals one merge of everything they and the carry recorded
    # (ReducingIntervalMap.merge with Timestamp::max is associative and commutative)
    b1, b2 = _range_batch(31), _range_batch(32)
    rng = np.random.default_rng(33)
    carry = _random_carry_ranges(rng, 600, 1_000_000, 25)
    chained = O.max_conflicts_export_ranges(b2, O.max_conflicts_export_ranges(b1, carry))
    pieces = [(int(s), int(e), (int(m), int(l), int(n))) for s, e, m, l, n in zip(*carry)]
    pieces += _recorded_ranges(b1) + _recorded_ranges(b2)
    xs = sorted({p for s, e, _ in pieces for p in (s, e)})
    want = []
    for g in range(len(xs) - 1):
        best = None
        for s, e, t in pieces:
            if s < xs[g + 1] <= e and (best is None or _order(*t) > _order(*best)):
                best = t
        if best is None:
            continue
        if want and want[-1][1] == xs[g] and want[-1][2] == best:
            want[-1] = (want[-1][0], xs[g + 1], best)
        else:
            want.append((xs[g], xs[g + 1], best))
    assert [(int(s), int(e), (int(m), int(l), int(n))) for s, e, m, l, n in zip(*chained)] == want
