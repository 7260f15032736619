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
