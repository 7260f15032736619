"""More of the reference's own property tests, restated as pins (round 5).  Each test's generator is regenerated
from its own source through tests/refgen.py (java.util.Random + RandomSource.nextInt(min, max)) and the
Property.qt loop (test/utils/Property.java:247-263: one DefaultRandom(seed), the example's draws, then
seed = nextLong(); setSeed(seed)); qt's seed is random per JUnit run (SeedProvider), so fixed seeds stand in.

* SortedArraysTest (test/utils/SortedArraysTest.java):
  - testLinearUnion (:173-187): linearUnion(a, b) == sorted(set(a) | set(b)), both argument orders;
  - testRemapperSequential / testRemapperParial (:42-70): remapToSuperset(src, trg)[i] indexes src[i] in trg.
  The oracle's linearUnion (oracle.cpp linear_union, RelationMultiMap.linearUnion) and, -m gpu, the device merge
  (ad_merge_host: k_merge, merge_kernels.h) are checked against the test's model.  A relation whose key 0 holds
  src and key 1 trg unions to trg's TxnIds, and key 0's keysToTxnIds is then exactly remapToSuperset(src, trg).
* SearchableRangeListTest (test/utils/SearchableRangeListTest.java:36-120), for the range index (a14):
  fullWorld (1000 unit ranges (i, i+1], queries (i, 1000] and (0, 1000 - i]) and random (1000-10000 ranges
  (s, s + U[1, 1000)] over the int domain sorted by start, queries = a stored range, a fresh range, or the span of
  a run of stored ranges); expected = every stored range r with query.compareIntersecting(r) == 0
  (Range.java:296-305).  Each stored range is a range Write, each query a range Read of one batch, so a query's
  RangeDeps TxnIds are exactly what SearchableRangeList.forEachRange visits (oracle, and -m gpu the device's
  k_range_deps over range_index.h).  Ints map to u64 keys by x + 2^31 (order-preserving).
* DepsTest.test (test/primitives/DepsTest.java:35-118): validateSelfWith (deps.with(deps) == deps: the device
  merge of a reply with itself), validateContains / validateMaxTxnId over the three classes of engine outputs.
"""
import numpy as np
import pytest

import oracle as O
import refgen as R
from accord_amd import abi, workload

INT_MIN, INT_MAX = -(1 << 31), (1 << 31) - 1
OFF = 1 << 31


def set_seed(r, seed):
    r.seed = (seed ^ R.MULT) & R.MASK48


def qt(seed, examples, draw):
    """Property.qt().check over `examples`: one DefaultRandom(seed), reseeded from its nextLong after each example
    (Property.java:247-263).  Yields draw(random) per example."""
    r = R.JavaRandom(seed)
    for _ in range(examples):
        yield draw(r)
        set_seed(r, _signed64(r.nextLong()))


def _signed64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def sorted_unique_ints(r, min_size, max_size=100):
    """SortedArraysTest.sortedUniqueIntegerArray(minSize) (:338-346): Gens.arrays(ints().all()).unique()
    .ofSizeBetween(minSize, 100): size = nextInt(min, max + 1) (Gens.java:672-676), elements nextInt() redrawn
    while already seen (GenReset :990-996), then Arrays.sort."""
    size = r.nextInt(min_size, max_size + 1)
    seen, out = set(), []
    while len(out) < size:
        v = r.nextInt()
        if v not in seen:
            seen.add(v)
            out.append(v)
    return sorted(out)


def remapper_sequential(r):
    """remapperSequentialSubset(sortedUniqueIntegerArray(1)) (:316-325)."""
    trg = sorted_unique_ints(r, 1)
    to = r.nextInt(0, len(trg))
    offset = 0 if to == 0 else r.nextInt(0, to)
    return trg[offset:to], trg


def remapper_partial(r):
    """remappedPartialSubset(sortedUniqueIntegerArray(0)) (:327-334): each element kept on nextBoolean()."""
    trg = sorted_unique_ints(r, 0)
    src = [x for x in trg if r.nextBoolean()] if trg else []
    return src, trg


def rel(key_lists):
    """(keys, vals, keysToTxnIds) of {key: sorted unique u32 values} in the KeyDeps layout (KeyDeps.java:153-172)."""
    keys = sorted(k for k, v in key_lists.items() if v)
    vals = sorted({x for k in keys for x in key_lists[k]})
    pos = {x: i for i, x in enumerate(vals)}
    body, ends = [], []
    for k in keys:
        body += [pos[x] for x in key_lists[k]]
        ends.append(len(keys) + len(body))
    return np.array(keys, np.uint64), np.array(vals, np.uint32), np.array(ends + body, np.int32)


def per_key(r_):
    keys, vals, m = r_
    out, start = {}, len(keys)
    for j, k in enumerate(keys):
        out[int(k)] = [int(x) for x in m[start:int(m[j])]]
        start = int(m[j])
    return out


UNION_SEEDS = (0x5eed, 7, -42, 123456789)
EXAMPLES = 250


def _u(xs):
    return [x + OFF for x in xs]


@pytest.mark.parametrize("seed", UNION_SEEDS)
def test_oracle_linear_union_model(seed):
    for a, b in qt(seed, EXAMPLES, lambda r: (sorted_unique_ints(r, 0), sorted_unique_ints(r, 0))):
        want = sorted(set(a) | set(b))
        for x, y in ((a, b), (b, a)):
            ok, ov, om = O.union_relation(rel({0: _u(x)}), rel({0: _u(y)}))
            assert [int(v) - OFF for v in ov] == want
            if want:
                assert per_key((ok, ov, om))[0] == list(range(len(want)))


@pytest.mark.parametrize("seed", UNION_SEEDS)
@pytest.mark.parametrize("gen", ["sequential", "partial"])
def test_oracle_remap_to_superset_model(seed, gen):
    draw = remapper_sequential if gen == "sequential" else remapper_partial
    for src, trg in qt(seed, EXAMPLES, draw):
        ok, ov, om = O.union_relation(rel({0: _u(src)}), rel({1: _u(trg)}))
        assert [int(v) - OFF for v in ov] == trg                     # trg is a superset: the union is trg
        if src:
            result = per_key((ok, ov, om))[0]                        # = remapToSuperset(src, trg)
            assert all(trg[result[i]] == src[i] for i in range(len(src)))


def _dense_batch(n, seed=5):
    return workload.generate(n, keys_per_txn=1, keyspace=1 << 30, seed=seed)


def _rows_to_csr(rows, n):
    """Per txn row i: {key: [TxnId ranks]} -> one canonical abi.Csr (KeyDeps layout)."""
    key_off, keys, k2t_off, k2t, txn_off, txns = [0], [], [0], [], [0], []
    for i in range(n):
        kl = rows[i] if i < len(rows) else {}
        ks, vs, m = rel(kl)
        keys += [int(k) for k in ks]
        txns += [int(v) for v in vs]
        k2t += [int(x) for x in m]
        key_off.append(len(keys)); txn_off.append(len(txns)); k2t_off.append(len(k2t))
    return abi.Csr(np.array(key_off, np.uint32), np.array(keys, np.uint64), np.array(k2t_off, np.uint32),
                   np.array(k2t, np.int32), np.array(txn_off, np.uint32), np.array(txns, np.uint32))


def _empty(n, is_range=False):
    z = np.zeros(n + 1, np.uint32)
    return abi.Csr(z, np.zeros(0, np.uint64), z.copy(), np.zeros(0, np.int32), z.copy(), np.zeros(0, np.uint32), is_range)


def _merge_cases(seed, gen):
    """One device row per qt example: reply 0 = {key 0: x}, reply 1 = {key 0 or 1: y}; the example's ints are rank-
    compressed over the whole case (an order-preserving map: union and remap commute with it)."""
    if gen == "union":
        ex = list(qt(seed, EXAMPLES, lambda r: (sorted_unique_ints(r, 0), sorted_unique_ints(r, 0))))
    else:
        ex = list(qt(seed, EXAMPLES, remapper_sequential if gen == "sequential" else remapper_partial))
    allv = sorted({v for x, y in ex for v in x + y})
    rank = {v: i for i, v in enumerate(allv)}
    n = max(len(allv), len(ex), 1)
    k1 = 0 if gen == "union" else 1
    r0 = [{0: [rank[v] for v in x]} for x, _ in ex]
    r1 = [{k1: [rank[v] for v in y]} for _, y in ex]
    return ex, rank, n, r0, r1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", UNION_SEEDS[:2])
@pytest.mark.parametrize("gen", ["union", "sequential", "partial"])
def test_gpu_merge_equals_sorted_arrays_model(engine_factory, seed, gen):
    ex, rank, n, r0, r1 = _merge_cases(seed, gen)
    eng = engine_factory(window=0, replicas=2, drop_p=0.0, seed=1)
    eng.load(_dense_batch(n))
    a, b = _rows_to_csr(r0, n), _rows_to_csr(r1, n)
    eng.merge_host([[a, _empty(n), _empty(n, True)], [b, _empty(n), _empty(n, True)]])
    got = eng.fetch_merged(abi.CLASS_KEY)
    for i, (x, y) in enumerate(ex):
        ks, tx, m = got.txn(i)
        pk = per_key((ks, tx, m))
        inv = {v: k for k, v in rank.items()}
        if gen == "union":
            want = sorted(set(x) | set(y))
            assert [inv[int(t)] for t in tx] == want, i
            if want:
                assert pk[0] == list(range(len(want)))
        else:
            assert [inv[int(t)] for t in tx] == y, i               # src subset of trg: the union is trg
            if x:
                assert all(y[pk[0][j]] == x[j] for j in range(len(x))), i
    # and the device equals the oracle's LinearMerger row by row
    for i in range(len(ex)):
        want = O.union_relation(rel(r0[i]), rel(r1[i]))
        ks, tx, m = got.txn(i)
        assert np.array_equal(ks, want[0]) and np.array_equal(tx, want[1]) and np.array_equal(m, want[2]), i


# ---- SearchableRangeListTest -----------------------------------------------------------------------------------
def full_world():
    ranges = [(i, i + 1) for i in range(1000)]
    queries = [(i, 1000) for i in range(1000)] + [(0, 1000 - i) for i in range(1000)]
    return ranges, queries


def searchable_random(r):
    """SearchableRangeListTest.random's example body (:59-117): numRanges = nextInt(1000, 10000) ranges
    (s, s + nextInt(1, 1000)] with s = nextInt(MIN, MAX - 1000), stable-sorted by start; 1000 queries by
    selection nextInt(0, 3): a picked stored range, a fresh one, or (start of ranges[a], end of ranges[a + d]]."""
    num = r.nextInt(1000, 10000)
    ranges = []
    for _ in range(num):
        s = r.nextInt(INT_MIN, INT_MAX - 1000)
        ranges.append((s, s + r.nextInt(1, 1000)))
    ranges.sort(key=lambda x: x[0])                     # Comparator.comparing(Range::start), stable
    queries = []
    for _ in range(1000):
        sel = r.nextInt(0, 3)
        if sel == 0:
            queries.append(ranges[0] if len(ranges) == 1 else ranges[r.nextInt(0, len(ranges))])
        elif sel == 1:
            s = r.nextInt(INT_MIN, INT_MAX - 1000)
            queries.append((s, s + r.nextInt(1, 1000)))
        else:
            a = r.nextInt(0, len(ranges))
            e = a + r.nextInt(0, len(ranges) - a)
            queries.append((ranges[a][0], ranges[e][1]))
    return ranges, queries


def _range_batch(ranges, queries):
    canonical = {t: [(s + OFF, e + OFF)] for t, (s, e) in enumerate(ranges)}
    return R.rangedeps_batch(canonical, [("range", (s + OFF, e + OFF)) for s, e in queries])


def _expected_sets(ranges, queries):
    """Per query: the stored ranges r with query.compareIntersecting(r) == 0 (start < r.end && end > r.start)."""
    st = np.array([s for s, _ in ranges], np.int64)
    en = np.array([e for _, e in ranges], np.int64)
    return [np.nonzero((qs < en) & (qe > st))[0] for qs, qe in queries]


def _check_range_deps(csr, ranges, queries, want):
    N = len(ranges)
    for q, w in enumerate(want):
        ks, tx, m = csr.txn(N + q)
        assert np.array_equal(tx.astype(np.int64), w), "query %d: %s" % (q, queries[q])
        # each dependency on its own (stored) range
        for j, rg in enumerate(ks):
            s, e = int(rg[0]) - OFF, int(rg[1]) - OFF
            lo = len(ks) if j == 0 else int(m[j - 1])
            for x in m[lo:int(m[j])]:
                assert ranges[int(tx[int(x)])] == (s, e)


def test_oracle_searchable_full_world():
    ranges, queries = full_world()
    want = _expected_sets(ranges, queries)
    assert [len(w) for w in want[:3]] == [1000, 999, 998]       # (i, 1000] meets (j, j+1] for j in [i, 1000)
    res = O.OracleResult(_range_batch(ranges, queries), abi.make_config(0, 1, 0.0, 1), 0)
    _check_range_deps(res.deps(0, abi.CLASS_RANGE), ranges, queries, want)


SEARCHABLE_SEEDS = (0x5ea7c4, -3, 99)


@pytest.mark.parametrize("seed", SEARCHABLE_SEEDS)
def test_oracle_searchable_random(seed):
    for ranges, queries in qt(seed, 2, searchable_random):
        want = _expected_sets(ranges, queries)
        res = O.OracleResult(_range_batch(ranges, queries), abi.make_config(0, 1, 0.0, 1), 0)
        _check_range_deps(res.deps(0, abi.CLASS_RANGE), ranges, queries, want)
        assert sum(len(w) for w in want) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["full_world"] + ["random_%d" % i for i in range(len(SEARCHABLE_SEEDS))])
def test_gpu_searchable_range_list(engine_factory, case):
    if case == "full_world":
        cases = [full_world()]
    else:
        cases = list(qt(SEARCHABLE_SEEDS[int(case.split("_")[1])], 2, searchable_random))
    for ranges, queries in cases:
        b = _range_batch(ranges, queries)
        eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
        eng.load(b)
        eng.preaccept_deps()
        got = eng.fetch_deps(0, abi.CLASS_RANGE)
        _check_range_deps(got, ranges, queries, _expected_sets(ranges, queries))
        ref = O.OracleResult(b, abi.make_config(0, 1, 0.0, 1), 0).deps(0, abi.CLASS_RANGE)
        assert got.equal(ref), "first difference at txn %s" % got.first_difference(ref)


# ---- DepsTest ------------------------------------------------------------------------------------------------------
def _max_txn_id(csrs, i):
    ts = [int(t) for c in csrs for t in c.txn(i)[1]]
    return max(ts) if ts else None


@pytest.mark.gpu
def test_gpu_deps_self_with_contains_max(engine_factory):
    """DepsTest.test's checks on the device's own Deps (C4-like mix: all three classes populated): with(self) ==
    self (validateSelfWith: Deps.merge of a reply with itself, ad_merge_host), contains (validateContains: every
    class's TxnIds are in the merged txnIds), maxTxnId == the max over the three classes (validateMaxTxnId)."""
    kinds = np.random.default_rng(31).choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT,
                                              abi.KIND_EXCLUSIVE_SYNC_POINT], p=[0.42, 0.42, 0.08, 0.08], size=6000)
    b = workload.generate(6000, keys_per_txn=3, keyspace=20_000, range_frac=0.1, range_width_max=300, seed=31,
                          kinds=kinds)             # key-domain sync points (witnessed by ExclusiveSyncPoints): directKeyDeps
    eng = engine_factory(window=8, replicas=1, drop_p=0.0, seed=2)
    eng.load(b)
    eng.preaccept_deps()
    reply = [eng.fetch_deps(0, c) for c in range(abi.NUM_CLASSES)]
    assert all(r.entries() > 0 for r in reply)
    eng.merge_host([reply, reply])
    merged = [eng.fetch_merged(c) for c in range(abi.NUM_CLASSES)]
    for c in range(abi.NUM_CLASSES):
        assert merged[c].equal(reply[c]), "with(self) != self in class %d" % c
    for i in range(0, b["n"], 97):
        allt = set(int(t) for c in merged for t in c.txn(i)[1])
        for c in reply:
            assert set(int(t) for t in c.txn(i)[1]) <= allt
        assert _max_txn_id(merged, i) == (max(allt) if allt else None)


# ---- the ts3_fold tie (DESIGN §7 "witnessedAt proposal"): known answers ----------------------------------------------
REJECTED = 0x8000


def _tie_batch():
    """Two txns on key 5: a committed Write (executeAt = its TxnId) and a later Read querying maxConflicts.get."""
    b = workload.generate(2, keys_per_txn=1, keyspace=100, seed=3, slow_frac=0.0,
                          kinds=np.array([abi.KIND_WRITE, abi.KIND_READ]))
    b["keys"] = np.array([5, 5], np.uint64)
    return b


def _tie_cases():
    """(carried point lsb, carried interval lsb or None, batch executeAt lsb, the answer).  All values are one Timestamp
    under compareTo (Timestamp.java:208-217 compares lsb >>> 16 and flags & 0x1E only), some with the REJECTED bit
    0x8000 that uniqueNow(..).asRejected() sets.
    * carry vs batch (cases 0, 1): the carried value stays on a tie, in both orders -- as the reference's single map
      does: MaxConflicts.update merges with Timestamp::max (MaxConflicts.java:55-58; Timestamp.java:265-268
      `a.compareTo(b) >= 0 ? a : b` keeps the existing value).
    * carried point vs carried interval over the same key (case 2): the device and the oracle keep the larger raw lsb;
      the reference holds one value per key, and which one survived its merges depends on their order (the
      documented divergence; no reference test observes these bits)."""
    b = _tie_batch()
    l0 = int(b["txn_lsb"][0])
    return b, [(l0 | REJECTED, None, l0, l0 | REJECTED), (l0, None, l0 | REJECTED, l0),
               (l0, l0 | REJECTED, l0, l0 | REJECTED)]


def _tie_inputs(b, carry_lsb, iv_lsb, exec_lsb):
    b = dict(b)
    b["exec_lsb"] = b["exec_lsb"].copy()
    b["exec_lsb"][0] = np.uint64(exec_lsb)
    carry = (np.array([5], np.uint64), b["txn_msb"][:1].copy(), np.array([carry_lsb], np.uint64), b["txn_node"][:1].copy())
    iv = None
    if iv_lsb is not None:
        iv = (np.array([4], np.uint64), np.array([5], np.uint64), b["txn_msb"][:1].copy(), np.array([iv_lsb], np.uint64),
              b["txn_node"][:1].copy())
    return b, carry, iv


def test_oracle_ts3_fold_tie_kat():
    base, cases = _tie_cases()
    cfg = abi.make_config(0, 1, 0.0, 1)
    for carry_lsb, iv_lsb, exec_lsb, want in cases:
        b, carry, iv = _tie_inputs(base, carry_lsb, iv_lsb, exec_lsb)
        m, l, nd, fast = O.max_conflicts_ts(b, cfg, carry=carry, carry_ranges=iv)
        assert int(m[0, 1]) == int(b["txn_msb"][0]) and int(nd[0, 1]) == int(b["txn_node"][0])
        assert int(l[0, 1]) == want and fast[0, 1] == 1                # the Read's TxnId is later: fast path


@pytest.mark.gpu
def test_gpu_ts3_fold_tie_kat(engine_factory):
    base, cases = _tie_cases()
    for carry_lsb, iv_lsb, exec_lsb, want in cases:
        b, carry, iv = _tie_inputs(base, carry_lsb, iv_lsb, exec_lsb)
        eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
        eng.load(b)
        eng.preaccept_deps()
        eng.max_conflicts_carry(carry)
        if iv is not None:
            eng.max_conflicts_carry_ranges(iv)
        m, l, nd, fast = eng.max_conflicts_ts()
        assert int(l[0, 1]) == want and int(m[0, 1]) == int(b["txn_msb"][0]) and fast[0, 1] == 1
        w = O.max_conflicts_ts(b, abi.make_config(0, 1, 0.0, 1), carry=carry, carry_ranges=iv)
        for x, y in zip((m, l, nd, fast), w):
            assert np.array_equal(x, y)


# ---- ReducingRangeMapTest.testRandomAdds (test/utils/ReducingRangeMapTest.java:166-232): the MaxConflicts range carry
# The test's additions (RandomMap.addOneRandom: 1-2 StartInclusive ranges [s, e) per addition, one Timestamp
# ts(b) = (epoch 1, hlc b, flags 0, node 1) each), its three maps merged with Timestamp::max, and the probes its
# validate() draws (decr/self/incr of every canonical key, 1000 random keys, 100 foldl key sets and their Ranges) are
# regenerated from the seed (refgen.rrm_random_adds).  Expected values come from the map's definition -- a point's
# value is the max over the added ranges containing it (Range.StartInclusive.contains: s <= p < e), a range query's
# the max over the added ranges it intersects -- not from the test's canonical TreeMap: that one keys each interval
# by its lower bound but reads it with ceilingEntry (:312-315), and the test swallows AssertionFailedError (:225-228),
# so its own expectation is not a usable oracle.
# Mapping: each addition is a recorded range Write (TxnId epoch 0, executeAt ts(b)) of one batch, [s, e) the
# interval (u(s) - 1, u(e) - 1] with u(x) = x + 2^31 + 1 (a key k stabs (k - 1, k]); a map is that batch's
# max_conflicts_export_ranges, the merge is the carry (MaxConflicts.update = merge(this, ...), Timestamp::max).  A probe
# is a txn of a second batch (status INVALID, so it records nothing) answered by max_conflicts_ts over the map alone.
RRM_OFF = (1 << 31) + 1
RRM_CASES = [(8532037884171168001, 3, 1, 3, 0.1, 0.1)] + [
    (seed, 3, adds, 3, cov, chance) for adds in (1, 10, 100) for cov in (0.01, 0.1, 0.5) for chance in (0.01, 0.1)
    for seed in (0x5EED0000 + 7 * adds + int(cov * 1000) + int(chance * 100), 0x0ACC0FFEE + adds)]


def _rrm_u(x):
    return x + RRM_OFF


def _rrm_ts(b):
    return (1 << 15, b << 16, 1)


def _rrm_batch(txns, epoch):
    """txns: [(kind, status, keys list, ranges [(a, b)) list, executeAt hlc or None)] -> a batch dict."""
    n = len(txns)
    tm, tl, tn, em, el, en, st, ko, ks, ro, rs, re_ = [], [], [], [], [], [], [], [0], [], [0], [], []
    for i, (kind, status, keys, ranges, ex) in enumerate(txns):
        flags = (kind << 1) | (1 if ranges else 0)
        m, l, nd = R.txn_id(epoch, i + 1, flags, 1)
        tm.append(m); tl.append(l); tn.append(nd)
        e = _rrm_ts(ex) if ex is not None else (m, l, nd)
        em.append(e[0]); el.append(e[1]); en.append(e[2])
        st.append(status)
        ks += [_rrm_u(k) for k in keys]
        ko.append(len(ks))
        for a, b in ranges:
            rs.append(_rrm_u(a) - 1); re_.append(_rrm_u(b) - 1)
        ro.append(len(rs))
    u64 = lambda v: np.array(v, np.uint64)  # noqa: E731
    return {"n": n, "txn_msb": u64(tm), "txn_lsb": u64(tl), "txn_node": np.array(tn, np.int32), "exec_msb": u64(em),
            "exec_lsb": u64(el), "exec_node": np.array(en, np.int32), "status": np.array(st, np.uint8),
            "key_off": np.array(ko, np.uint32), "keys": u64(ks), "range_off": np.array(ro, np.uint32) if rs else None,
            "range_start": u64(rs) if rs else None, "range_end": u64(re_) if rs else None}


def _rrm_adds_batch(adds):
    return _rrm_batch([(abi.KIND_WRITE, abi.ST_APPLIED, [], ranges, b) for ranges, b in adds], 0)


def _rrm_probe_batch(probes):
    points, folds = probes
    txns = [(abi.KIND_READ, abi.ST_INVALID, [p], [], None) for p in points]
    for keys, ranges in folds:
        txns.append((abi.KIND_READ, abi.ST_INVALID, keys, [], None))
        txns.append((abi.KIND_READ, abi.ST_INVALID, [], ranges, None))
    return _rrm_batch(txns, 2)


def _rrm_expected(adds, probes):
    """Per probe txn the map's answer: (msb, lsb, node) of the max ts(b), or Timestamp.NONE (0, 0, 0)."""
    rs = [(s, e, b) for ranges, b in adds for s, e in ranges]

    def point(p):
        return max((b for s, e, b in rs if s <= p < e), default=None)

    def span(a, c):
        return max((b for s, e, b in rs if s < c and a < e), default=None)
    points, folds = probes
    vals = [point(p) for p in points]
    for keys, ranges in folds:
        vals.append(max((v for v in (point(k) for k in keys) if v is not None), default=None))
        vals.append(max((v for v in (span(a, c) for a, c in ranges) if v is not None), default=None))
    out = np.array([_rrm_ts(v) if v is not None else (0, 0, 0) for v in vals], np.int64)
    return out[:, 0].astype(np.uint64), out[:, 1].astype(np.uint64), out[:, 2].astype(np.int32)


def _rrm_normal_form(adds):
    """The map as maximal pieces of one value, in the export's coordinates: (starts, ends, msb, lsb, node)."""
    rs = [(s, e, b) for ranges, b in adds for s, e in ranges]
    cuts = sorted({x for s, e, _ in rs for x in (s, e)})
    pieces = []
    for x, y in zip(cuts, cuts[1:]):
        v = max((b for s, e, b in rs if s <= x and y <= e), default=None)
        if v is None:
            continue
        if pieces and pieces[-1][1] == x and pieces[-1][2] == v:
            pieces[-1][1] = y
        else:
            pieces.append([x, y, v])
    u64 = lambda v: np.array(v, np.uint64)  # noqa: E731
    return (u64([_rrm_u(x) - 1 for x, _, _ in pieces]), u64([_rrm_u(y) - 1 for _, y, _ in pieces]),
            u64([1 << 15] * len(pieces)), u64([v << 16 for _, _, v in pieces]), np.ones(len(pieces), np.int32))


def _rrm_case(case):
    try:
        return R.rrm_random_adds(*case)
    except ValueError:                      # nextInt(MAX_VALUE - length - 1) with a bound <= 0: the Java test throws
        return None


def _rrm_check(export_ranges, answer, case):
    """export_ranges(batch, carry) -> the map; answer(batch, carry) -> (msb, lsb, node) arrays [n]."""
    got = _rrm_case(case)
    if got is None:
        return False
    maps, final = got
    carry = None
    for adds, probes in maps:
        own = export_ranges(_rrm_adds_batch(adds), None)
        want = _rrm_normal_form(adds)
        assert all(np.array_equal(x, y) for x, y in zip(own, want)), "%s: map pieces" % (case,)
        for x, y, name in zip(answer(_rrm_probe_batch(probes), own), _rrm_expected(adds, probes), ("msb", "lsb", "node")):
            bad = np.nonzero(x != y)[0]
            assert len(bad) == 0, "%s: validate %s differs at probes %s" % (case, name, bad[:8])
        carry = export_ranges(_rrm_adds_batch(adds), carry)
    alladds = [a for adds, _ in maps for a in adds]
    assert all(np.array_equal(x, y) for x, y in zip(carry, _rrm_normal_form(alladds))), "%s: merged pieces" % (case,)
    for x, y in zip(answer(_rrm_probe_batch(final), carry), _rrm_expected(alladds, final)):
        assert np.array_equal(x, y), "%s: final validate" % (case,)
    return True


def test_oracle_reducing_range_map_random_adds():
    cfg = abi.make_config(0, 1, 0.0, 1)

    def answer(b, carry):
        m, l, nd, _ = O.max_conflicts_ts(b, cfg, None, carry)
        return m[0], l[0], nd[0]
    done = sum(_rrm_check(O.max_conflicts_export_ranges, answer, c) for c in RRM_CASES)
    assert done >= len(RRM_CASES) - 3


@pytest.mark.gpu
def test_gpu_reducing_range_map_random_adds(engine_factory):
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)

    def run(b, carry):
        eng.load(b)
        eng.preaccept_deps()
        eng.max_conflicts_carry(O.EMPTY_CARRY)
        eng.max_conflicts_carry_ranges(O.EMPTY_CARRY_RANGES if carry is None else carry)
        return eng.max_conflicts_ts()

    def export_ranges(b, carry):
        run(b, carry)
        return tuple(a.copy() for a in eng.max_conflicts_export_ranges())

    def answer(b, carry):
        m, l, nd, _ = run(b, carry)
        return m[0].copy(), l[0].copy(), nd[0].copy()
    done = sum(_rrm_check(export_ranges, answer, c) for c in RRM_CASES[::2])
    assert done >= len(RRM_CASES[::2]) - 2
