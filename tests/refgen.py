"""Restatement of the reference's own seeded test generators (TEST INFRASTRUCTURE).

The reference's property tests draw from ``accord.utils.DefaultRandom`` (a ``java.util.Random``,
core/utils/DefaultRandom.java:23-33) through ``RandomSource`` (core/utils/RandomSource.java:79-108) and
``WrappedRandomSource`` (nextInt()/nextInt(bound)/nextBoolean delegate to java.util.Random).  Both are
spec-defined, so the reference tests' inputs for a given seed are regenerated here bit-exactly:

* ``JavaRandom``            — java.util.Random (48-bit LCG, next(bits), nextInt(bound), nextBoolean)
* ``nextInt(min, max)``     — RandomSource.nextInt(int, int) default method (:81-108)
* ``int_hash_key``          — test/impl/IntHashKey.hash (:256-263): CRC32 over the 4 low bytes; keys
                              compare by hash only (:276-279), so the order-preserving u64 is the hash
* ``txn_id``                — TxnId.fromValues(epoch, hlc, flags, node) bits (Timestamp.java:81-89)
* ``keydeps_generate``      — KeyDepsTest.Deps.generate(random, ...) (test/primitives/KeyDepsTest.java:364-407)
* ``keydeps_supplier``      — KeyDepsTest.supplier (:520-535), used by testMerge (:115-126) / main (:612-618)
"""
import zlib

MASK48 = (1 << 48) - 1
MULT = 0x5DEECE66D


def _i32(x):
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= 1 << 31 else x


class JavaRandom:
    def __init__(self, seed):
        self.seed = (seed ^ MULT) & MASK48

    def next(self, bits):
        self.seed = (self.seed * MULT + 0xB) & MASK48
        return _i32(self.seed >> (48 - bits))

    def nextInt(self, bound=None, hi=None):
        if bound is None:
            return self.next(32)
        if hi is not None:                      # RandomSource.nextInt(min, max)
            return self._range(bound, hi)
        # java.util.Random.nextInt(bound) (WrappedRandomSource.nextInt(int) delegates to it)
        if bound <= 0:
            raise ValueError("bound must be positive")
        r = self.next(31)
        m = bound - 1
        if bound & m == 0:
            return _i32((bound * r) >> 31)
        u = r
        while True:
            r = u % bound
            if _i32(u - r + m) >= 0:
                return r
            u = self.next(31)

    def _range(self, lo, hi):
        if lo >= hi:
            raise ValueError("Min (%d) should be less than max (%d)." % (lo, hi))
        result = self.next(32)
        delta = _i32(hi - lo)
        mask = _i32(delta - 1)
        if delta & mask == 0:
            return _i32((result & mask) + lo)
        if delta > 0:
            u = (result & 0xFFFFFFFF) >> 1
            while True:
                result = u % delta
                if _i32(u + mask - result) >= 0:
                    return result + lo
                u = (self.next(32) & 0xFFFFFFFF) >> 1
        while result < lo or result >= hi:
            result = self.next(32)
        return result

    def nextBoolean(self):
        return self.next(1) != 0

    def nextLong(self):
        return ((self.next(32) << 32) + self.next(32)) & 0xFFFFFFFFFFFFFFFF


def int_hash_key(k):
    """IntHashKey.hash — CRC32 of (k, k>>8, k>>16, k>>24) low bytes, & 0xffff."""
    b = bytes([(k >> s) & 0xFF for s in (0, 8, 16, 24)])
    return zlib.crc32(b) & 0xFFFF


def txn_id(epoch, hlc, flags, node):
    """(msb, lsb, node) of TxnId.fromValues — Timestamp(epoch, hlc, flags, node) bit layout."""
    msb = (epoch << 15) | (hlc >> 48)
    lsb = ((hlc << 16) & 0xFFFFFFFFFFFFFFFF) | flags
    return (msb, lsb, node)


def txn_order_key(t):
    """Timestamp.compareTo as a Python sort key (msb unsigned, lsb>>>16, flags & 0x1E, node signed)."""
    msb, lsb, node = t
    return (msb, lsb >> 16, lsb & 0x1E, node)


class GenDeps:
    """canonical: {key_hash: set(txn)}, plus the builder add order the reference used."""

    def __init__(self, canonical, in_order_keys, in_order_values):
        self.canonical = canonical
        self.in_order_keys = in_order_keys
        self.in_order_values = in_order_values

    def add_order(self):
        """(key, txn) pairs in the order KeyDepsTest.Deps.generate feeds KeyDeps.builder()."""
        keys = sorted(self.canonical)
        if not self.in_order_keys:
            keys = keys[::-1]
        out = []
        for k in keys:
            ids = sorted(self.canonical[k], key=txn_order_key)
            if not self.in_order_values:
                ids = ids[::-1]
            out.extend((k, t) for t in ids)
        return out


def keydeps_generate(r, unique_txn_ids, epoch_range, hlc_range, flags_range, node_range, unique_keys, empty_keys,
                     key_range, total_count):
    tmp = set()
    while len(tmp) < unique_keys:
        tmp.add(int_hash_key(r.nextInt(key_range)))
    populate = sorted(tmp)
    while len(tmp) < unique_keys + empty_keys:
        tmp.add(int_hash_key(r.nextInt(key_range)))
    txns = set()
    while len(txns) < unique_txn_ids:
        e = r.nextInt(epoch_range)
        h = r.nextInt(hlc_range)
        f = 0 if flags_range == 0 else r.nextInt(flags_range)
        n = r.nextInt(node_range)
        txns.add(txn_id(e, h, f, n))
    txns = sorted(txns, key=txn_order_key)
    canonical = {}
    for _ in range(total_count):
        k = populate[r.nextInt(unique_keys)]
        t = txns[r.nextInt(unique_txn_ids)]
        canonical.setdefault(k, set()).add(t)
    ink = r.nextBoolean()
    inv = r.nextBoolean()
    return GenDeps(canonical, ink, inv)


def keydeps_supplier(r, unique_txn_ids_range, epoch_range, hlc_range, flag_range, node_range, unique_keys_range,
                     empty_keys_range, key_range, total_count_range):
    def get():
        if r.nextInt(100) == 0:
            return GenDeps({}, True, True)
        u = 1 + r.nextInt(unique_txn_ids_range - 1)
        uk = 1 + r.nextInt(unique_keys_range - 1)
        ek = 1 + r.nextInt(empty_keys_range - 1)
        tc = r.nextInt(min(total_count_range, uk * u))
        return keydeps_generate(r, u, epoch_range, hlc_range, flag_range, node_range, uk, ek, key_range, tc)
    return get


def testmerge_inputs(seed, unique_txn_ids_range=100, epoch_range=3, hlc_range=50, node_range=4, unique_keys_range=4,
                     empty_keys_range=2, key_range=100, total_count_range=10, merge_count_range=4):
    """The list of Deps KeyDepsTest.testMerge(seed, ...) merges (defaults = KeyDepsTest.main's first loop)."""
    r = JavaRandom(seed)
    sup = keydeps_supplier(r, unique_txn_ids_range, epoch_range, hlc_range, 0, node_range, unique_keys_range,
                           empty_keys_range, key_range, total_count_range)
    count = 1 + r.nextInt(merge_count_range)
    return [sup() for _ in range(count)]


# ---------------------------------------------------------------------------------------------------------
# RangeDepsTest (test/primitives/RangeDepsTest.java) — seeded inputs and its Validate queries
# ---------------------------------------------------------------------------------------------------------
def _f32(x):
    import numpy as np
    return np.float32(x)


def next_float(r):
    """java.util.Random.nextFloat(): next(24) / (float)(1 << 24), an IEEE single."""
    return _f32(r.next(24)) / _f32(1 << 24)


def _java_int(x):
    """(int) cast of a float: truncation toward zero (values here are small and finite)."""
    return int(x)


class GenerateRanges:
    """RangeDepsTest.GenerateRanges (:43-81): float arithmetic in IEEE single precision, as Java evaluates it."""

    def __init__(self, range_domain, min_dom, max_dom, min_span, max_span):
        self.range_domain = range_domain
        self.min_dom, self.max_dom = _f32(min_dom), _f32(max_dom)
        self.min_span, self.max_span = _f32(min_span), _f32(max_span)

    def generate(self, r, count):
        """generateRanges(random, rangeCount) -> list of (start, end] int pairs."""
        dom = _f32(self.range_domain)
        txn_domain = max(count, _java_int(((next_float(r) * (self.max_dom - self.min_dom)) + self.min_dom) * dom))
        txn_span = max(txn_domain, _java_int(((next_float(r) * (self.max_span - self.min_span)) + self.min_span) * dom))
        gap_span = txn_span - txn_domain
        start = 0 if self.range_domain == txn_span else r.nextInt(self.range_domain - txn_span)
        end = start + txn_span
        gaps, gap_spans = [], []
        for i in range(count):
            gaps.append(start + r.nextInt(end - start))
            if i == count - 1 or gap_span <= 1:
                gap_spans.append(gap_span)
            else:
                gap_spans.append(1 + r.nextInt(max(1, _java_div(2 * gap_span, count - i))))
        gaps.sort()
        out = []
        for i in range(count):
            end = max(start + 1, gaps[i])
            out.append((start, end))
            start = end + gap_spans[i]
        return out


def _java_div(a, b):
    """Java int division (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def ranges_of(ranges):
    """Ranges.of (AbstractRanges.of :678-684): sort by Range::compare (start, end), then merge ranges that
    overlap (MERGE_OVERLAPPING: prev.end > next.start; touching ranges stay apart)."""
    rs = sorted(ranges)
    out = []
    for s, e in rs:
        if out and out[-1][1] > s:
            out[-1] = (out[-1][0], max(out[-1][1], e))
        else:
            out.append((s, e))
    return out


def rangedeps_generate(r, gen, txn_count, range_count):
    """RangeDepsTest.generate (:197-207): {txn index: Ranges}."""
    out = {}
    for t in range(txn_count):
        this = range_count if txn_count == 1 else 1 + r.nextInt(_java_div(2 * range_count, txn_count) - 1)
        out[t] = ranges_of(gen.generate(r, this))
    return out


def rangedeps_identical(r, gen, txn_count, range_count):
    """RangeDepsTest.generateIdenticalTxns (:209-216)."""
    rs = ranges_of(gen.generate(r, _java_div(range_count, txn_count)))
    return {t: list(rs) for t in range(txn_count)}


def rangedeps_nemesis(width, nemesis_count, range_count, non_nemesis_per_nemesis):
    """RangeDepsTest.generateNemesisRanges (:218-233) -> ({txn: Ranges}, its GenerateRanges)."""
    build = {}
    non_count = nemesis_count * non_nemesis_per_nemesis
    range_count = _java_div(range_count, 1 + non_nemesis_per_nemesis)
    domain = 0
    for i in range(range_count):
        build.setdefault(i % nemesis_count, []).append((i, i + width))
        for _ in range(non_nemesis_per_nemesis):
            build.setdefault(nemesis_count + (i % non_count), []).append((i, i + 1))
        domain = i + width
    return {t: ranges_of(build[t]) for t in range(nemesis_count + non_count)}, GenerateRanges(domain, 0.0, 1.0, 0.0, 1.0)


def rangedeps_validate_queries(r, gen, canonical):
    """The queries Validate.validate(random) (:171-193) issues, in order, drawing from the same Random:
    ('range', (s, e)), ('key', k) and ('slice', [(s, e), ...]).  test.range(i) iterates RangeDeps' sorted
    unique ranges."""
    uniq = sorted({rg for rs in canonical.values() for rg in rs})
    q = []
    for rg in uniq:
        q += [("range", rg), ("key", rg[0]), ("key", rg[1])]
    for _ in range(len(uniq)):
        rg = gen.generate(r, 1)[0]
        q += [("range", rg), ("key", rg[0]), ("key", rg[1])]
    for _ in range(10):
        q.append(("slice", ranges_of(gen.generate(r, r.nextInt(10) + 1))))
    return q


# RangeDepsTest's own recorded seeds (the commented reproduction seeds in the test source)
RANGEDEPS_RANDOM_SEEDS = (-6268194734307361517, -1531261279965735959, 1953755836248097851)   # testRandom :262-268
RANGEDEPS_IDENTICAL_SEED = -4951029115911714505                                             # testIdenticalTransactions :278
RANGEDEPS_NEMESIS_SEED = 2005526220972215410                                                # testNemesisRanges :301


def rangedeps_batch(canonical, queries):
    """An engine batch whose PreAccept RangeDeps answer RangeDepsTest's Validate queries: the test's TxnIds
    become range-domain Writes (hlc = 1 + t, in TxnId order) holding their Ranges, followed by one Read per query
    (a range / slice query: range domain with its ranges; a key query: key domain with the one key).  Reads
    witness Writes only (Txn.java:221-245), so each query's RangeDeps are exactly the stored txns its footprint
    intersects (InMemoryCommandStore.mapReduceRangesInternal, :884-1017)."""
    import numpy as np
    from accord_amd import abi
    N = len(canonical)
    n = N + len(queries)
    hlc = np.arange(1, n + 1, dtype=np.int64)
    kinds = np.array([abi.KIND_WRITE] * N + [abi.KIND_READ] * len(queries), np.int64)
    domain = np.array([1] * N + [0 if q[0] == "key" else 1 for q in queries], np.int64)
    flags = (kinds << 1) | domain
    msb = (np.uint64(1) << np.uint64(15)) | (hlc.astype(np.uint64) >> np.uint64(48))
    lsb = (hlc.astype(np.uint64) << np.uint64(16)) | flags.astype(np.uint64)
    key_off, keys, range_off, rs, re_ = [0], [], [0], [], []
    for t in range(N):
        for s, e in canonical[t]:
            rs.append(s); re_.append(e)
        key_off.append(len(keys)); range_off.append(len(rs))
    for kind, v in queries:
        if kind == "key":
            keys.append(v)
        else:
            for s, e in ([v] if kind == "range" else v):
                rs.append(s); re_.append(e)
        key_off.append(len(keys)); range_off.append(len(rs))
    node = np.ones(n, np.int32)
    return {"n": n, "txn_msb": msb, "txn_lsb": lsb, "txn_node": node, "exec_msb": msb.copy(), "exec_lsb": lsb.copy(),
            "exec_node": node.copy(), "status": np.full(n, abi.ST_APPLIED, np.uint8),
            "key_off": np.array(key_off, np.uint32), "keys": np.array(keys, np.uint64),
            "range_off": np.array(range_off, np.uint32), "range_start": np.array(rs, np.uint64),
            "range_end": np.array(re_, np.uint64)}


def rangedeps_expected(canonical, queries):
    """Per batch txn, the canonical RangeDeps (sorted unique ranges, sorted unique dependency ranks, and
    rangesToTxnIds = per-range end offsets then indices) from RangeDepsTest.Validate's model: a stored txn i is
    a dependency on each of its ranges that intersects the query's footprint ((s, e] semantics,
    Range.EndInclusive) or contains the query key."""
    def inter(a, b):
        return max(a[0], b[0]) < min(a[1], b[1])
    N = len(canonical)
    foot = [("ranges", canonical[t]) for t in range(N)]
    foot += [("key", q[1]) if q[0] == "key" else ("ranges", [q[1]] if q[0] == "range" else q[1]) for q in queries]
    out = []
    for t, (kind, v) in enumerate(foot):
        pairs = set()
        for i in range(min(t, N)):
            for r in canonical[i]:
                if (kind == "key" and r[0] < v <= r[1]) or (kind == "ranges" and any(inter(r, q) for q in v)):
                    pairs.add((r, i))
        ks = sorted({p[0] for p in pairs})
        tx = sorted({p[1] for p in pairs})
        pos = {x: j for j, x in enumerate(tx)}
        ends, idx = [], []
        for k in ks:
            lst = sorted(pos[i] for (r, i) in pairs if r == k)
            idx += lst
            ends.append(len(ks) + len(idx))
        out.append((ks, tx, ends + idx))
    return out


# ---------------------------------------------------------------------------------------------------------
# ReducingRangeMapTest.testRandomAdds (test/utils/ReducingRangeMapTest.java:166-232, RandomMap :234-292,
# RandomWithCanonical.validate :385-470) — the additions and the probes its validate() draws, in stream order
# ---------------------------------------------------------------------------------------------------------
INT_MIN_J, INT_MAX_J = -(1 << 31), (1 << 31) - 1


def next_double(r):
    """java.util.Random.nextDouble(): ((long) next(26) << 27) + next(27)) * 2^-53."""
    return ((r.next(26) << 27) + r.next(27)) * (1.0 / (1 << 53))


def _jint_of_double(x):
    """(int) of a double: truncation toward zero, saturating at the int range."""
    return max(INT_MIN_J, min(INT_MAX_J, int(x)))


def rrm_rk(r):
    """ReducingRangeMapTest.rk(Random) (:62-69)."""
    k = r.nextInt()
    if r.nextBoolean():
        k = _i32(-k)
    if k == INT_MAX_J:
        k -= 1
    if k == INT_MIN_J:
        k += 1
    return k


def rrm_add_one(r, max_range_count, max_coverage, min_chance):
    """RandomMap.addOneRandom (:251-275) -> (StartInclusive ranges [s, e) after Ranges.of, hlc of ts(b))."""
    count = 1 if max_range_count == 1 else 1 + r.nextInt(max_range_count - 1)
    b = r.nextInt(INT_MAX_J)
    cov = float(_f32(max_coverage))
    chance = _f32(min_chance)
    ranges = []
    for _ in range(count):
        length = _jint_of_double(2 * next_double(r) * cov * INT_MAX_J)
        if length == 0:
            length = 1
        if next_float(r) <= chance:
            if r.nextBoolean():
                ranges.append((INT_MIN_J + 1, INT_MIN_J + 1 + length))
            else:
                ranges.append((INT_MAX_J - length - 1, INT_MAX_J - 1))
        else:
            start = r.nextInt(INT_MAX_J - length - 1)       # ValueError when the bound is <= 0, as Java throws
            ranges.append((start, start + length))
    return ranges_of(ranges), b


def rrm_validate_probes(r, canonical_keys):
    """The points and foldl queries RandomWithCanonical.validate (:385-470) draws: (points, [(keys, ranges)]).
    points = decr/self/incr of every canonical key (int arithmetic wraps, as IntKey.Routing's does) then 1000
    rk(random); each foldl query is RoutingKeys.of(1 + nextInt(20) random keys) and the Ranges built from them
    (:409-428; [MIN_VALUE, k) / [k, MAX_VALUE) ends use MINIMUM_EXCL / MAXIMUM_EXCL)."""
    points = []
    for k in canonical_keys:
        points += [_i32(k - 1), k, _i32(k + 1)]
    for _ in range(1000):
        points.append(rrm_rk(r))
    folds = []
    for _ in range(100):
        count = 1 + r.nextInt(20)
        keys = sorted(set(rrm_rk(r) for _ in range(count)))
        rs, i = [], 0
        if len(keys) % 2 == 1 and r.nextBoolean():
            rs.append((INT_MIN_J, keys[0]))
            i = 1
        while i + 1 < len(keys):
            rs.append((keys[i], keys[i + 1]))
            i += 2
        if i < len(keys):
            rs.append((keys[i], INT_MAX_J))
        folds.append((keys, ranges_of(rs)))
    return points, folds


def rrm_canonical_keys(additions):
    """The keys of RandomWithCanonical.canonical after the additions (:374-379): MIN_VALUE, MAX_VALUE and every
    range's start and end."""
    ks = {INT_MIN_J, INT_MAX_J}
    for ranges, _ in additions:
        for s, e in ranges:
            ks.add(s)
            ks.add(e)
    return sorted(ks)


def rrm_random_adds(seed, merges, additions, max_ranges, max_coverage, min_chance):
    """ReducingRangeMapTest.testRandomAdds(seed, ...) (:210-232): per merged map its additions [(ranges, b)] and the
    probes its validate drew; the merge choices (random.nextBoolean per merge, :300-302); the probes of the final
    validate over the merged map.  Returns (maps: [(additions, probes)], final_probes)."""
    r = JavaRandom(seed)
    maps = []
    for _ in range(merges):
        adds = [rrm_add_one(r, max_ranges, max_coverage, min_chance) for _ in range(additions)]
        maps.append((adds, rrm_validate_probes(r, rrm_canonical_keys(adds))))
    for _ in maps:
        r.nextBoolean()                           # ReducingRangeMap.merge or mergeIntervals: the same map
    allad = [a for adds, _ in maps for a in adds]
    return maps, rrm_validate_probes(r, rrm_canonical_keys(allad))
