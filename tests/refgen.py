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
