"""Pins the oracle's RelationMultiMap builder and linearUnion (the KeyDeps/RangeDeps CSR arithmetic) to
the reference's own KeyDepsTest, regenerating its seeded inputs bit-exactly (tests/refgen.py) and
checking against the same canonical TreeMap<Key, TreeSet<TxnId>> model:

* testSimpleEquality  (test/primitives/KeyDepsTest.java:432-464)  built CSR == canonical model
* testMergedProperty  (:308-316)  KeyDeps.merge(list) == canonical union == reduce(KeyDeps::with)
* builder             (:319-335)  per-key add order does not matter
* testMerge / main    (:115-126, :612-618)  the seeded inputs, seeds 0..N
* RelationMultiMap.AbstractBuilder rejects a key visited twice (core/utils/RelationMultiMap.java:234-239)
"""
import random

import numpy as np
import pytest

import oracle as O
import refgen


def ranks_of(deps_list):
    allt = sorted({t for d in deps_list for s in d.canonical.values() for t in s}, key=refgen.txn_order_key)
    return {t: i for i, t in enumerate(allt)}


def build(pairs, rank):
    keys = np.array([k for k, _ in pairs], np.uint64)
    vals = np.array([rank[t] for _, t in pairs], np.uint32)
    return O.build_relation(keys, vals)


def check_relation(rel, canonical, rank):
    """KeyDeps layout (KeyDeps.java:153-172): sorted unique keys, sorted unique TxnIds, keysToTxnIds =
    nKeys end offsets (base nKeys) followed by per-key ascending TxnId indices."""
    keys, vals, k2t = rel
    exp_keys = sorted(k for k, s in canonical.items() if s)
    assert list(keys) == exp_keys
    exp_vals = sorted({rank[t] for s in canonical.values() for t in s})
    assert list(vals) == exp_vals
    nk = len(keys)
    if nk == 0:
        assert len(k2t) == 0
        return
    assert len(k2t) == k2t[nk - 1]
    start = nk
    for ki, k in enumerate(keys):
        end = int(k2t[ki])
        idx = [int(x) for x in k2t[start:end]]
        assert idx == sorted(set(idx)), "per-key indices must be strictly ascending"
        assert [int(vals[x]) for x in idx] == sorted(rank[t] for t in canonical[int(k)])
        start = end


def union_canonical(deps_list):
    out = {}
    for d in deps_list:
        for k, s in d.canonical.items():
            out.setdefault(k, set()).update(s)
    return out


def test_java_random_known_values():
    # java.util.Random reference values (spec-defined LCG)
    assert refgen.JavaRandom(42).nextInt() == -1170105035
    assert refgen.JavaRandom(0).nextInt() == -1155484576
    assert refgen.JavaRandom(42).nextInt(10) == 0
    assert refgen.JavaRandom(42).nextLong() == (-5025562857975149833) % (1 << 64)


@pytest.mark.parametrize("lo,hi", [(0, 400), (400, 800)])
def test_testmerge_seeds_main_loop(lo, hi):
    """KeyDepsTest.main's first loop: testMerge(seed, 100, 3, 50, 4, 4, 2, 100, 10, 4) for seeds 0..N."""
    for seed in range(lo, hi):
        deps = refgen.testmerge_inputs(seed)
        rank = ranks_of(deps)
        rels = []
        for d in deps:
            rel = build(d.add_order(), rank) if d.canonical else O.EMPTY_RELATION
            check_relation(rel, d.canonical, rank)
            rels.append(rel)
        merged = O.EMPTY_RELATION
        for rel in rels:                       # LinearMerger folds the list in order
            merged = O.union_relation(merged, rel)
        check_relation(merged, union_canonical(deps), rank)
        rev = O.EMPTY_RELATION
        for rel in rels[::-1]:                 # reduce(with) in any order gives the same canonical form
            rev = O.union_relation(rel, rev)
        assert all(np.array_equal(a, b) for a, b in zip(merged, rev))


def test_testmerge_reference_test_shapes():
    """KeyDepsTest.testMerge's @Test parameter sets (:111-112) at fixed seeds."""
    for seed in range(40):
        for args in ((100, 3, 500, 4, 10, 5, 200, 100, 10), (1000, 3, 500, 4, 100, 10, 200, 1000, 10)):
            deps = refgen.testmerge_inputs(seed, *args)
            rank = ranks_of(deps)
            merged = O.EMPTY_RELATION
            for d in deps:
                rel = build(d.add_order(), rank) if d.canonical else O.EMPTY_RELATION
                check_relation(rel, d.canonical, rank)
                merged = O.union_relation(merged, rel)
            check_relation(merged, union_canonical(deps), rank)


def test_builder_order_independent():
    """KeyDepsTest.builder: keys in order, values shuffled per key -> the same KeyDeps."""
    for seed in range(60):
        r = refgen.JavaRandom(1000 + seed)
        d = refgen.keydeps_generate(r, 300, 3, 500, 0, 4, 50, 5, 400, 600)
        rank = ranks_of([d])
        ref = build(d.add_order(), rank)
        check_relation(ref, d.canonical, rank)
        py = random.Random(seed)
        pairs = []
        for k in sorted(d.canonical):
            ids = list(d.canonical[k])
            py.shuffle(ids)
            pairs.extend((k, t) for t in ids)
        got = build(pairs, rank)
        assert all(np.array_equal(a, b) for a, b in zip(ref, got))


def test_builder_rejects_key_visited_twice():
    with pytest.raises(ValueError):
        O.build_relation(np.array([5, 7, 5], np.uint64), np.array([0, 1, 2], np.uint32))


def test_builder_duplicate_values_deduplicated():
    keys, vals, k2t = O.build_relation(np.array([9, 9, 9, 3], np.uint64), np.array([4, 2, 4, 1], np.uint32))
    assert list(keys) == [3, 9] and list(vals) == [1, 2, 4]
    assert list(k2t) == [3, 5, 0, 1, 2]


def check_inverse(rel, canonical, rank):
    """KeyDepsTest.testSimpleEquality's inverse check (:443-450): participatingKeys(txnId) == invertCanonical()
    for every TxnId, where participatingKeys reads txnIdsToKeys = RelationMultiMap.invert(keysToTxnIds)
    (KeyDeps.java:318-330, :362-367; RelationMultiMap.java:907-938)."""
    keys, vals, k2t = rel
    inv = O.invert(k2t, len(keys), len(vals))
    nt = len(vals)
    assert len(inv) == nt + len(k2t) - len(keys)
    inverted = {}
    for k, s in canonical.items():
        for t in s:
            inverted.setdefault(rank[t], []).append(k)
    assert sorted(inverted) == [int(v) for v in vals]
    start = nt
    for ti, v in enumerate(vals):
        end = int(inv[ti])
        assert [int(keys[x]) for x in inv[start:end]] == sorted(inverted[int(v)])
        start = end
    assert start == len(inv)


def test_invert_matches_invert_canonical():
    """txnIdsToKeys over the KeyDepsTest.main seeds (testMerge inputs, built and merged)."""
    for seed in range(200):
        deps = refgen.testmerge_inputs(seed)
        rank = ranks_of(deps)
        merged = O.EMPTY_RELATION
        for d in deps:
            if not d.canonical:
                continue
            rel = build(d.add_order(), rank)
            check_inverse(rel, d.canonical, rank)
            merged = O.union_relation(merged, rel)
        check_inverse(merged, union_canonical(deps), rank)


def test_invert_edge_cases():
    assert len(O.invert(np.zeros(0, np.int32), 0, 0)) == 0
    # one key, three txns
    assert list(O.invert(np.array([4, 0, 1, 2], np.int32), 1, 3)) == [4, 5, 6, 0, 0, 0]
    # two keys sharing txn 1; the reference layout is nKeys end offsets then indices
    assert list(O.invert(np.array([4, 5, 0, 1, 1], np.int32), 2, 2)) == [3, 5, 0, 0, 1]
    # a TxnId without keys (legal for SerializerSupport input) gets an empty run
    assert list(O.invert(np.array([3, 0, 2], np.int32), 1, 3)) == [4, 4, 5, 0, 0]
