"""Pins the oracle's range-interval overlap join (InMemoryCommandStore.mapReduceRangesInternal :884-1017, the
RangeDeps builder) with the reference's own RangeDepsTest inputs (test/primitives/RangeDepsTest.java).

The test's generators (GenerateRanges, generate, generateIdenticalTxns, generateNemesisRanges :43-233) and
its Validate query sequence (:171-193) are regenerated bit-exactly from the seeds recorded in the test source
(tests/refgen.py: java.util.Random + IEEE-single float arithmetic).  Each case becomes one engine batch: the
test's TxnIds as range Writes holding their Ranges, then one Read per Validate query (a range, a range's
start / end key, a slice).  The oracle's PreAccept RangeDeps of every txn must equal Validate's canonical model
(the stored txns whose Ranges intersect / contain the footprint, each on its intersecting ranges), CSR for CSR.
The fixtures tests/golden/rangedeps_*.npz freeze two of these batches with the model's answers for the GPU
(tests/test_golden.py)."""
import numpy as np
import pytest

import oracle as O
import refgen as R
from accord_amd import abi


def _check(canonical, queries):
    b = R.rangedeps_batch(canonical, queries)
    want = R.rangedeps_expected(canonical, queries)
    res = O.OracleResult(b, abi.make_config(0, 1, 0.0, 1), O.FLAG_MERGE)
    got = res.deps(0, abi.CLASS_RANGE)
    for t, (ks, tx, m) in enumerate(want):
        gk, gt, gm = got.txn(t)
        assert [tuple(int(x) for x in r) for r in gk] == list(ks), "txn %d ranges" % t
        assert list(gt) == tx, "txn %d TxnIds" % t
        assert list(gm) == m, "txn %d rangesToTxnIds" % t
    # every footprint-intersecting stored txn, and only those (Validate's set equality)
    assert sum(len(w[1]) for w in want) > 0
    return b, want


@pytest.mark.parametrize("seed", R.RANGEDEPS_RANDOM_SEEDS)
def test_rangedeps_random_seeds(seed):
    # testRandom: GenerateRanges(1000, 0.01f, 0.3f, 0.1f, 1f), 100 TxnIds, 1000 ranges (:257-270)
    r = R.JavaRandom(seed)
    gen = R.GenerateRanges(1000, 0.01, 0.3, 0.1, 1.0)
    canonical = R.rangedeps_generate(r, gen, 100, 1000)
    _check(canonical, R.rangedeps_validate_queries(r, gen, canonical))


@pytest.mark.parametrize("copies", [1, 2, 7, 64, 499])
def test_rangedeps_identical_txns(copies):
    # testIdenticalTransactions (:272-284): `copies` TxnIds with the same Ranges
    r = R.JavaRandom(R.RANGEDEPS_IDENTICAL_SEED)
    gen = R.GenerateRanges(1000, 0.01, 0.3, 0.1, 1.0)
    canonical = R.rangedeps_identical(r, gen, copies, 1000)
    _check(canonical, R.rangedeps_validate_queries(r, gen, canonical))


@pytest.mark.parametrize("non_nemesis", [0, 1])
def test_rangedeps_nemesis(non_nemesis):
    # testNemesisRanges / testHalfNemesisRanges (:286-325): width 1 + nextInt(511), 1 + nextInt(99) nemesis
    # TxnIds, 1000 ranges; the first iterations of the recorded seed
    r = R.JavaRandom(R.RANGEDEPS_NEMESIS_SEED)
    for _ in range(3):
        width, count = 1 + r.nextInt(511), 1 + r.nextInt(99)
        canonical, gen = R.rangedeps_nemesis(width, count, 1000, non_nemesis)
        _check(canonical, R.rangedeps_validate_queries(r, gen, canonical))


def test_rangedeps_builder_is_canonical():
    # RangeDeps.of(map) (:919-935): the RelationMultiMap builder over (range, TxnId) pairs; the oracle's builder
    # (fed in a shuffled add order) must give sorted unique ranges, every TxnId, and per range exactly the TxnIds
    # holding it
    r = R.JavaRandom(R.RANGEDEPS_RANDOM_SEEDS[1])
    canonical = R.rangedeps_generate(r, R.GenerateRanges(1000, 0.01, 0.3, 0.1, 1.0), 100, 1000)
    pairs = [(rg, t) for t, rs in canonical.items() for rg in rs]
    rng = np.random.default_rng(3)
    order = rng.permutation(len(pairs))
    # range keys through the u64 builder: encode (s, e) order-preservingly as s << 32 | e
    keys = np.array([(pairs[k][0][0] << 32) | pairs[k][0][1] for k in order], np.uint64)
    vals = np.array([pairs[k][1] for k in order], np.uint32)
    # the builder wants each key's values contiguous (Deps.Builder adds key by key): sort by key only
    srt = np.argsort(keys, kind="stable")
    ok, ov, om = O.build_relation(keys[srt], vals[srt])
    uniq = sorted({p[0] for p in pairs})
    assert [((int(k) >> 32), int(k) & 0xFFFFFFFF) for k in ok] == uniq
    assert list(ov) == sorted(canonical)
    for j, rg in enumerate(uniq):
        lo = len(uniq) if j == 0 else int(om[j - 1])
        got = [int(ov[x]) for x in om[lo:int(om[j])]]
        assert got == sorted(t for t, rs in canonical.items() if rg in rs)
