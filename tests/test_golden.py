"""Golden fixtures (tests/golden/*.npz, written by tests/golden/make_golden.py).

CPU: the oracle still reproduces every fixture byte for byte.  GPU: the HIP path, through the C-ABI,
reproduces them too (deps of every replica view and class, merged Deps, execution levels and order).
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

import make_golden as G  # noqa: E402
import oracle as O  # noqa: E402
from accord_amd import abi  # noqa: E402

NAMES = sorted(G.CASES)


def _cmp(name, got, z, prefix, is_range):
    want = G.csr_from(z, prefix, is_range)
    if not got.equal(want):
        i = got.first_difference(want)
        raise AssertionError("%s %s differs at txn %s" % (name, prefix, i))


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    b, (w, r, p, s), z = G.load(name)
    levels = "level" in z
    res = O.OracleResult(b, abi.make_config(w, r, p, s), O.FLAG_MERGE | (O.FLAG_LEVELS if levels else 0))
    for v in range(r):
        for c in range(abi.NUM_CLASSES):
            _cmp(name, res.deps(v, c), z, "deps_%d_%d_" % (v, c), c == abi.CLASS_RANGE)
    for c in range(abi.NUM_CLASSES):
        _cmp(name, res.merged(c), z, "merged_%d_" % c, c == abi.CLASS_RANGE)
    if levels:
        lv, order = res.levels()
        assert np.array_equal(lv, z["level"]) and np.array_equal(order, z["order"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_reproduces_golden(engine_factory, name):
    b, (w, r, p, s), z = G.load(name)
    eng = engine_factory(window=w, replicas=r, drop_p=p, seed=s)
    eng.load(b)
    eng.preaccept_deps()
    for v in range(r):
        for c in range(abi.NUM_CLASSES):
            _cmp(name, eng.fetch_deps(v, c), z, "deps_%d_%d_" % (v, c), c == abi.CLASS_RANGE)
    eng.merge()
    for c in range(abi.NUM_CLASSES):
        _cmp(name, eng.fetch_merged(c), z, "merged_%d_" % c, c == abi.CLASS_RANGE)
    if "level" in z:
        lv, order, _ = eng.exec_levels()
        assert np.array_equal(lv, z["level"]), "levels differ"
        assert np.array_equal(order, z["order"]), "order differs"


def _keydeps_replies(z):
    r = int(z["cfg"][1])
    reps = [G.csr_from(z, "reply_%d_" % v, False) for v in range(r)]
    n = reps[0].n
    empty = abi.Csr(np.zeros(n + 1, np.uint32), np.zeros(0, np.uint64), np.zeros(n + 1, np.uint32), np.zeros(0, np.int32),
                    np.zeros(n + 1, np.uint32), np.zeros(0, np.uint32))
    empty_r = abi.Csr(np.zeros(n + 1, np.uint32), np.zeros(0, np.uint64), np.zeros(n + 1, np.uint32), np.zeros(0, np.int32),
                      np.zeros(n + 1, np.uint32), np.zeros(0, np.uint32), is_range=True)
    return [[rep, empty, empty_r] for rep in reps]


def test_keydeps_merge_fixture_reproduces():
    # KeyDepsTest.testMerge seeds 0..63 (tests/refgen.py) folded by the oracle's LinearMerger: still the fixture
    batch, replies, merged = G.keydeps_merge_case()
    z = dict(np.load(os.path.join(HERE, "golden", "keydeps_merge.npz")))
    for v, rep in enumerate(replies):
        assert rep.equal(G.csr_from(z, "reply_%d_" % v, False))
    assert merged.equal(G.csr_from(z, "merged_0_", False))


@pytest.mark.gpu
def test_gpu_keydeps_merge_golden(engine_factory):
    # the reference's own KeyDepsTest merge inputs through ad_merge_host (validated upload + R-way device merge)
    z = dict(np.load(os.path.join(HERE, "golden", "keydeps_merge.npz")))
    b = {"n": int(len(z["in_txn_msb"]))}
    for f in abi.BATCH_FIELDS:
        b[f] = z.get("in_" + f)
    r = int(z["cfg"][1])
    eng = engine_factory(window=0, replicas=r, drop_p=0.0, seed=0)
    eng.load(b)
    eng.merge_host(_keydeps_replies(z))
    _cmp("keydeps_merge", eng.fetch_merged(abi.CLASS_KEY), z, "merged_0_", False)
