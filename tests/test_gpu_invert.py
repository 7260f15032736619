"""ad_fetch_inverse — KeyDeps.txnIdsToKeys / RangeDeps.txnIdsToRanges on the device.

The reference builds the txn -> keys inverse lazily per Deps with RelationMultiMap.invert
(utils/RelationMultiMap.java:907-938; KeyDeps.java:362-367, RangeDeps.java:576-582).  The device inverts every
row of a window at once (invert_kernels.h).  Checked bit-exact against the oracle's restatement of invert
(oracle.cpp oracle_invert, itself pinned to KeyDepsTest's invertCanonical model in test_oracle_keydeps.py) applied
row by row to the same CSRs: replica views and the merged Deps of C2 / C4-shaped batches, every class, row windows,
and the KeyDepsTest merge inputs (tests/golden/keydeps_merge.npz) through ad_merge_host.
"""
import os

import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def oracle_inverse(csr, lo, hi):
    off, parts = [0], []
    for i in range(lo, hi):
        nk = int(csr.key_off[i + 1] - csr.key_off[i])
        nt = int(csr.txn_off[i + 1] - csr.txn_off[i])
        k2t = csr.k2t[csr.k2t_off[i]:csr.k2t_off[i + 1]]
        inv = O.invert(k2t, nk, nt) if nt else np.zeros(0, np.int32)
        parts.append(inv)
        off.append(off[-1] + len(inv))
    return np.array(off, np.uint32), (np.concatenate(parts) if parts else np.zeros(0, np.int32)).astype(np.int32)


def check(eng, view, cls, csr, lo=0, hi=None):
    hi = csr.n if hi is None else hi
    off, inv = eng.fetch_inverse(view, cls, lo, hi)
    roff, rinv = oracle_inverse(csr, lo, hi)
    assert np.array_equal(off, roff), "inverse offsets differ (view %d class %d rows %d..%d)" % (view, cls, lo, hi)
    assert np.array_equal(inv, rinv), "inverse differs (view %d class %d rows %d..%d)" % (view, cls, lo, hi)
    return len(inv)


@pytest.mark.parametrize("cfg,n", [("C2", 20000), ("C3", 20000), ("C4", 8000)])
def test_inverse_views_and_merged(engine_factory, cfg, n):
    batch = workload.config(cfg, n=n)
    R = 3
    eng = engine_factory(window=32, replicas=R, drop_p=0.1, seed=workload.SEEDS[cfg])
    eng.load(batch)
    eng.preaccept_deps()
    total = 0
    for v in range(R):
        for c in range(abi.NUM_CLASSES):
            total += check(eng, v, c, eng.fetch_deps(v, c))
    eng.merge()
    for c in range(abi.NUM_CLASSES):
        m = eng.fetch_merged(c)
        total += check(eng, R, c, m)
        # row windows (paged inverse), including empty and one-row windows
        for lo, hi in ((0, 0), (17, 18), (n // 3, n // 2), (n - 5, n)):
            check(eng, R, c, m, lo, hi)
    assert total > 0


def test_inverse_keydeps_test_inputs(engine_factory):
    """Each row's Deps = one KeyDepsTest.testMerge input set merged (seeds 0..63, tests/golden/keydeps_merge.npz)."""
    z = dict(np.load(os.path.join(HERE, "golden", "keydeps_merge.npz")))
    b = {"n": int(len(z["in_txn_msb"]))}
    for f in abi.BATCH_FIELDS:
        b[f] = z.get("in_" + f)
    r = int(z["cfg"][1])
    from test_golden import _keydeps_replies
    eng = engine_factory(window=0, replicas=r, drop_p=0.0, seed=0)
    eng.load(b)
    eng.merge_host(_keydeps_replies(z))
    m = eng.fetch_merged(abi.CLASS_KEY)
    assert check(eng, r, abi.CLASS_KEY, m) > 0


def test_inverse_errors(engine_factory):
    batch = workload.config("C2", n=1000)
    eng = engine_factory(window=32, replicas=1, drop_p=0.0, seed=1)
    eng.load(batch)
    with pytest.raises(RuntimeError):
        eng.fetch_inverse(0, abi.CLASS_KEY)          # before ad_preaccept_deps
    eng.preaccept_deps()
    with pytest.raises(RuntimeError):
        eng.fetch_inverse(1, abi.CLASS_KEY)          # merged before ad_merge_deps
    with pytest.raises(RuntimeError):
        eng.fetch_inverse(0, 3)
    with pytest.raises(RuntimeError):
        eng.fetch_inverse(0, abi.CLASS_KEY, 10, 2000)
    off, inv = eng.fetch_inverse(0, abi.CLASS_RANGE)   # an empty class: all-zero offsets
    assert not off.any() and len(inv) == 0
