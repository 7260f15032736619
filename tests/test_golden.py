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
