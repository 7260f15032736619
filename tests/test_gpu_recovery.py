"""BeginRecovery's store queries on the device (ad_recover, csrc/recovery_kernels.h) equal the oracle
(oracle_recover, pinned by tests/test_oracle_recovery.py) on the same batch and the same per-txn Deps: the
hand-built known answers (Deps supplied through ad_merge_host), seeded mixed batches whose Deps are the device's own
merged Accept-bound deps (keys, ranges, all five kinds), and a 200k-txn batch with 20k recovering txns."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, engine, workload
from batchkit import make_batch
from test_oracle_recovery import (_kat, _mixed, merged_from, entries, R, W, SP, ER, KEY, DIRECT, RANGE)
from batchkit import T

pytestmark = pytest.mark.gpu


def _same(got, want, rows):
    (go, gr), (wo, wr) = got, want
    for which in range(2):
        for c in range(3):
            for q in range(len(rows)):
                assert entries(go, which, c, q) == entries(wo, which, c, q), "row %d which %d class %d" % (rows[q], which, c)
    assert np.array_equal(gr, wr)


def _host_deps(engine_factory, b, merged, rows):
    eng = engine_factory(window=0, replicas=1, drop_p=0.0)
    eng.load(b)
    eng.preaccept_deps()
    eng.merge_host([merged])
    return eng.recover(rows)


def test_gpu_kats(engine_factory):
    b = _kat()
    A, E, B, Bacc, Tr, C, D = range(7)
    deps = {A: {KEY: {5: [Tr]}}, B: {KEY: {5: [A]}}, Bacc: {KEY: {5: [A]}}, C: {KEY: {7: [Tr]}}, D: {KEY: {5: [A, B]}}}
    m = merged_from(7, deps)
    got = _host_deps(engine_factory, b, m, [Tr])
    assert entries(got[0], 0, KEY, 0) == [(5, A)] and entries(got[0], 1, KEY, 0) == [(5, B)] and got[1][0] == 1
    _same(got, O.recover(b, m, [Tr]), [Tr])
    txns = [T(10, W, keys=[5], exec_hlc=100, status=abi.ST_STABLE), T(20, SP, keys=[5], exec_hlc=90, status=abi.ST_COMMITTED),
            T(30, W, ranges=[(0, 10)], status=abi.ST_PREACCEPTED), T(40, ER, keys=[5], status=abi.ST_PREACCEPTED),
            T(50, W, ranges=[(3, 8), (20, 30)], exec_hlc=120, status=abi.ST_COMMITTED)]
    b = make_batch(txns)
    deps = {0: {RANGE: {(0, 10): [2]}}, 1: {KEY: {5: [0]}}, 4: {RANGE: {(3, 8): [2]}}}
    m = merged_from(5, deps)
    rows = [2, 3, 4, 0]
    got = _host_deps(engine_factory, b, m, rows)
    assert entries(got[0], 1, DIRECT, 0) == [(5, 1)]
    _same(got, O.recover(b, m, rows), rows)


@pytest.mark.parametrize("n,keyspace,range_frac,window,drop,seed", [
    (600, 60, 0.0, 16, 0.3, 1), (900, 200, 0.15, 32, 0.2, 2), (500, 40, 0.3, 0, 0.0, 3), (5000, 400, 0.05, 32, 0.3, 4)])
def test_gpu_mixed_equals_oracle(engine_factory, n, keyspace, range_frac, window, drop, seed):
    b = _mixed(n, keyspace, range_frac, seed)
    eng = engine_factory(window=window, replicas=1, drop_p=drop, seed=seed)
    eng.load(b)
    eng.accept_deps()
    eng.merge()
    merged = [eng.fetch_merged(c) for c in range(3)]
    rows = [i for i in range(n) if b["status"][i] < abi.ST_COMMITTED]
    rows += [i for i in range(n) if b["status"][i] >= abi.ST_COMMITTED][:20]    # PreCommitted: empty answers
    got = eng.recover(rows)
    want = O.recover(b, merged, rows)
    _same(got, want, rows)
    assert sum(len(got[0][w][c][2]) for w in range(2) for c in range(3)) > 0 and got[1].any()


def test_gpu_large_key_batch(engine_factory):
    rng = np.random.default_rng(11)
    n = 200_000
    kinds = rng.choice([R, W, SP], size=n, p=[0.45, 0.5, 0.05])
    status = rng.choice([abi.ST_APPLIED, abi.ST_STABLE, abi.ST_COMMITTED, abi.ST_ACCEPTED, abi.ST_PREACCEPTED],
                        size=n, p=[0.4, 0.15, 0.15, 0.15, 0.15]).astype(np.uint8)
    b = workload.generate(n, keys_per_txn=4, keyspace=200_000, kinds=kinds, status=status, slow_frac=0.3,
                          bump_max=60, seed=11)
    eng = engine_factory(window=32, replicas=3, drop_p=0.1, seed=5)
    eng.load(b)
    eng.accept_deps()
    eng.merge()
    merged = [eng.fetch_merged(c) for c in range(3)]
    cand = np.nonzero(b["status"] < abi.ST_COMMITTED)[0]
    rows = np.sort(rng.choice(cand, size=20_000, replace=False)).astype(np.uint32)
    got = eng.recover(rows)
    want = O.recover(b, merged, rows)
    _same(got, want, rows)


def test_gpu_recover_state_errors(engine_factory):
    b = _mixed(300, 40, 0.0, 7)
    eng = engine_factory(window=16, replicas=1, drop_p=0.0)
    eng.load(b)
    with pytest.raises(engine.AccordDepsError):
        eng.recover([0])                              # no deps / merged Deps yet
    eng.preaccept_deps()
    eng.merge()
    with pytest.raises(engine.AccordDepsError):
        eng.recover([300])                            # row out of range
    out, rej = eng.recover([])
    assert len(rej) == 0 and all(len(out[w][c][2]) == 0 for w in range(2) for c in range(3))
