"""ad_accept_deps (Accept.calculatePartialDeps :113-116 / GetDeps.apply :76: PreAccept.calculatePartialDeps with
bound = executeAt) vs the oracle's executeAt-bound mode (oracle.cpp: Oracle.accept), every view and class, then
Deps.merge of those replies; key batches (small and >16-key txns), Zipf hot keys, far slow-path bumps, mixed kinds,
range txns."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload

pytestmark = pytest.mark.gpu


def check_accept(engine_factory, b, window=32, replicas=3, drop_p=0.1, seed=0xACC0D1, bound_max=False):
    # bound_max: GetEphemeralReadDeps (bound Timestamp.MAX, GetEphemeralReadDeps.java:76) vs the oracle's MAX bound
    cfg = abi.make_config(window, replicas, drop_p, seed)
    ref = O.OracleResult(b, cfg, O.FLAG_MERGE | (O.FLAG_BOUND_MAX if bound_max else O.FLAG_ACCEPT))
    eng = engine_factory(window=window, replicas=replicas, drop_p=drop_p, seed=seed)
    eng.load(b)
    if bound_max:
        eng.ephemeral_read_deps()
    else:
        eng.accept_deps()
    for v in range(replicas):
        for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY, abi.CLASS_RANGE):
            got, want = eng.fetch_deps(v, c), ref.deps(v, c)
            i = got.first_difference(want)
            assert i is None, "view %d class %d txn %d: gpu %s oracle %s" % (v, c, i, got.txn(i), want.txn(i))
    eng.merge()
    for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY, abi.CLASS_RANGE):
        assert eng.fetch_merged(c).equal(ref.merged(c)), "merged class %d" % c
    return eng, ref


@pytest.mark.parametrize("name,n", [("C2", 20000), ("C3", 20000), ("C2", 200000)])
def test_accept_configs(engine_factory, name, n):
    check_accept(engine_factory, workload.config(name, n=n))


def test_accept_slow_paths_far_bumps(engine_factory):
    b = workload.generate(20000, keys_per_txn=3, keyspace=400, slow_frac=0.5, bump_max=3000, seed=17)
    check_accept(engine_factory, b, window=16)


def test_accept_window_zero_and_hot_keys(engine_factory):
    b = workload.generate(6000, keys_per_txn=2, keyspace=5, slow_frac=0.4, bump_max=200, seed=18)
    check_accept(engine_factory, b, window=0)


def test_accept_mixed_kinds(engine_factory):
    rng = np.random.default_rng(19)
    n = 6000
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT,
                        abi.KIND_EXCLUSIVE_SYNC_POINT], size=n, p=[0.35, 0.35, 0.1, 0.1, 0.1])
    status = rng.choice([abi.ST_APPLIED, abi.ST_COMMITTED, abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN], size=n,
                        p=[0.7, 0.1, 0.1, 0.1]).astype(np.uint8)
    b = workload.generate(n, keys_per_txn=3, keyspace=150, kinds=kinds, status=status, slow_frac=0.3, bump_max=100,
                          seed=19)
    check_accept(engine_factory, b, window=8)


def test_accept_large_txns(engine_factory):
    # > 16 keys: the virtual-item walk starts at the bound's position in every key segment
    rng = np.random.default_rng(20)
    base = workload.generate(1500, keys_per_txn=1, keyspace=300, slow_frac=0.4, bump_max=80, seed=20)
    cnt = rng.integers(1, 41, size=1500)
    keys, off = [], [0]
    for c in cnt:
        keys.append(np.sort(rng.choice(300, size=c, replace=False)).astype(np.uint64))
        off.append(off[-1] + c)
    base["keys"] = np.concatenate(keys)
    base["key_off"] = np.array(off, np.uint32)
    check_accept(engine_factory, base, window=12)


def test_accept_range_txns(engine_factory):
    b = workload.generate(8000, 4, 40_000, "uniform", range_frac=0.15, range_width_max=400, slow_frac=0.3,
                          bump_max=100, seed=21)
    check_accept(engine_factory, b, window=8)


def test_accept_then_preaccept_on_one_handle(engine_factory):
    # the bound mode does not stick: a PreAccept run after an Accept run answers with TxnId bounds again
    b = workload.config("C3", n=10000)
    eng, _ = check_accept(engine_factory, b)
    cfg = abi.make_config(32, 3, 0.1, 0xACC0D1)
    ref = O.OracleResult(b, cfg, O.FLAG_MERGE)
    eng.preaccept_deps()
    for v in range(3):
        assert eng.fetch_deps(v, abi.CLASS_KEY).equal(ref.deps(v, abi.CLASS_KEY))


@pytest.mark.parametrize("case", ["C2", "C3", "hot", "mixed", "large", "ranges"])
def test_ephemeral_read_deps_bound_max(engine_factory, case):
    # GetEphemeralReadDeps: every witnessed txn of the txn's keys / ranges, later TxnIds included, the window at the
    # batch's end; every view and class and the merged Deps vs the oracle
    rng = np.random.default_rng(41)
    if case in ("C2", "C3"):
        b, w = workload.config(case, n=20000), 32
    elif case == "hot":
        b, w = workload.generate(6000, keys_per_txn=2, keyspace=5, slow_frac=0.4, bump_max=200, seed=42), 0
    elif case == "mixed":
        n = 6000
        kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT,
                            abi.KIND_EXCLUSIVE_SYNC_POINT], size=n, p=[0.35, 0.35, 0.1, 0.1, 0.1])
        status = rng.choice([abi.ST_APPLIED, abi.ST_COMMITTED, abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN], size=n,
                            p=[0.7, 0.1, 0.1, 0.1]).astype(np.uint8)
        b, w = workload.generate(n, keys_per_txn=3, keyspace=150, kinds=kinds, status=status, slow_frac=0.3,
                                 bump_max=100, seed=43), 8
    elif case == "large":
        b, w = workload.generate(3000, keys_per_txn=24, keyspace=2000, seed=44), 16
    else:
        b, w = workload.generate(8000, keys_per_txn=3, keyspace=20000, range_frac=0.15, range_width_max=3000, seed=45), 16
    eng, ref = check_accept(engine_factory, b, window=w, bound_max=True)
    # later TxnIds do appear (the PreAccept bound would leave them out)
    got = eng.fetch_deps(0, abi.CLASS_KEY)
    later = 0
    for i in range(0, b["n"], 97):
        later += int((got.txn(i)[1] > i).sum())
    assert later > 0


def test_accept_rejects_executeat_below_txnid(engine_factory):
    # an executeAt below its TxnId is no Accept / GetDeps bound (the arrival search assumes
    # executeAt >= TxnId); the batch is refused with IllegalArgumentException, and PreAccept on it still works
    from accord_amd import engine
    b = workload.config("C2", n=5000)
    b["exec_lsb"] = b["exec_lsb"].copy()
    b["exec_lsb"][1234] = b["txn_lsb"][1234] - np.uint64(7 << 16)
    eng = engine_factory()
    eng.load(b)
    with pytest.raises(engine.IllegalArgumentException):
        eng.accept_deps()
    eng.preaccept_deps()
