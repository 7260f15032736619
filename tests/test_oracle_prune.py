"""The pruned oracle (FLAG_PRUNE: Pruning.maybePrune restated for the steady state, local/cfk/Pruning.java:164-233;
the mode bench.py's cpu_baseline times, with 1 and with T key-range threads) must give exactly the same
PreAccept deps of every view and class, merged Deps and execution levels / order as the unpruned oracle: pruning
only drops CommandsForKey entries that the elision (CommandsForKey.mapReduceActive :930-962) would skip anyway."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload




def _same(a, b, replicas, levels=True):
    for v in range(replicas):
        for c in range(abi.NUM_CLASSES):
            assert a.deps(v, c).equal(b.deps(v, c)), "view %d class %d" % (v, c)
    for c in range(abi.NUM_CLASSES):
        assert a.merged(c).equal(b.merged(c)), "merged class %d" % c
    if levels:
        la, oa = a.levels()
        lb, ob = b.levels()
        assert np.array_equal(la, lb) and np.array_equal(oa, ob)


@pytest.mark.parametrize("name,n,window,drop", [("C2", 30000, 32, 0.1), ("C3", 30000, 32, 0.1), ("C3", 20000, 0, 0.0),
                                                ("C2", 20000, 4, 0.5)])
def test_pruned_equals_unpruned(name, n, window, drop):
    b = workload.config(name, n=n)
    cfg = abi.make_config(window, 3, drop, workload.SEEDS[name])
    flags = O.FLAG_MERGE | O.FLAG_LEVELS
    _same(O.OracleResult(b, cfg, flags | O.FLAG_PRUNE), O.OracleResult(b, cfg, flags), 3)


def test_pruned_hot_keys_and_bumps():
    b = workload.generate(6000, keys_per_txn=2, keyspace=7, slow_frac=0.5, bump_max=400, seed=17)
    cfg = abi.make_config(6, 2, 0.2, 17)
    flags = O.FLAG_MERGE | O.FLAG_LEVELS
    _same(O.OracleResult(b, cfg, flags | O.FLAG_PRUNE), O.OracleResult(b, cfg, flags), 2)


def test_pruned_mixed_statuses():
    rng = np.random.default_rng(19)
    n = 5000
    status = rng.choice([abi.ST_APPLIED, abi.ST_STABLE, abi.ST_COMMITTED, abi.ST_PREACCEPTED, abi.ST_INVALID,
                         abi.ST_TRANSITIVELY_KNOWN], size=n, p=[0.6, 0.1, 0.1, 0.1, 0.05, 0.05]).astype(np.uint8)
    b = workload.generate(n, keys_per_txn=3, keyspace=60, status=status, slow_frac=0.3, bump_max=100, seed=19)
    cfg = abi.make_config(8, 2, 0.2, 19)
    _same(O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS | O.FLAG_PRUNE),
          O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS), 2)


def test_threaded_pruned_equals_serial():
    # the T-thread key-range-sharded restatement (one single-threaded store per shard, PreAccept.reduce)
    b = workload.config("C2", n=40000)
    cfg = abi.make_config(32, 3, 0.1, workload.SEEDS["C2"])
    flags = O.FLAG_MERGE | O.FLAG_LEVELS | O.FLAG_PRUNE
    _same(O.OracleResult(b, cfg, flags | O.FLAG_KEY_SHARDS, threads=4), O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS), 3)


@pytest.mark.parametrize("name", ["C2", "C3", "C4"])
def test_txn_range_threads_equal_serial(name):
    # the CPU baseline's threading: T threads over TxnId ranges sharing one CFK index, each with its own pruning
    # state (C4: range txns too); deps of every view and class, merged Deps and levels equal the serial oracle's
    b = workload.config(name, n=20000 if name != "C4" else 6000)
    cfg = abi.make_config(32, 3, 0.1, workload.SEEDS[name])
    flags = O.FLAG_MERGE | O.FLAG_LEVELS | O.FLAG_PRUNE
    _same(O.OracleResult(b, cfg, flags, threads=7), O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS), 3)
