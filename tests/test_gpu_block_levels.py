"""Execution levels by executeAt blocks (csrc/block_levels.h) vs the oracle's release-order DP (oracle.cpp
exec_levels: CommandsForKey.notifyManaged + unappliedCounters, local/cfk/CommandsForKey.java:1208-1330).

AD_LEVELS_BLOCKS forces the block path on every key-only batch (short chains included), AUTO takes it when a
key chain is long (Zipf hot keys, dense keyspaces); both must reproduce the oracle's levels and order bit for
bit, including the block-boundary cases (blocks are cut every 1008 entries: batches just below / above,
key-less txns taking a slot, 16-key txns straddling a cut) and far slow-path bumps (the chain-order check
fails and the serial per-key insertion order runs)."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, engine, workload

pytestmark = pytest.mark.gpu

BLOCKS = engine.DepsEngine.LEVELS_BLOCKS


def check_levels(engine_factory, b, mode=BLOCKS, window=32, replicas=2, drop_p=0.1, seed=0xACC0D1, expect_blocks=True,
                 check_depth=True):
    ref = O.OracleResult(b, abi.make_config(window, replicas, drop_p, seed), O.FLAG_MERGE | O.FLAG_LEVELS)
    eng = engine_factory(window=window, replicas=replicas, drop_p=drop_p, seed=seed)
    eng.set_level_mode(mode)
    eng.load(b)
    eng.preaccept_deps()
    eng.merge()
    lv, order, depth = eng.exec_levels()
    rlv, rorder = ref.levels()
    bad = np.nonzero(lv != rlv)[0]
    assert len(bad) == 0, "levels differ at %s (gpu %s, oracle %s)" % (bad[:8], lv[bad[:8]], rlv[bad[:8]])
    assert np.array_equal(order, rorder), "order differs"
    if len(lv) and check_depth:
        assert depth == int(lv.max()) + 1
    st = eng.last_times()
    if expect_blocks:
        assert st["level_blocks"] >= 1, st
    return eng


def _ragged(n, kmin, kmax, keyspace, seed):
    rng = np.random.default_rng(seed)
    b = workload.generate(n, keys_per_txn=1, keyspace=keyspace, seed=seed)
    cnt = rng.integers(kmin, kmax + 1, size=n)
    keys, off = [], [0]
    for c in cnt:
        keys.append(np.sort(rng.choice(keyspace, size=c, replace=False)).astype(np.uint64))
        off.append(off[-1] + c)
    b["keys"] = np.concatenate(keys) if keys else np.zeros(0, np.uint64)
    b["key_off"] = np.array(off, np.uint32)
    return b


@pytest.mark.parametrize("name,n", [("C2", 20000), ("C3", 20000), ("C3", 200000), ("C2", 200000)])
def test_blocks_configs(engine_factory, name, n):
    check_levels(engine_factory, workload.config(name, n=n))


@pytest.mark.parametrize("name,n", [("C3", 200000), ("C3", 20000)])
def test_blocks_wide_scan_words(engine_factory, name, n):
    # the 64-bit packed scan words batches of more than 2^20 txns use (LEVELS_BLOCKS_WIDE forces them here)
    check_levels(engine_factory, workload.config(name, n=n), mode=engine.DepsEngine.LEVELS_BLOCKS_WIDE)
    check_levels(engine_factory, workload.generate(4000, keys_per_txn=4, keyspace=40, seed=7),
                 mode=engine.DepsEngine.LEVELS_BLOCKS_WIDE)


@pytest.mark.parametrize("keyspace,n", [(300, 5000), (40, 3000), (4000, 20000), (3, 2000)])
def test_blocks_dense_keyspaces(engine_factory, keyspace, n):
    # very deep graphs: every block is one or a few long key runs coupled by every txn
    check_levels(engine_factory, workload.generate(n, keys_per_txn=min(4, keyspace), keyspace=keyspace, seed=keyspace + n))


@pytest.mark.parametrize("n", [1, 2, 251, 252, 253, 1007, 1008, 1009, 4095, 4097])
def test_blocks_edge_sizes(engine_factory, n):
    # 4 keys per txn: 252 txns = 1008 entries = one block exactly
    check_levels(engine_factory, workload.generate(n, keyspace=60, seed=n))


def test_blocks_ragged_16_keys(engine_factory):
    check_levels(engine_factory, _ragged(6000, 1, 16, 700, 4))
    check_levels(engine_factory, _ragged(3000, 12, 16, 90, 5))


def test_blocks_far_bumps(engine_factory):
    # slow-path bumps moving executeAt thousands of ranks: the windowed chain order fails its check
    b = workload.generate(20000, keys_per_txn=4, keyspace=500, slow_frac=0.5, bump_max=5000, seed=21)
    check_levels(engine_factory, b)


def test_blocks_all_writes_all_reads(engine_factory):
    n = 5000
    check_levels(engine_factory, workload.generate(n, keyspace=200, kinds=np.full(n, abi.KIND_WRITE), seed=2))
    check_levels(engine_factory, workload.generate(n, keyspace=200, kinds=np.full(n, abi.KIND_READ), seed=3))


@pytest.mark.parametrize("name,n", [("C3", 100000)])
def test_auto_takes_blocks_for_deep_chains(engine_factory, name, n):
    # AUTO: the Kahn chain build finds the hot keys' long chains and hands the batch to the block path
    check_levels(engine_factory, workload.config(name, n=n), mode=engine.DepsEngine.LEVELS_AUTO)


def test_auto_keeps_kahn_for_short_chains(engine_factory):
    eng = check_levels(engine_factory, workload.config("C2", n=50000), mode=engine.DepsEngine.LEVELS_AUTO,
                       expect_blocks=False)
    assert eng.last_times()["level_blocks"] == 0


def test_blocks_pipeline_repeat(engine_factory):
    # the device pipeline twice on one handle (buffers reused), then a different deep batch
    eng = engine_factory(window=32, replicas=3, drop_p=0.1, seed=0xACC0D2)
    cfg = abi.make_config(32, 3, 0.1, 0xACC0D2)
    for b in (workload.config("C3", n=60000), workload.config("C3", n=60000), workload.config("C3", n=90000, seed=3)):
        eng.load(b)
        for _ in range(2):
            eng.run_pipeline()
            lv, order = eng.fetch_levels()
            rlv, rorder = O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS).levels()
            assert np.array_equal(lv, rlv) and np.array_equal(order, rorder)
        assert eng.last_times()["level_blocks"] > 0


def test_long_chain_hint_alternating_batches(engine_factory):
    # AUTO on one handle: after a deep batch the next batch is first tested for long chains (one light kernel)
    # and goes straight to the block path; a short-chain batch after it must fall back to the pull path
    eng = engine_factory(window=32, replicas=3, drop_p=0.1, seed=0xACC0D2)
    eng.set_level_mode(engine.DepsEngine.LEVELS_AUTO)
    cfg = abi.make_config(32, 3, 0.1, 0xACC0D2)
    for name, n, blocks in (("C3", 60000, True), ("C3", 60000, True), ("C2", 50000, False), ("C2", 50000, False),
                            ("C3", 90000, True)):
        b = workload.config(name, n=n)
        eng.load(b)
        eng.run_pipeline()
        lv, order = eng.fetch_levels()
        rlv, rorder = O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS).levels()
        assert np.array_equal(lv, rlv) and np.array_equal(order, rorder), (name, n)
        assert (eng.last_times()["level_blocks"] > 0) == blocks, (name, n)


def test_blocks_mode_with_sync_points_takes_relaxation(engine_factory):
    # the block path covers pure Read/Write key batches only: with sync points a forced BLOCKS run resolves the
    # unmanaged waits on the relaxation path (its iteration count is not the depth) and still equals the oracle
    n = 2000
    kinds = np.where(np.arange(n) % 7 == 3, abi.KIND_SYNC_POINT, abi.KIND_WRITE)
    b = workload.generate(n, keyspace=100, kinds=kinds, seed=6)
    eng = check_levels(engine_factory, b, window=8, replicas=1, drop_p=0.0, expect_blocks=False, check_depth=False)
    assert eng.last_times()["level_blocks"] == 0
