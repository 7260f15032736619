"""GPU parity: the HIP path (through the C-ABI) vs the CPU oracle, bit-exact.

Compared per txn: PreAccept PartialDeps of every replica view (keyDeps + directKeyDeps in the exact
KeyDeps.SerializerSupport layout), the merged Deps, and execution levels + order.
"""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload

pytestmark = pytest.mark.gpu


def _assert_csr(name, got, want):
    if got.equal(want):
        return
    i = got.first_difference(want)
    raise AssertionError("%s differs at txn %s:\n gpu=%s\n cpu=%s" % (name, i, got.txn(i) if i is not None and i < got.n else None,
                                                                      want.txn(i) if i is not None and i < want.n else None))


def check(engine_factory, batch, window=32, replicas=3, drop_p=0.1, seed=0xACC0D1, levels=True, fixpoint=False, eng=None):
    cfg = abi.make_config(window, replicas, drop_p, seed)
    flags = O.FLAG_MERGE | (O.FLAG_LEVELS if levels else 0)
    ref = O.OracleResult(batch, cfg, flags)
    if eng is None:
        eng = engine_factory(window=window, replicas=replicas, drop_p=drop_p, seed=seed)
    if fixpoint:
        eng.set_level_mode(fixpoint)          # True: the chain fixpoint; an int: that AD_LEVELS_* mode
    eng.load(batch)
    eng.preaccept_deps()
    for v in range(replicas):
        for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY, abi.CLASS_RANGE):
            _assert_csr("deps view %d %s" % (v, abi.CLASS_NAMES[c]), eng.fetch_deps(v, c), ref.deps(v, c))
    eng.merge()
    for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY, abi.CLASS_RANGE):
        _assert_csr("merged %s" % abi.CLASS_NAMES[c], eng.fetch_merged(c), ref.merged(c))
    if levels:
        lv, order, iters = eng.exec_levels()
        rlv, rorder = ref.levels()
        assert np.array_equal(lv, rlv), "levels differ at %s" % np.nonzero(lv != rlv)[0][:10]
        assert np.array_equal(order, rorder), "order differs"
    return ref


@pytest.mark.parametrize("name,n", [("C2", 20000), ("C3", 20000), ("C2", 200000)])
def test_configs_small(engine_factory, name, n):
    check(engine_factory, workload.config(name, n=n))


@pytest.mark.parametrize("fixpoint", [False, True, 3])
@pytest.mark.parametrize("keyspace,n", [(10_000_000, 200000), (40000, 20000), (4000, 6000), (300, 2000)])
def test_levels_kahn_and_fixpoint(engine_factory, keyspace, n, fixpoint):
    # short key chains and no range txns: AUTO takes the one-pass pull levels, 3 (AD_LEVELS_KAHN) the Kahn
    # wavefront, FIXPOINT the chain fixpoint; all must give the oracle's levels and order (the denser keyspaces
    # give deeper graphs, up to long chains)
    b = workload.generate(n, keys_per_txn=4, keyspace=keyspace, seed=keyspace % 97 + n)
    check(engine_factory, b, fixpoint=fixpoint)


@pytest.mark.parametrize("bump", [5000, 10 ** 7])
def test_pull_levels_far_bumps(engine_factory, bump):
    # the pull levels wait for predecessors with a smaller executeAt; a slow-path bump makes some of them later
    # TxnIds (later workgroups): near ones are dispatched as earlier workgroups retire, and if lanes wait too
    # long the pass aborts into the Kahn wavefronts — the levels are the oracle's either way
    b = workload.generate(30000, keys_per_txn=4, keyspace=20000, slow_frac=0.3, bump_max=bump, seed=bump % 1000 + 7)
    check(engine_factory, b)
    check(engine_factory, b, fixpoint=3)


@pytest.mark.parametrize("name,bump", [("C2", 16), ("bumps", 5000), ("hot", 60)])
def test_pull_levels_forced_abort(engine_factory, name, bump):
    # the pull levels' abort path (placeholder levels, the abort flag, levels re-zeroed, chains rebuilt in
    # successor mode, Kahn wavefronts) forced on every lane (AD_LEVELS_PULL_ABORT): the oracle's levels and order
    if name == "C2":
        b = workload.config("C2", n=60000, seed=31)
    else:
        b = workload.generate(30000, keys_per_txn=4, keyspace=20000 if name == "bumps" else 8000, slow_frac=0.3,
                              bump_max=bump, seed=bump + 3)
    eng = engine_factory()
    check(engine_factory, b, fixpoint=4, eng=eng)
    assert eng.last_times()["level_path"] == 3, "the pull pass must have aborted into the Kahn wavefronts"


def test_pull_levels_far_predecessors_full_size(engine_factory):
    # 1,048,576 txns where slow-path bumps move executeAt millions of ranks ahead, so a txn's
    # predecessor can be a TxnId far after it, in a workgroup not resident while the waiting lanes occupy the
    # chip.  The chain build flags predecessors more than 65536 rows ahead and the batch takes the Kahn
    # wavefronts directly (no ~1 s spin until the abort cap): levels / order equal the Kahn mode's (which is
    # oracle-checked at every smaller size), in well under a second.
    import time
    b = workload.generate(1 << 20, keys_per_txn=4, keyspace=10_000_000, slow_frac=0.2, bump_max=10 ** 7, seed=77)
    eng = engine_factory()
    eng.load(b)
    eng.preaccept_deps()
    eng.merge()
    eng.exec_levels()                                   # warm-up (allocations)
    t0 = time.perf_counter()
    lv, order, _ = eng.exec_levels()
    dt = time.perf_counter() - t0
    assert eng.last_times()["level_path"] == 2, "far predecessors must send the batch to the Kahn wavefronts"
    assert dt < 0.5, "levels took %.3f s" % dt
    eng.set_level_mode(3)
    klv, korder, _ = eng.exec_levels()
    assert np.array_equal(lv, klv) and np.array_equal(order, korder)
    # and the near case stays on the pull pass
    c2 = engine_factory()
    c2.load(workload.config("C2", n=1 << 20))
    c2.preaccept_deps()
    c2.merge()
    c2.exec_levels()
    assert c2.last_times()["level_path"] == 1


@pytest.mark.parametrize("fixpoint", [False, True])
def test_order_far_bumps(engine_factory, fixpoint):
    # slow-path bumps that move executeAt hundreds of ranks: the windowed-rank order fast path fails its
    # verification (sync path: radix fallback at once; optimistic Kahn path: redone after the sync)
    b = workload.generate(20000, keys_per_txn=4, keyspace=10_000_000, slow_frac=0.5, bump_max=5000, seed=21)
    check(engine_factory, b, fixpoint=fixpoint)
    eng = engine_factory()
    eng.load(b)
    eng.run_pipeline()                # optimistic order inside the device pipeline, redone after its sync
    lv, order = eng.fetch_levels()
    ref = O.OracleResult(b, abi.make_config(32, 3, 0.1, 0xACC0D1), O.FLAG_MERGE | O.FLAG_LEVELS)
    rlv, rorder = ref.levels()
    assert np.array_equal(lv, rlv) and np.array_equal(order, rorder)


def test_pipeline_levels_equal_oracle(engine_factory):
    b = workload.config("C2", n=50000, seed=9)
    eng = engine_factory()
    eng.load(b)
    for _ in range(2):
        eng.run_pipeline()
        lv, order = eng.fetch_levels()
        rlv, rorder = O.OracleResult(b, abi.make_config(32, 3, 0.1, 0xACC0D1), O.FLAG_MERGE | O.FLAG_LEVELS).levels()
        assert np.array_equal(lv, rlv) and np.array_equal(order, rorder)


def test_repeated_batches_one_engine(engine_factory):
    # a handle reuses its device buffers across batches: the deps offsets scan then also lays out the
    # per-txn CSR rows in place (fused), falling back to the separate layout kernel when a batch outgrows
    # the buffers; every batch must still match the oracle
    eng = engine_factory()
    batches = [workload.config("C2", n=20000), workload.config("C3", n=20000, seed=5),
               workload.config("C2", n=60000, seed=6), workload.config("C2", n=20000),
               workload.generate(3000, keys_per_txn=1, keyspace=40, seed=8)]
    for b in batches:
        check(engine_factory, b, eng=eng)


def test_c3_more_views_no_drop(engine_factory):
    b = workload.config("C3", n=30000, seed=77)
    check(engine_factory, b, replicas=1, drop_p=0.0)
    check(engine_factory, b, replicas=5, drop_p=0.3, seed=5)


def test_snapshot_window_zero(engine_factory):
    check(engine_factory, workload.config("C3", n=5000, seed=3), window=0)


def test_undecided_execute_at_is_not_read(engine_factory):
    # the boundary needs no executeAt for a txn that is not committed (the reference's TxnInfo has none before
    # COMMITTED): with W = 0 (the plain snapshot a CommandStore holds) the deps of every view and the merged Deps
    # are the same whether undecided rows carry their eventual executeAt or just their TxnId
    rng = np.random.default_rng(21)
    n = 8000
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT],
                       size=n, p=[0.4, 0.4, 0.1, 0.1])
    status = rng.choice([abi.ST_APPLIED, abi.ST_STABLE, abi.ST_COMMITTED, abi.ST_PREACCEPTED, abi.ST_ACCEPTED,
                         abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN, abi.ST_HISTORICAL], size=n,
                        p=[0.3, 0.1, 0.1, 0.2, 0.1, 0.1, 0.05, 0.05]).astype(np.uint8)
    a = workload.generate(n, keys_per_txn=3, keyspace=300, kinds=kinds, status=status, slow_frac=0.5, seed=22)
    b = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in a.items()}
    undecided = ~np.isin(status, [abi.ST_COMMITTED, abi.ST_STABLE, abi.ST_APPLIED])
    for f, g in (("exec_msb", "txn_msb"), ("exec_lsb", "txn_lsb"), ("exec_node", "txn_node")):
        b[f][undecided] = a[g][undecided]
    assert undecided.sum() > 1000 and not np.array_equal(a["exec_lsb"], b["exec_lsb"])
    got = []
    for batch in (a, b):
        eng = engine_factory(window=0, replicas=2, drop_p=0.0, seed=1)
        eng.load(batch)
        eng.preaccept_deps()
        eng.merge()
        got.append([eng.fetch_deps(v, c) for v in range(2) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)] +
                   [eng.fetch_merged(c) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)])
    for x, y in zip(*got):
        assert x.equal(y)
    check(engine_factory, b, window=0, replicas=2, drop_p=0.0, levels=False)     # and the oracle agrees


def test_hot_single_key_and_big_bumps(engine_factory):
    # every txn on one of 3 keys; slow path bumps far beyond the window's hlc span exercise the exact
    # maxCommittedWriteBefore fallback (executeAt of an applied write >= the query's TxnId)
    b = workload.generate(4000, keys_per_txn=2, keyspace=3, slow_frac=0.5, bump_max=600, seed=11)
    check(engine_factory, b, window=4)


def test_mixed_kinds_and_statuses(engine_factory):
    rng = np.random.default_rng(9)
    n = 6000
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT,
                        abi.KIND_EXCLUSIVE_SYNC_POINT], size=n, p=[0.35, 0.35, 0.1, 0.1, 0.1])
    status = rng.choice([abi.ST_APPLIED, abi.ST_STABLE, abi.ST_COMMITTED, abi.ST_PREACCEPTED, abi.ST_ACCEPTED,
                         abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN, abi.ST_HISTORICAL], size=n,
                        p=[0.5, 0.1, 0.1, 0.05, 0.05, 0.1, 0.05, 0.05]).astype(np.uint8)
    b = workload.generate(n, keys_per_txn=3, keyspace=200, kinds=kinds, status=status, seed=12)
    check(engine_factory, b, window=8)


def test_ragged_keys(engine_factory):
    # 1..16 keys per txn
    rng = np.random.default_rng(4)
    base = workload.generate(3000, keys_per_txn=1, keyspace=500, seed=4)
    cnt = rng.integers(1, 17, size=3000)
    keys, off = [], [0]
    for c in cnt:
        keys.append(np.sort(rng.choice(500, size=c, replace=False)).astype(np.uint64))
        off.append(off[-1] + c)
    base["keys"] = np.concatenate(keys)
    base["key_off"] = np.array(off, np.uint32)
    check(engine_factory, base, window=16)


def test_edge_sizes(engine_factory):
    for n in (1, 2, 63, 64, 65, 4095, 4096, 4097):
        check(engine_factory, workload.generate(n, keyspace=50, seed=n))


def test_empty_batch(engine_factory):
    b = workload.generate(0)
    eng = engine_factory()
    eng.load(b)
    sizes = eng.preaccept_deps()
    assert all(s.keys == 0 for s in sizes)


def test_unsorted_batch_rejected(engine_factory):
    from accord_amd import engine

    b = workload.generate(100, seed=1)
    b["txn_lsb"] = b["txn_lsb"][::-1].copy()
    eng = engine_factory()
    eng.load(b)
    with pytest.raises(engine.AccordDepsError):
        eng.preaccept_deps()


@pytest.mark.parametrize("seed,width", [(21, 400), (22, 40), (23, 3000)])
def test_range_txns_mixed(engine_factory, seed, width):
    # RangeDeps interval join + range-domain queries over CFK keys (virtual items)
    b = workload.generate(3000, 3, 20000, "uniform", range_frac=0.15, range_width_max=width, seed=seed)
    check(engine_factory, b, window=16)


def wide_range_batch(keyspace):
    """keyspace single-key Writes over keyspace keys, then 3 range Reads over the whole key space: each range
    txn's KeyDeps hold about one TxnId per key (more than one LDS union pass holds)."""
    b = workload.generate(keyspace, 1, keyspace, "uniform", seed=keyspace)
    n = b["n"]
    is_range = np.zeros(n, bool)
    is_range[-3:] = True
    kind = np.where(is_range, abi.KIND_READ, abi.KIND_WRITE).astype(np.uint64)
    flags = (kind << np.uint64(1)) | is_range.astype(np.uint64)
    b["txn_lsb"] = (b["txn_lsb"].astype(np.uint64) & ~np.uint64(0xF)) | flags
    b["exec_lsb"] = (b["exec_lsb"].astype(np.uint64) & ~np.uint64(0xF)) | flags
    ko = b["key_off"].astype(np.int64)
    b["keys"] = np.ascontiguousarray(b["keys"][np.repeat(~is_range, np.diff(ko))])
    b["key_off"] = np.concatenate([[0], np.cumsum(np.where(is_range, 0, np.diff(ko)))]).astype(np.uint32)
    ro = np.concatenate([[0], np.cumsum(is_range.astype(np.int64))]).astype(np.uint32)
    b["range_off"] = ro
    b["range_start"] = np.zeros(int(ro[-1]), np.uint64)
    b["range_end"] = np.full(int(ro[-1]), keyspace + 1, np.uint64)
    return b


@pytest.mark.parametrize("keyspace", [24000, 70000])
def test_union_overflow_wide_ranges(engine_factory, keyspace):
    # 24k keys: the 1024-thread 128 KiB LDS overflow pass; 70k keys: its global-memory sort
    check(engine_factory, wide_range_batch(keyspace), window=4, levels=False)


def test_range_txns_writes_and_sync_points(engine_factory):
    rng = np.random.default_rng(31)
    n = 2500
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT], size=n,
                       p=[0.4, 0.4, 0.1, 0.1])
    status = rng.choice([abi.ST_APPLIED, abi.ST_INVALID, abi.ST_COMMITTED], size=n, p=[0.8, 0.1, 0.1]).astype(np.uint8)
    b = workload.generate(n, 2, 3000, "uniform", range_frac=0.3, range_width_max=200, kinds=kinds, status=status, seed=31)
    check(engine_factory, b, window=8, replicas=4, drop_p=0.25)


def test_many_keys_large_path(engine_factory):
    # key txns with more than KMAX (16) keys take the virtual-item path
    rng = np.random.default_rng(8)
    base = workload.generate(1500, keys_per_txn=1, keyspace=400, seed=8)
    cnt = rng.integers(1, 41, size=1500)
    keys, off = [], [0]
    for c in cnt:
        keys.append(np.sort(rng.choice(400, size=c, replace=False)).astype(np.uint64))
        off.append(off[-1] + c)
    base["keys"] = np.concatenate(keys)
    base["key_off"] = np.array(off, np.uint32)
    check(engine_factory, base, window=12)


def test_unsorted_keys_rejected(engine_factory):
    from accord_amd import engine

    b = workload.generate(50, keys_per_txn=3, seed=2)
    b["keys"] = b["keys"].copy()
    b["keys"][0], b["keys"][1] = b["keys"][1], b["keys"][0]
    eng = engine_factory()
    eng.load(b)
    with pytest.raises(engine.IllegalArgumentException):
        eng.preaccept_deps()


def test_levels_sync_points_and_ephemeral_reads(engine_factory):
    # key-domain SyncPoint / ExclusiveSyncPoint / EphemeralRead are unmanaged: per-key bounds over their deps
    # (+ the byId range between them for sync points), and awaitsOnlyDeps kinds wait for every dependency
    rng = np.random.default_rng(41)
    for n, keyspace, slow in ((3000, 40, 0.3), (20000, 2000, 0.1)):
        kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT,
                            abi.KIND_EXCLUSIVE_SYNC_POINT], size=n, p=[0.3, 0.3, 0.14, 0.13, 0.13])
        b = workload.generate(n, 3, keyspace, kinds=kinds, slow_frac=slow, bump_max=60, seed=n)
        check(engine_factory, b, window=16)
        check(engine_factory, b, window=16, fixpoint=True)      # the relaxation path (b)/(c) edges too


def test_levels_reject_local_only(engine_factory):
    from accord_amd import engine

    kinds = np.array([abi.KIND_WRITE, abi.KIND_LOCAL_ONLY, abi.KIND_READ] * 10)
    b = workload.generate(30, 2, 50, kinds=kinds, seed=3)
    eng = engine_factory()
    eng.load(b)
    eng.preaccept_deps()
    eng.merge()
    with pytest.raises(engine.AccordDepsError):
        eng.exec_levels()


def test_c4_scaled(engine_factory):
    # BASELINE configs[3] shape (10% range txns, widths U[1, 2^13]) scaled to 40k txns over a 400k keyspace
    b = workload.generate(40000, 4, 400_000, "uniform", range_frac=0.1, range_width_max=1 << 13,
                          seed=workload.SEEDS["C4"])
    check(engine_factory, b)


@pytest.mark.parametrize("n,keyspace,rf,width,slow,bump", [(40000, 400_000, 0.1, 1 << 13, 0.1, 16),
                                                            (30000, 20000, 0.2, 300, 0.3, 16),
                                                            (30000, 20000, 0.2, 300, 0.3, 200),
                                                            (20000, 3000, 0.05, 50, 0.5, 2000)])
def test_mixed_pull_levels(engine_factory, n, keyspace, rf, width, slow, bump):
    # mixed key + range batches take the executeAt-ordered pull (k_level_pull_mixed, level_path 11) unless a
    # slow-path bump moves an executeAt beyond the rank window (then 14 -> Kahn); either way the oracle's levels
    # and order, and the Kahn wavefronts (AD_LEVELS_KAHN) on the same batch agree
    kinds = np.where(np.random.default_rng(n).random(n) < 0.5, abi.KIND_WRITE, abi.KIND_READ)
    b = workload.generate(n, 4, keyspace, "uniform", range_frac=rf, range_width_max=width, slow_frac=slow,
                          bump_max=bump, kinds=kinds, seed=n + keyspace)
    eng = engine_factory()
    check(engine_factory, b, eng=eng)
    path = eng.last_times()["level_path"]
    assert path in (11, 14), path
    if bump <= 16:                                            # within k_window_rank's +-64 rows
        assert path == 11
    lv, order, _ = eng.exec_levels()
    lv, order = lv.copy(), order.copy()
    eng.set_level_mode(3)                                     # AD_LEVELS_KAHN
    lk, ok, _ = eng.exec_levels()
    assert np.array_equal(lv, lk) and np.array_equal(order, ok)
    assert lv.max() > 10


def test_mixed_pull_forced_abort(engine_factory):
    # AD_LEVELS_PULL_ABORT: the mixed pull aborts at once (level_path 15) and the Kahn wavefronts recompute the
    # batch from scratch (pred-mode runs, flags and levels reset): still the oracle's levels and order
    b = workload.generate(20000, 4, 200_000, "uniform", range_frac=0.1, range_width_max=1 << 12, seed=91)
    eng = engine_factory()
    eng.set_level_mode(4)                                     # AD_LEVELS_PULL_ABORT
    check(engine_factory, b, eng=eng)
    assert eng.last_times()["level_path"] == 15


def test_mixed_pull_skips_awaits_only_deps(engine_factory):
    # an ExclusiveSyncPoint / EphemeralRead may depend on a larger executeAt: the mixed pull is skipped (13)
    rng = np.random.default_rng(77)
    n = 6000
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ], size=n, p=[0.45, 0.45, 0.1])
    b = workload.generate(n, 3, 5000, "uniform", range_frac=0.1, range_width_max=100, kinds=kinds, seed=77)
    eng = engine_factory(window=16)
    check(engine_factory, b, eng=eng, window=16)
    assert eng.last_times()["level_path"] in (0, 13)


def test_merge_host_equals_oracle_merge(engine_factory):
    # Deps.merge of replies supplied by the host (the coordinator's network replies): feed the oracle's
    # per-view replies in, compare with the oracle's LinearMerger result
    for b, cfg in ((workload.config("C3", n=8000, seed=41), (16, 4, 0.3, 41)),
                   (workload.generate(3000, 3, 20000, "uniform", range_frac=0.15, range_width_max=400, seed=42), (16, 3, 0.2, 42))):
        w, r, p, s = cfg
        ref = O.OracleResult(b, abi.make_config(w, r, p, s), O.FLAG_MERGE)
        eng = engine_factory(window=w, replicas=r, drop_p=p, seed=s)
        eng.load(b)
        replies = [[ref.deps(v, c) for c in range(abi.NUM_CLASSES)] for v in range(r)]
        eng.merge_host(replies)
        for c in range(abi.NUM_CLASSES):
            _assert_csr("merge_host %s" % abi.CLASS_NAMES[c], eng.fetch_merged(c), ref.merged(c))
        # merge of one reply is that reply; of two in reverse order, the per-txn union (testMergedProperty)
        eng.merge_host([replies[r - 1]])
        for c in range(abi.NUM_CLASSES):
            _assert_csr("merge_host single %s" % abi.CLASS_NAMES[c], eng.fetch_merged(c), replies[r - 1][c])
        eng.merge_host([replies[2], replies[0]])
        from batchkit import deps_of
        for c in range(abi.NUM_CLASSES):
            got = eng.fetch_merged(c)
            for i in range(0, b["n"], 97):
                want = {}
                for rep in (replies[0], replies[2]):
                    for k, ts in deps_of(rep[c], i).items():
                        want.setdefault(k, set()).update(ts)
                assert deps_of(got, i) == {k: sorted(v) for k, v in want.items()}


def test_merge_host_rejects_malformed(engine_factory):
    from accord_amd import engine

    b = workload.config("C2", n=2000)
    ref = O.OracleResult(b, abi.make_config(32, 1, 0.0, 1), O.FLAG_MERGE)
    eng = engine_factory(replicas=1)
    eng.load(b)
    rep = [ref.deps(0, c) for c in range(abi.NUM_CLASSES)]
    bad = abi.Csr(rep[0].key_off.copy(), rep[0].keys.copy(), rep[0].k2t_off.copy(), rep[0].k2t.copy(),
                  rep[0].txn_off.copy(), rep[0].txns.copy())
    i = int(np.nonzero(np.diff(bad.txn_off) > 0)[0][0])
    bad.k2t[bad.k2t_off[i] + (bad.key_off[i + 1] - bad.key_off[i])] = 10 ** 6      # index out of range
    with pytest.raises(engine.IllegalArgumentException):
        eng.merge_host([[bad, rep[1], rep[2]]])


@pytest.mark.parametrize("hot", [False, True])
def test_wide_64bit_keys(engine_factory, hot):
    # Murmur3-style 64-bit key tokens (the full u64 range): sorted in two 32-bit LSD halves, key segments by full
    # 64-bit equality; deps, merge and levels equal the oracle
    b = workload.generate(20000, keys_per_txn=4, keyspace=300 if hot else 10_000_000, seed=31 + hot)
    rng = np.random.default_rng(7)
    uniq = np.unique(b["keys"])
    tok = np.unique(rng.integers(0, np.iinfo(np.uint64).max, size=2 * len(uniq), dtype=np.uint64, endpoint=True))
    tok = np.sort(rng.choice(tok, size=len(uniq), replace=False))
    b["keys"] = tok[np.searchsorted(uniq, b["keys"])]      # order-preserving remap onto 64-bit tokens
    check(engine_factory, b)


def test_wide_64bit_ranges(engine_factory):
    # range endpoints spread over ~2^62: each endpoint sorted in two 32-bit halves; keys scaled the same way
    b = workload.generate(4000, 4, 20000, "uniform", range_frac=0.1, range_width_max=400, seed=33)
    scale = np.uint64(1 << 44)
    b["keys"] = b["keys"] * scale + np.uint64(12345)
    b["range_start"] = b["range_start"] * scale + np.uint64(12345)
    b["range_end"] = b["range_end"] * scale + np.uint64(12345)
    check(engine_factory, b, window=8)
