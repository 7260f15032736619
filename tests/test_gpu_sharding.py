"""Key-range sharding (SURVEY §8e / BASELINE C5) on one GPU: S stores (handles) in one process run the full
protocol (deps on sliced local batches, export, exchange, home merge, levels, order) and must reproduce the
unsharded engine bit for bit: KeyDeps are shard-invariant, and window/drop decisions use global arrival ranks.
Levels: levels="gather" (the default: every store's constraint edges gathered once and solved,
ad_shard_level_edges / ad_shard_levels_solve / ad_shard_levels_gather) and levels="rounds" (the per-round
delta / dense exchange, rounds = graph depth)."""
import os

import numpy as np
import pytest

from accord_amd import abi, blob, sharding, workload

pytestmark = pytest.mark.gpu


def unsharded(engine_factory, b, w, r, p, s):
    eng = engine_factory(window=w, replicas=r, drop_p=p, seed=s)
    eng.load(b)
    eng.preaccept_deps()
    views = [[eng.fetch_deps(v, c) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)] for v in range(r)]
    eng.merge()
    merged = [eng.fetch_merged(c) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)]
    lv, order, _ = eng.exec_levels()
    return views, merged, lv, order


def same_txn(got, h, want, g):
    a, b = got.txn(h), want.txn(g)
    return all(np.array_equal(x, y) for x, y in zip(a, b))


@pytest.mark.parametrize("name,shards,levels,delta,slot", [("C2", 2, "gather", False, None), ("C2", 4, "gather", True, None),
                                                            ("C3", 3, "gather", False, None), ("C2", 2, "rounds", True, None),
                                                            ("C3", 3, "rounds", True, None), ("C3", 3, "rounds", False, None),
                                                            ("C2", 4, "rounds", False, None), ("C2", 2, "kahn", True, None),
                                                            ("C3", 3, "kahn", True, None), ("C2", 4, "kahn", True, None),
                                                            ("C2", 4, "kahn", True, 97), ("C3", 3, "kahn", True, 13)])
def test_sharded_equals_unsharded(engine_factory, name, shards, levels, delta, slot):
    # levels="rounds" + delta: level rounds exchange only raised levels of shared txns (ad_shard_set_holders);
    # rounds without delta: the dense all-reduce of the whole level array; "gather": one edge exchange; kahn with a
    # slot: at most that many READYs per (source, destination) and wave, the rest in later waves (ad_shard_kahn_run's
    # fixed slots): the levels ride in the READYs, so late ones change the wave count, never a level
    w, r, p, s = 32, 3, 0.1, 0xACC0D1
    b = workload.config(name, n=30000)
    views, merged, lv, order = unsharded(engine_factory, b, w, r, p, s)
    bounds = sharding.even_bounds(0, 10_000_000, shards)
    hs = sharding.home_stores(b, bounds)
    masks = sharding.holder_masks(b, bounds)
    stores = []
    try:
        for k in range(shards):
            local, gid, home = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            assert np.array_equal(home, (hs[gid] == k).astype(np.uint8))
            st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
            stores.append(st)
            st.load(local, gid, hs[gid], b["n"], k, shards, holders=masks[gid] if delta else None)
        rounds = sharding.LocalTransport.run(stores, levels=levels, kahn_slot=slot)
        assert rounds >= 1 and (levels != "gather" or rounds == 1)
        if levels == "kahn":
            assert all(st.depth == lv.max() + 1 for st in stores)
            assert rounds == int(lv.max()) + 2 if slot is None else rounds > int(lv.max()) + 2
        seen = np.zeros(b["n"], bool)
        pos = {int(t): i for i, t in enumerate(order)}
        for st in stores:
            for v in range(r + 1):
                for ci, c in enumerate((abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)):
                    got, hg = st.fetch(v, c)
                    want = merged[ci] if v == r else views[v][ci]
                    for hh, g in enumerate(hg):
                        assert same_txn(got, hh, want, int(g)), "store view %d class %d txn %d differs" % (v, c, g)
            hl, ho = st.order()
            _, hg = st.fetch(r, abi.CLASS_KEY)
            assert np.array_equal(hl, lv[hg]), "levels differ"
            # the store's order is the global order restricted to its home txns
            assert [pos[int(t)] for t in ho] == sorted(pos[int(t)] for t in ho)
            assert not seen[hg].any()
            seen[hg] = True
        assert seen[np.diff(b["key_off"]) > 0].all(), "every txn has exactly one home store"
    finally:
        for st in stores:
            st.close()


@pytest.mark.parametrize("name,shards", [("C2", 2), ("C3", 3), ("C3", 4)])
def test_sharded_witnessed_at(engine_factory, name, shards):
    # per-store witnessedAt proposals (ad_max_conflicts on each store's sliced batch, global ranks) folded by
    # PreAccept.reduce's mergeMax equal the unsharded store's: MaxConflicts is a max over the txn's keys
    w, r, p, s = 32, 3, 0.1, 0xACC0D1
    b = workload.config(name, n=30000)
    eng = engine_factory(window=w, replicas=r, drop_p=p, seed=s)
    eng.load(b)
    eng.preaccept_deps()
    want_rank, want_fast = eng.max_conflicts()
    bounds = sharding.even_bounds(0, 10_000_000, shards)
    hs = sharding.home_stores(b, bounds)
    stores, parts = [], []
    try:
        for k in range(shards):
            local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
            stores.append(st)
            st.load(local, gid, hs[gid], b["n"], k, shards)
            st.preaccept()
            rank, fast = st.max_conflicts()
            parts.append((gid, rank.copy(), fast.copy()))
        got_rank, got_fast, _ = sharding.reduce_witnessed(b, parts)
        assert np.array_equal(got_rank, want_rank) and np.array_equal(got_fast, want_fast)
        if name == "C3":
            assert want_fast.min() == 0
    finally:
        for st in stores:
            st.close()


@pytest.mark.parametrize("shards,window,drop", [(2, 32, 0.1), (3, 8, 0.3), (4, 0, 0.0)])
def test_sharded_witnessed_at_range_txns(engine_factory, shards, window, drop):
    # range footprints too (MaxConflicts as a ReducingRangeMap, k_mc_range_keys / k_mc_range_entries): each store
    # answers for its slices with global-rank windows and drops, the fold equals the unsharded store's answer
    r, s = 3, 0xC0DE
    b = workload.generate(20000, 4, 200_000, "uniform", range_frac=0.1, range_width_max=1 << 14, seed=60 + shards)
    eng = engine_factory(window=window, replicas=r, drop_p=drop, seed=s)
    eng.load(b)
    eng.preaccept_deps()
    want_rank, want_fast = eng.max_conflicts()
    bounds = sharding.even_bounds(0, 200_000, shards)
    hs = sharding.home_stores(b, bounds)
    stores, parts = [], []
    try:
        for k in range(shards):
            local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            st = sharding.ShardStore(0, window=window, replicas=r, drop_p=drop, seed=s)
            stores.append(st)
            st.load(local, gid, hs[gid], b["n"], k, shards)
            st.preaccept()
            rank, fast = st.max_conflicts()
            parts.append((gid, rank.copy(), fast.copy()))
        got_rank, got_fast, _ = sharding.reduce_witnessed(b, parts)
        assert np.array_equal(got_rank, want_rank) and np.array_equal(got_fast, want_fast)
        assert want_fast.min() == 0
    finally:
        for st in stores:
            st.close()


def _make_stores(b, shards, w, r, p, s, keyspace, delta=True):
    bounds = sharding.even_bounds(0, keyspace, shards)
    hs = sharding.home_stores(b, bounds)
    masks = sharding.holder_masks(b, bounds)
    stores = []
    for k in range(shards):
        local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
        st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
        stores.append(st)
        st.load(local, gid, hs[gid], b["n"], k, shards, holders=masks[gid] if delta else None)
    return stores, bounds, hs


def _check_against_unsharded(stores, views, merged, lv, order, r, n_global):
    """Every store's home txns (vectorised row selection): per-view and merged deps, levels, and its order
    equal to the global order restricted to its home txns."""
    pos = np.empty(len(order), np.int64)
    pos[order] = np.arange(len(order))
    seen = np.zeros(n_global, bool)
    for st in stores:
        for v in range(r + 1):
            for ci, c in enumerate((abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)):
                got, hg = st.fetch(v, c)
                want = merged[ci] if v == r else views[v][ci]
                assert blob._rows_of(want, hg).equal(got), "store view %d class %d differs" % (v, c)
        hl, ho = st.order()
        _, hg = st.fetch(r, abi.CLASS_KEY)
        assert np.array_equal(hl, lv[hg]), "levels differ"
        assert np.all(np.diff(pos[ho]) > 0), "store order is not the global order restricted to its home txns"
        assert not seen[hg].any()
        seen[hg] = True
    return seen


def test_blob_codec_matches_engine_bytes(engine_factory):
    # accord_amd.blob.export over a store's own local CSRs (local ranks) must reproduce the bytes ad_shard_export
    # wrote for every destination (the codec the CPU gloo test pushes is the engine's format)
    w, r, p, s = 32, 3, 0.1, 0xACC0D1
    b = workload.config("C2", n=20000)
    stores, bounds, hs = _make_stores(b, 3, w, r, p, s, 10_000_000)
    try:
        for k, st in enumerate(stores):
            st.eng.preaccept_deps()
            csrs = [st.eng.fetch_deps(v, c) for v in range(r) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)]
            sizes = st.export()
            dev = st.send_buffer()
            host, hsz = blob.export(st.gid, st.home_store, csrs, 3)
            assert np.array_equal(sizes, hsz)
            assert np.array_equal(dev, host), "store %d: blob bytes differ from the host codec" % k
    finally:
        for st in stores:
            st.close()


def test_host_fragments_import(engine_factory):
    # fragments resolved elsewhere and packed by the host codec: ad_shard_import_host + ad_shard_merge on every
    # store must equal the unsharded engine (the engine merges what the wire format carries, whoever produced it)
    w, r, p, s = 32, 2, 0.1, 0xACC0D1
    b = workload.config("C2", n=20000)
    views, merged, lv, order = unsharded(engine_factory, b, w, r, p, s)
    shards = 3
    stores, bounds, hs = _make_stores(b, shards, w, r, p, s, 10_000_000)
    try:
        bufs, sizes = [], []
        for st in stores:
            st.eng.preaccept_deps()
            csrs = [st.eng.fetch_deps(v, c) for v in range(r) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)]
            bb, sz = blob.export(st.gid, st.home_store, csrs, shards)
            bufs.append(bb)
            sizes.append(sz)
        offs = [np.concatenate([[0], np.cumsum(z)]).astype(np.int64) for z in sizes]
        for d, st in enumerate(stores):
            parts = [bufs[k][offs[k][d]:offs[k][d + 1]] for k in range(shards)]
            st.import_host(np.concatenate(parts), np.array([sizes[k][d] for k in range(shards)], np.uint64))
            st.merge()
            for v in range(r + 1):
                for ci, c in enumerate((abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)):
                    got, hg = st.fetch(v, c)
                    want = merged[ci] if v == r else views[v][ci]
                    assert blob._rows_of(want, hg).equal(got)
    finally:
        for st in stores:
            st.close()


@pytest.mark.parametrize("levels,delta,run_loop", [("gather", False, True), ("rounds", True, True), ("rounds", False, True),
                                                   ("kahn", True, True), ("kahn", True, False), ("auto", True, True)])
def test_rccl_world1_run_store(engine_factory, tmp_path, levels, delta, run_loop):
    # the RCCL transport end to end on the one GPU: a world = 1 communicator (ad_comm_init), the grouped
    # ncclSend/ncclRecv all-to-all (ad_shard_alltoall, to self) and the levels — gather: ncclAllGather of the
    # edge counts + the edge send/recv (ad_shard_levels_gather); rounds + delta: ncclAllGather of the pair counts
    # (ad_shard_levels_exchange); rounds, dense: ncclAllReduce of the level array (ad_shard_levels_allreduce) —
    # driven by the same run_store the N>1 bench uses; equal to the unsharded engine
    import torch.distributed as dist
    w, r, p, s = 32, 3, 0.1, workload.SEEDS["C5"]
    b = workload.generate(200_000, 4, 10_000_000, "uniform", seed=s)
    views, merged, lv, order = unsharded(engine_factory, b, w, r, p, s)
    dist.init_process_group("gloo", init_method="file://%s" % (tmp_path / "rdv"), rank=0, world_size=1)
    stores = []
    try:
        stores, _, _ = _make_stores(b, 1, w, r, p, s, 10_000_000, delta=delta)
        tr = sharding.RcclTransport(dist, stores[0], 0, 1)
        assert tr.name == "rccl"
        tr.kahn_run_loop = run_loop
        if run_loop and levels == "kahn":
            tr.kahn_slot = 1024             # < the busiest wave's READYs: some arrive waves late
        rounds = sharding.run_store(stores[0], tr, levels=levels)
        assert rounds >= 1 and (levels != "gather" or rounds == 1)
        if levels in ("kahn", "auto"):
            assert stores[0].depth == int(lv.max()) + 1
            if run_loop:                    # ad_shard_kahn_run: fixed slots, a pending check every 4 waves read 2 later
                assert rounds >= int(lv.max()) + 1 and (rounds % tr.kahn_check_every == 0 or rounds == 129)
            else:                           # ad_shard_kahn_exchange: counts all-gather, self copy, one wave per level
                assert rounds == int(lv.max()) + 2
        seen = _check_against_unsharded(stores, views, merged, lv, order, r, b["n"])
        assert seen[np.diff(b["key_off"]) > 0].all()
        # a second communicator on the same handle is refused (no leak of the first)
        import accord_amd.engine as E
        with pytest.raises(E.AccordDepsError):
            stores[0].comm_init(1, 0, sharding.unique_id())
    finally:
        for st in stores:
            st.close()
        dist.destroy_process_group()


def test_levels_round_cap_raises(engine_factory):
    # run_store / LocalTransport must not report levels that are still changing when the round cap is hit
    w, r, p, s = 32, 2, 0.1, 0xACC0D1
    b = workload.config("C3", n=20000)
    stores, _, _ = _make_stores(b, 3, w, r, p, s, 10_000_000)
    try:
        with pytest.raises(sharding.LevelsNotConverged):
            sharding.LocalTransport.run(stores, max_rounds=1, levels="rounds")
    finally:
        for st in stores:
            st.close()


def test_c5_four_stores_1m_each(engine_factory):
    # C5's generator at 1,048,576 txns per store over S = 4 key-range stores (4,194,304 txns, 40M keys): the full
    # cross-store protocol (local deps, export, exchange, home merge, one level-edge exchange, order) equals the
    # unsharded engine on the whole batch, bit for bit, for every home txn of every store
    w, r, p, s = 32, 3, 0.1, workload.SEEDS["C5"]
    shards, per = 4, 1 << 20
    b = workload.generate(shards * per, 4, 10_000_000 * shards, "uniform", seed=s)
    views, merged, lv, order = unsharded(engine_factory, b, w, r, p, s)
    stores, _, _ = _make_stores(b, shards, w, r, p, s, 10_000_000 * shards)
    try:
        rounds = sharding.LocalTransport.run(stores)
        assert rounds == 1
        seen = _check_against_unsharded(stores, views, merged, lv, order, r, b["n"])
        assert seen[np.diff(b["key_off"]) > 0].all(), "every txn has exactly one home store"
    finally:
        for st in stores:
            st.close()


def unsharded3(engine_factory, b, w, r, p, s):
    eng = engine_factory(window=w, replicas=r, drop_p=p, seed=s)
    eng.load(b)
    eng.preaccept_deps()
    views = [[eng.fetch_deps(v, c) for c in range(3)] for v in range(r)]
    eng.merge()
    merged = [eng.fetch_merged(c) for c in range(3)]
    lv, order, _ = eng.exec_levels()
    return views, merged, lv, order


@pytest.mark.parametrize("shards,levels,delta,special", [(2, "gather", True, False), (3, "gather", True, True),
                                                          (4, "gather", False, True), (4, "rounds", True, False),
                                                          (3, "rounds", False, False), (3, "kahn", True, True),
                                                          (4, "kahn", True, False)])
def test_sharded_range_txns_equal_presplit_unsharded(engine_factory, shards, levels, delta, special):
    # range txns sliced at the store bounds; the stores together must equal the unsharded engine on
    # the batch whose ranges are cut at the same bounds (sharding.presplit; the CPU test
    # test_sharding_ranges.py pins that claim with the oracle): every view and class incl. RangeDeps, the merged
    # Deps, levels (rules (b)/(c) applied per store from its own views' Deps.merge) and the order.  special:
    # key-domain sync points / ephemeral reads too, and range sync points / exclusive sync points (their levels
    # run ~10^3 deep: one edge exchange, not one round per level).
    w, r, p, s = 32, 3, 0.1, 0xACC0D1
    n, ks = 12000, 160_000
    kinds = None
    if special:
        kinds = np.random.default_rng(shards).choice(
            [abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT, abi.KIND_EPHEMERAL_READ],
            size=n, p=[0.4, 0.4, 0.07, 0.07, 0.06])
    b = workload.generate(n, 4, ks, "uniform", range_frac=0.1, range_width_max=1 << 13, kinds=kinds, seed=40 + shards)
    bounds = sharding.even_bounds(0, ks, shards)
    views, merged, lv, order = unsharded3(engine_factory, sharding.presplit(b, bounds), w, r, p, s)
    hs = sharding.home_stores(b, bounds)
    masks = sharding.holder_masks(b, bounds)
    stores = []
    try:
        for k in range(shards):
            local, gid, home = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
            stores.append(st)
            st.load(local, gid, hs[gid], b["n"], k, shards, holders=masks[gid] if delta else None)
        assert sharding.LocalTransport.run(stores, levels=levels) >= 1
        seen = np.zeros(b["n"], bool)
        pos = {int(t): i for i, t in enumerate(order)}
        ranged = 0
        for st in stores:
            for v in range(r + 1):
                for c in range(3):
                    got, hg = st.fetch(v, c)
                    want = merged[c] if v == r else views[v][c]
                    for hh, g in enumerate(hg):
                        assert same_txn(got, hh, want, int(g)), "store view %d class %d txn %d differs" % (v, c, g)
                    if c == abi.CLASS_RANGE:
                        ranged += int(got.txn_off[-1])
            hl, ho = st.order()
            _, hg = st.fetch(r, abi.CLASS_KEY)
            assert np.array_equal(hl, lv[hg]), "levels differ"
            assert [pos[int(t)] for t in ho] == sorted(pos[int(t)] for t in ho)
            assert not seen[hg].any()
            seen[hg] = True
        assert ranged > 300
        touched = (np.diff(b["key_off"]) > 0) | (np.diff(b["range_off"]) > 0)
        assert seen[touched].all(), "every txn has exactly one home store"
    finally:
        for st in stores:
            st.close()


def test_sharded_range_blob_bytes_equal_host_codec(engine_factory):
    # the engine's export with RangeDeps classes (header nvc | nr << 16, 16-byte range keys) byte-equal to
    # accord_amd.blob.export over the store's own fetched CSRs
    w, r, p, s = 16, 2, 0.1, 7
    b = workload.generate(4000, 3, 50_000, "uniform", range_frac=0.2, range_width_max=20000, seed=77)
    bounds = sharding.even_bounds(0, 50_000, 2)
    hs = sharding.home_stores(b, bounds)
    local, gid, _ = sharding.slice_for_shard(b, bounds[1], bounds[2])
    st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
    try:
        st.load(local, gid, hs[gid], b["n"], 1, 2)
        st.eng.preaccept_deps()                        # the store's deps stage, sizes kept for fetch_deps
        sizes = st.export()
        buf = st.send_buffer()
        csrs = [st.eng.fetch_deps(v, c) for v in range(r) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)]
        csrs += [st.eng.fetch_deps(v, abi.CLASS_RANGE) for v in range(r)]
        hbuf, hsizes = blob.export(gid, hs[gid], csrs, 2)
        assert np.array_equal(sizes, hsizes) and np.array_equal(buf, hbuf)
    finally:
        st.close()


def _range_batch_check(stores, views, merged, lv, order, r, b):
    """Every store's home txns against the unsharded (presplit) engine, all three classes, vectorised."""
    pos = np.empty(len(order), np.int64)
    pos[order] = np.arange(len(order))
    seen = np.zeros(b["n"], bool)
    for st in stores:
        for v in range(r + 1):
            for c in range(3):
                got, hg = st.fetch(v, c)
                want = merged[c] if v == r else views[v][c]
                assert blob._rows_of(want, hg).equal(got), "store view %d class %d differs" % (v, c)
        hl, ho = st.order()
        _, hg = st.fetch(r, abi.CLASS_KEY)
        assert np.array_equal(hl, lv[hg]), "levels differ"
        assert np.all(np.diff(pos[ho]) > 0)
        assert not seen[hg].any()
        seen[hg] = True
    touched = (np.diff(b["key_off"]) > 0) | (np.diff(b["range_off"]) > 0)
    assert seen[touched].all(), "every txn has exactly one home store"


def test_sharded_deep_range_sync_points(engine_factory):
    # the configuration that did not converge under the per-round exchange (round 2: still raising levels after
    # 68 rounds at 0.5 s each): 30k txns, 3 stores, 10 % range txns of every kind incl. range sync points and
    # exclusive sync points up to 2^15 wide over 4*10^5 keys, key-domain sync points / ephemeral reads.  One edge
    # exchange; levels ~10^3 deep; every class, merged Deps, levels and order equal the presplit unsharded engine.
    shards = 3
    w, r, p, s = 32, 3, 0.1, 0xACC0D1
    n, ks = 30000, 400_000
    kinds = np.random.default_rng(shards).choice(
        [abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT, abi.KIND_EPHEMERAL_READ],
        size=n, p=[0.4, 0.4, 0.07, 0.07, 0.06])
    b = workload.generate(n, 4, ks, "uniform", range_frac=0.1, range_width_max=1 << 15, kinds=kinds, seed=40 + shards)
    bounds = sharding.even_bounds(0, ks, shards)
    views, merged, lv, order = unsharded3(engine_factory, sharding.presplit(b, bounds), w, r, p, s)
    assert lv.max() > 500, "the configuration is meant to be deep"
    hs = sharding.home_stores(b, bounds)
    stores = []
    try:
        for k in range(shards):
            local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
            stores.append(st)
            st.load(local, gid, hs[gid], b["n"], k, shards)
        assert sharding.LocalTransport.run(stores) == 1
        assert all(st.depth == lv.max() + 1 for st in stores)
        _range_batch_check(stores, views, merged, lv, order, r, b)
    finally:
        for st in stores:
            st.close()


def test_sharded_c3_full_size_8_stores(engine_factory):
    # BASELINE C3 at its full 1,048,576 txns (Zipf 0.99: the hot keys chain ~1.6*10^5 levels) over 8 key-range
    # stores: one edge exchange, levels and order equal the unsharded engine's (deep narrow frontiers solved
    # inside one workgroup), and every view / merged Deps of every home txn
    w, r, p, s = 32, 3, 0.1, workload.SEEDS["C3"]
    b = workload.config("C3")
    views, merged, lv, order = unsharded(engine_factory, b, w, r, p, s)
    stores, _, _ = _make_stores(b, 8, w, r, p, s, 10_000_000, delta=False)
    try:
        assert sharding.LocalTransport.run(stores) == 1
        assert all(st.depth == lv.max() + 1 for st in stores)
        seen = _check_against_unsharded(stores, views, merged, lv, order, r, b["n"])
        assert seen[np.diff(b["key_off"]) > 0].all()
    finally:
        for st in stores:
            st.close()


def test_c5_full_shape_8_stores(engine_factory):
    # BASELINE C5 at its shape, in one process: 16,777,216 txns (4 uniform keys over 10^7) over 8 key-range stores
    # through LocalTransport (export, exchange, home merge, the levels by the default "auto" protocol -- Kahn waves,
    # each store walking only its own constraint edges -- and order), against the unsharded engine on the same batch:
    # every view and the merged Deps of every home txn of every store, levels and order.  Records the level-exchange
    # bytes each store sends (8 B per READY / RELEASE message to another store): the one-exchange gather shipped
    # every store's constraint edges to every GPU (62.1 M edges, 497 MB received per store in round 3).
    import time
    w, r, p, s = 32, 3, 0.1, workload.SEEDS["C5"]
    t0 = time.perf_counter()
    b = workload.config("C5")
    views, merged, lv, order = unsharded(engine_factory, b, w, r, p, s)
    t1 = time.perf_counter()
    stores, _, _ = _make_stores(b, 8, w, r, p, s, 10_000_000, delta=True)
    try:
        timings = {}
        rounds = sharding.LocalTransport.run(stores, levels="auto", timings=timings)
        assert rounds <= sharding.AUTO_ROUND_CAP, "C5 is shallow: the Kahn waves finish"
        level_bytes = [int(st.kahn_bytes) for st in stores]
        # per txn one READY from each holder to each other holder over the batch (one exchange per wave): ~129 MB per
        # store (E[h(h-1)] = 8.07 messages per txn at 8 stores; round 4's READY-to-coordinator + RELEASE sent ~77 MB in
        # twice the exchanges), vs the gather's 497 MB of edges on every store and the delta rounds' ~534 MB per store
        assert max(level_bytes) < 160 << 20, level_bytes
        t2 = time.perf_counter()
        for st in stores:
            st.order()
        timings["order"] = time.perf_counter() - t2
        t2 = time.perf_counter()
        seen = _check_against_unsharded(stores, views, merged, lv, order, r, b["n"])     # levels included
        assert seen[np.diff(b["key_off"]) > 0].all(), "every txn has exactly one home store"
        rec = {"txns": int(b["n"]), "stores": 8, "unsharded_s": t1 - t0, "protocol_s": t2 - t1,
               "check_s": time.perf_counter() - t2, "phases_s_summed_over_stores": timings,
               "local_txns_per_store": [int(st.gid.size) for st in stores], "depth": int(lv.max() + 1),
               "level_protocol": "Kahn waves", "level_waves": rounds, "level_bytes_sent_per_store": level_bytes}
        print("C5 16M x 8 stores:", rec)
        out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
        if os.path.isdir(out):
            import json
            with open(os.path.join(out, "c5_8_stores.json"), "w") as f:
                json.dump(rec, f)
    finally:
        for st in stores:
            st.close()


@pytest.mark.parametrize("deps,shards,range_frac", [("accept", 2, 0.0), ("accept", 3, 0.1), ("ephemeral", 3, 0.1),
                                                    ("accept", 4, 0.05)])
def test_sharded_accept_equals_presplit_unsharded(engine_factory, deps, shards, range_frac):
    # Accept / GetDeps (bound executeAt, answered at the bound's GLOBAL arrival position: ad_shard_query_positions)
    # and GetEphemeralReadDeps (bound Timestamp.MAX) on every store, then the home merge: each home txn's per-view
    # and merged Deps equal the unsharded engine's on the presplit batch (Accept.java:113-116 per store through
    # CommandStores.mapReduce, CommandStores.java:576-593)
    w, r, p, s = 32, 3, 0.1, 0xACC0D1
    ks = 400_000
    b = workload.generate(20000, 4, ks, "uniform", range_frac=range_frac, range_width_max=1 << 12, slow_frac=0.3,
                          bump_max=200, seed=60 + shards)
    bounds = sharding.even_bounds(0, ks, shards)
    eng = engine_factory(window=w, replicas=r, drop_p=p, seed=s)
    eng.load(sharding.presplit(b, bounds))
    if deps == "ephemeral":
        eng.ephemeral_read_deps()
    else:
        eng.accept_deps()
    classes = range(3) if range_frac else (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)
    views = [{c: eng.fetch_deps(v, c) for c in classes} for v in range(r)]
    eng.merge()
    merged = {c: eng.fetch_merged(c) for c in classes}
    hs = sharding.home_stores(b, bounds)
    gq = sharding.query_positions(b)
    stores = []
    try:
        for k in range(shards):
            local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
            stores.append(st)
            st.load(local, gid, hs[gid], b["n"], k, shards)
        assert sharding.LocalTransport.run(stores, levels=None, deps=deps, gq=gq) == 0
        seen = np.zeros(b["n"], bool)
        for st in stores:
            for v in range(r + 1):
                for c in classes:
                    got, hg = st.fetch(v, c)
                    want = merged[c] if v == r else views[v][c]
                    assert blob._rows_of(want, hg).equal(got), "store view %d class %d differs" % (v, c)
            _, hg = st.fetch(r, abi.CLASS_KEY)
            assert not seen[hg].any()
            seen[hg] = True
    finally:
        for st in stores:
            st.close()


def test_sharded_store_recovery(engine_factory):
    # BeginRecovery's store queries on sharded stores (BeginRecovery.java:118 through CommandStores.mapReduce): every
    # store answers from its own slice and its own replicas' merged Deps (the store's PartialDeps) — the oracle on
    # that slice with those Deps, for the store's recovering rows
    import oracle as O
    from test_gpu_recovery import _same
    from test_oracle_recovery import _mixed
    shards, w, r, p, s = 3, 16, 2, 0.2, 9
    b = _mixed(3000, 300, 0.1, 21)
    bounds = sharding.even_bounds(0, 300, shards)
    hs = sharding.home_stores(b, bounds)
    gq = sharding.query_positions(b)
    total = 0
    for k in range(shards):
        local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
        st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
        try:
            st.load(local, gid, hs[gid], b["n"], k, shards)
            st.accept(gq[gid])
            st.eng.merge()
            merged = [st.eng.fetch_merged(c) for c in range(3)]
            rows = [i for i in range(local["n"]) if local["status"][i] < abi.ST_COMMITTED][:400]
            rows += [i for i in range(local["n"]) if local["status"][i] >= abi.ST_COMMITTED][:20]
            got = st.eng.recover(rows)
            _same(got, O.recover(local, merged, rows), rows)
            total += sum(len(got[0][x][c][2]) for x in range(2) for c in range(3))
        finally:
            st.close()
    assert total > 0
