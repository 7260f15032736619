"""Key-range sharding (SURVEY §8e / BASELINE C5) on one GPU: S stores (handles) in one process run the full
protocol (deps on sliced local batches, export, exchange, home merge, distributed level rounds, order) and must
reproduce the unsharded engine bit for bit: KeyDeps are shard-invariant, and window/drop decisions use global
arrival ranks."""
import numpy as np
import pytest

from accord_amd import abi, sharding, workload

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


@pytest.mark.parametrize("name,shards", [("C2", 2), ("C2", 4), ("C3", 3)])
def test_sharded_equals_unsharded(engine_factory, name, shards):
    w, r, p, s = 32, 3, 0.1, 0xACC0D1
    b = workload.config(name, n=30000)
    views, merged, lv, order = unsharded(engine_factory, b, w, r, p, s)
    bounds = sharding.even_bounds(0, 10_000_000, shards)
    hs = sharding.home_stores(b, bounds)
    stores = []
    try:
        for k in range(shards):
            local, gid, home = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
            assert np.array_equal(home, (hs[gid] == k).astype(np.uint8))
            st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=s)
            stores.append(st)
            st.load(local, gid, hs[gid], b["n"], k, shards)
        rounds = sharding.LocalTransport.run(stores)
        assert rounds >= 1
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
        got_rank, got_fast = sharding.reduce_witnessed(b, parts)
        assert np.array_equal(got_rank, want_rank) and np.array_equal(got_fast, want_fast)
        if name == "C3":
            assert want_fast.min() == 0
    finally:
        for st in stores:
            st.close()
