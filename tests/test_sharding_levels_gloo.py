"""The distributed levels on CPU: two processes over gloo (world_size 2, 127.0.0.1).

One-exchange levels (the default, sharding.run_store(levels="gather")): each rank exports the constraint edges
of its own key chains over global ranks (host model of ad_shard_level_edges: the Read/Write transitive
reduction per key in executeAt order), GlooTransport.gather_levels all-gathers the variable-size edge lists and
every rank solves their union (host model of ad_shard_levels_solve: longest path in executeAt order).  Both
ranks must hold the oracle's levels of the unsharded batch for every txn after that single exchange.

The per-round delta exchange (levels="rounds"):

Each rank holds the key chains of its key range only (a store's CommandsForKey); per round it resolves the
levels of its local txns from its chains with the levels it knows as lower bounds, and sends each peer that
also holds a txn the levels it raised (u64 global rank << 32 | level pairs) — the product path
sharding.run_levels + GlooTransport.allreduce_levels in delta mode, with the store's local round played by a
host model of the engine's round (HostLevelStore: the notifyManaged DP over the store's own chains, oracle.cpp
exec_levels restricted to the store's keys).  The fixpoint must equal the oracle's levels of the unsharded
batch for every txn, and pairs travel only between holders.
"""
import os
import socket
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class HostLevelStore:
    """Host model of ad_shard_levels_round / _deltas / _apply (csrc/shard_kernels.h k_level_deltas,
    k_level_apply) for pure key batches of Reads and Writes."""

    delta = True

    def __init__(self, local, gid, holders, n_global, rank, world):
        self.b, self.gid, self.holders = local, gid, holders.astype(np.int64)
        self.rank, self.world = rank, world
        self.G = np.zeros(n_global, np.uint64)
        lsb, msb = local["exec_lsb"], local["exec_msb"]
        self.by_exec = np.lexsort((local["exec_node"].astype(np.int64), lsb & np.uint64(0x1E), lsb >> np.uint64(16), msb))
        self.write = ((local["txn_lsb"] >> np.uint64(1)) & np.uint64(7)) == 1
        self.sent = []

    def levels_round(self, first):
        n = self.b["n"]
        lo = np.zeros(n, np.int64) if first else self.G[self.gid].astype(np.int64)
        lvl = np.zeros(n, np.int64)
        max_all, max_w = {}, {}
        ko, keys = self.b["key_off"], self.b["keys"]
        for t in self.by_exec:
            lv = -1
            ks = [int(k) for k in keys[ko[t]:ko[t + 1]]]
            for k in ks:
                lv = max(lv, max_all.get(k, -1) if self.write[t] else max_w.get(k, -1))
            lvl[t] = max(lv + 1, lo[t])
            for k in ks:
                max_all[k] = max(max_all.get(k, -1), lvl[t])
                if self.write[t]:
                    max_w[k] = max(max_w.get(k, -1), lvl[t])
        up = lvl > self.G[self.gid].astype(np.int64)
        self.G[self.gid[up]] = lvl[up].astype(np.uint64)
        others = ((1 << self.world) - 1) & ~(1 << self.rank)
        self.cnt = np.zeros(self.world, np.uint32)
        parts = []
        for d in range(self.world):
            sel = up & ((self.holders & others & (1 << d)) != 0)
            self.cnt[d] = sel.sum()
            parts.append((self.gid[sel].astype(np.uint64) << np.uint64(32)) | lvl[sel].astype(np.uint64))
        self.pairs = np.concatenate(parts) if parts else np.zeros(0, np.uint64)
        self.sent.append(int(self.cnt.sum()))
        return bool(self.cnt.sum())

    def level_deltas(self):
        return self.cnt, self.pairs

    def levels_apply(self, pairs):
        g = (pairs >> np.uint64(32)).astype(np.int64)
        lv = pairs & np.uint64(0xFFFFFFFF)
        np.maximum.at(self.G, g, lv)


class HostEdgeStore:
    """Host model of ad_shard_level_edges / ad_shard_levels_solve (csrc/global_levels.h) for pure key batches
    of Reads and Writes."""

    def __init__(self, local, gid, n_global, glob):
        self.b, self.gid, self.n_global, self.glob = local, gid, n_global, glob

    @staticmethod
    def _exec_order(b):
        lsb, msb = b["exec_lsb"], b["exec_msb"]
        return np.lexsort((b["exec_node"].astype(np.int64), lsb & np.uint64(0x1E), lsb >> np.uint64(16), msb))

    def level_edges(self):
        b = self.b
        write = ((b["txn_lsb"] >> np.uint64(1)) & np.uint64(7)) == 1
        chains = {}
        ko, keys = b["key_off"], b["keys"]
        for t in self._exec_order(b):
            for k in keys[ko[t]:ko[t + 1]]:
                chains.setdefault(int(k), []).append(int(t))
        edges = []
        for ch in chains.values():
            last_w, reads = -1, []
            for t in ch:
                if write[t]:
                    for s in (reads if reads else ([last_w] if last_w >= 0 else [])):
                        edges.append((int(self.gid[s]) << 32) | int(self.gid[t]))
                    last_w, reads = t, []
                else:
                    if last_w >= 0:
                        edges.append((int(self.gid[last_w]) << 32) | int(self.gid[t]))
                    reads.append(t)
        return np.array(edges, np.uint64)

    def levels_solve(self, edges):
        src = (edges >> np.uint64(32)).astype(np.int64)
        dst = (edges & np.uint64(0xFFFFFFFF)).astype(np.int64)
        pos = np.empty(self.n_global, np.int64)
        pos[self._exec_order(self.glob)] = np.arange(self.n_global)
        assert np.all(pos[src] < pos[dst]), "every constraint edge runs forward in executeAt order"
        order = np.argsort(pos[dst], kind="stable")
        self.G = np.zeros(self.n_global, np.int64)
        for e in order:                                    # dst ascending in executeAt: srcs final first
            self.G[dst[e]] = max(self.G[dst[e]], self.G[src[e]] + 1)
        return int(self.G.max()) + 1


def _gather_worker(rank, world, port, n):
    sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from accord_amd import abi, sharding, workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = workload.generate(n, 3, 3000, "zipf", seed=12)           # deep chains crossing both stores
        bounds = sharding.even_bounds(0, 3000, world)
        local, gid, _ = sharding.slice_for_shard(b, bounds[rank], bounds[rank + 1])
        store = HostEdgeStore(local, gid, n, b)
        depth = sharding.GlooTransport(dist).gather_levels(store)
        want, _ = O.OracleResult(b, abi.make_config(32, 1, 0.0, 1), O.FLAG_MERGE | O.FLAG_LEVELS).levels()
        assert np.array_equal(store.G.astype(np.uint32), want), "rank %d: levels differ" % rank
        assert depth == int(want.max()) + 1 and depth > 20           # deep, and one exchange resolved it
    finally:
        dist.destroy_process_group()


def test_gather_level_exchange_over_gloo():
    mp.spawn(_gather_worker, args=(2, _free_port(), 2500), nprocs=2, join=True)


def _worker(rank, world, port, n):
    sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import torch
    from accord_amd import abi, sharding, workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = workload.generate(n, 3, 3000, "zipf", seed=11)           # deep chains crossing both stores
        bounds = sharding.even_bounds(0, 3000, world)
        masks = sharding.holder_masks(b, bounds)
        local, gid, _ = sharding.slice_for_shard(b, bounds[rank], bounds[rank + 1])
        assert (masks[gid] & (1 << rank)).all()
        store = HostLevelStore(local, gid, masks[gid], n, rank, world)
        tr = sharding.GlooTransport(dist)
        rounds = sharding.run_levels(store, tr)
        assert rounds >= 2                                           # the chains really couple across stores
        want, _ = O.OracleResult(b, abi.make_config(32, 1, 0.0, 1), O.FLAG_MERGE | O.FLAG_LEVELS).levels()
        got = store.G[gid].astype(np.uint32)
        assert np.array_equal(got, want[gid]), "rank %d: levels differ at %s" % (rank, np.nonzero(got != want[gid])[0][:8])
        # only levels of txns the peer also holds travel, never more than once per raise
        shared = int(((masks[gid] & ~np.uint8(1 << rank)) != 0).sum())
        assert store.sent[0] <= shared
        tot = torch.tensor([sum(store.sent)], dtype=torch.int64)
        dist.all_reduce(tot)
        assert tot.item() > 0
    finally:
        dist.destroy_process_group()


def test_delta_level_exchange_over_gloo():
    mp.spawn(_worker, args=(2, _free_port(), 3000), nprocs=2, join=True)


def test_holder_masks():
    sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
    from accord_amd import sharding
    b = {"n": 4, "key_off": np.array([0, 2, 2, 3, 5], np.uint32),
         "keys": np.array([1, 9, 5, 2, 8], np.uint64)}
    m = sharding.holder_masks(b, sharding.even_bounds(0, 10, 2))
    assert m.tolist() == [3, 0, 2, 3]


class HostKahnStore:
    """Host model of ad_shard_kahn_begin / _step / _finish / _depth (csrc/kahn_shard_kernels.h) for pure key batches of
    Reads and Writes: the store's own constraint edges (HostEdgeStore.level_edges, the engine's levels_export_edges) over
    its local rows; a row whose last local predecessor was released sends READY (with its level bound: 1 + the greatest
    level among its local predecessors) to every holder of its txn (itself included); a row is released once all of its
    txn's holders reported it, at the greatest bound of their READYs (whatever wave delivered them)."""

    delta = True

    def __init__(self, local, gid, holders, home, n_global, rank, world, glob):
        self.gid, self.holders = gid, holders.astype(np.int64)
        self.rank, self.world, self.n_global = rank, world, n_global
        self._edges = HostEdgeStore(local, gid, n_global, glob)
        self.row = {int(g): i for i, g in enumerate(gid)}
        self.G = np.zeros(n_global, np.uint64)

    def _ready(self, i):
        for d in range(self.world):
            if (self.holders[i] >> d) & 1:
                self.out[d].append(int(self.gid[i]) | (int(self.plv[i]) << 32))

    def kahn_begin(self):
        n = len(self.gid)
        e = self._edges.level_edges()
        self.succ = [[] for _ in range(n)]
        self.rem = np.zeros(n, np.int64)
        for x in e:
            s_, d_ = self.row[int(x) >> 32], self.row[int(x) & 0xFFFFFFFF]
            self.succ[s_].append(d_)
            self.rem[d_] += 1
        self.rcnt = np.zeros(n, np.int64)
        self.lacc = np.zeros(n, np.int64)
        self.plv = np.zeros(n, np.int64)
        self.lvl = np.full(n, -1, np.int64)
        self.sent = 0
        self.out = {d: [] for d in range(self.world)}
        for i in np.nonzero(self.rem == 0)[0]:
            self._ready(i)

    def kahn_outbox(self):
        cnt = np.array([len(self.out[d]) for d in range(self.world)], np.uint32)
        self.sent += int(cnt.sum()) - int(cnt[self.rank])
        msgs = np.array([g for d in range(self.world) for g in self.out[d]], np.uint64)
        self.out = {d: [] for d in range(self.world)}
        return cnt, msgs

    def kahn_inbox(self, msgs):
        self.inbox = [int(g) for g in msgs]

    def kahn_step(self, level):
        for m in self.inbox:
            g, lb = m & 0xFFFFFFFF, m >> 32
            r = self.row[g]
            assert self.lvl[r] < 0, "no READY for a released txn"
            self.lacc[r] = max(self.lacc[r], lb)
            self.rcnt[r] += 1
            if self.rcnt[r] == bin(int(self.holders[r])).count("1"):
                L = int(self.lacc[r])
                self.lvl[r] = L
                self.G[g] = L
                for s_ in self.succ[r]:
                    self.plv[s_] = max(self.plv[s_], L + 1)
                    self.rem[s_] -= 1
                    if self.rem[s_] == 0:
                        self._ready(s_)
        self.inbox = []

    def kahn_finish(self):
        return int((self.lvl < 0).sum())

    def kahn_depth(self):
        return int(self.lvl.max()) + 1 if len(self.lvl) else 0

    def kahn_sent(self):
        return self.sent


class HostAutoStore(HostKahnStore):
    """Both level interfaces (Kahn waves and edges) over one store, as the engine's ShardStore has them."""

    def level_edges(self):
        return self._edges.level_edges()

    def levels_solve(self, edges):
        depth = self._edges.levels_solve(edges)
        self.G = self._edges.G.astype(np.uint64)
        return depth


def _kahn_worker(rank, world, port, n, dist_kind, slot=None):
    sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import torch
    from accord_amd import abi, sharding, workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ks = 3000 if dist_kind == "zipf" else 200_000
        b = workload.generate(n, 3, ks, dist_kind, seed=14)
        bounds = sharding.even_bounds(0, ks, world)
        masks = sharding.holder_masks(b, bounds)
        hs = sharding.home_stores(b, bounds)
        local, gid, _ = sharding.slice_for_shard(b, bounds[rank], bounds[rank + 1])
        store = HostKahnStore(local, gid, masks[gid], hs[gid], n, rank, world, b)
        waves = sharding.run_levels_kahn(store, sharding.GlooTransport(dist, kahn_slot=slot))
        want, _ = O.OracleResult(b, abi.make_config(32, 1, 0.0, 1), O.FLAG_MERGE | O.FLAG_LEVELS).levels()
        assert np.array_equal(store.lvl.astype(np.uint32), want[gid]), "rank %d: levels differ" % rank
        assert store.depth == int(want.max()) + 1
        # every queued READY each wave: one wave per level; bounded slots: READYs arrive late, the levels do not move
        assert waves == store.depth + 1 if slot is None else waves > store.depth + 1
        # per local row exactly one READY to each other holder crosses the wire over the batch (never per round)
        others = ((masks[gid].astype(np.int64) & ~(1 << rank)) != 0).sum()
        bound = torch.tensor([store.kahn_sent(), int(sum(bin(int(m)).count("1") - 1 for m in masks[gid]))],
                             dtype=torch.int64)
        assert bound[0] == bound[1] and (others == 0 or bound[0] > 0), bound
        assert store.kahn_bytes == 8 * store.kahn_sent()
    finally:
        dist.destroy_process_group()


def test_kahn_level_waves_over_gloo():
    # uniform keys (C5-like, shallow) and Zipf hot keys (deep chains crossing both stores)
    mp.spawn(_kahn_worker, args=(2, _free_port(), 3000, "uniform"), nprocs=2, join=True)
    mp.spawn(_kahn_worker, args=(2, _free_port(), 2000, "zipf"), nprocs=2, join=True)


def test_kahn_level_waves_bounded_slots_over_gloo():
    # at most a few READYs per (source, destination) and wave (ad_shard_kahn_run's fixed slots): late READYs, exact
    # levels; three ranks too
    mp.spawn(_kahn_worker, args=(2, _free_port(), 3000, "uniform", 5), nprocs=2, join=True)
    mp.spawn(_kahn_worker, args=(3, _free_port(), 2000, "zipf", 3), nprocs=3, join=True)


def _auto_worker(rank, world, port, n, dist_kind, cap):
    sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from accord_amd import abi, sharding, workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ks = 3000 if dist_kind == "zipf" else 200_000
        b = workload.generate(n, 3, ks, dist_kind, seed=13)
        bounds = sharding.even_bounds(0, ks, world)
        masks = sharding.holder_masks(b, bounds)
        local, gid, _ = sharding.slice_for_shard(b, bounds[rank], bounds[rank + 1])
        store = HostAutoStore(local, gid, masks[gid], sharding.home_stores(b, bounds)[gid], n, rank, world, b)
        rounds = sharding.run_levels_auto(store, sharding.GlooTransport(dist), round_cap=cap)
        want, _ = O.OracleResult(b, abi.make_config(32, 1, 0.0, 1), O.FLAG_MERGE | O.FLAG_LEVELS).levels()
        assert np.array_equal(store.G[gid].astype(np.uint32), want[gid]), "rank %d: levels differ" % rank
        if dist_kind == "zipf":
            assert rounds == cap + 1, "a deep graph falls back to the one-exchange gather"
        else:
            assert rounds <= cap, "a shallow graph finishes in Kahn waves"
        # the next batch on the same store: the previous depth decides up front (a deep one skips the waves)
        begun = []
        store.kahn_begin = lambda f=store.kahn_begin: (begun.append(1), f())[1]
        again = sharding.run_levels_auto(store, sharding.GlooTransport(dist), round_cap=cap)
        assert np.array_equal(store.G[gid].astype(np.uint32), want[gid])
        if dist_kind == "zipf":
            assert again == cap + 1 and not begun, "deep again: straight to the gather"
        else:
            assert again <= cap and begun
    finally:
        dist.destroy_process_group()


def test_auto_levels_rounds_over_gloo():
    # C5-like uniform keys: the Kahn waves finish, no edge exchange
    mp.spawn(_auto_worker, args=(2, _free_port(), 3000, "uniform", 64), nprocs=2, join=True)


def test_auto_levels_fall_back_to_gather_over_gloo():
    # Zipf hot keys with a small round cap: every rank switches to the gather together, levels still exact
    mp.spawn(_auto_worker, args=(2, _free_port(), 2500, "zipf", 3), nprocs=2, join=True)
