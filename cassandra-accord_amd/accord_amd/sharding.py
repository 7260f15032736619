"""Key-range sharding of a batch across CommandStores / GPUs (BASELINE C5).

Mirrors Accord's per-range CommandStore sharding (local/CommandStores.java:576-593,
local/ShardDistributor.java:32-80) and PreAccept.reduce across stores (messages/PreAccept.java:141-156):

* ``even_bounds`` / ``slice_for_shard`` / ``home_stores`` — host-side partitioning: store s owns keys in
  [bounds[s], bounds[s+1]); its local batch is every txn touching that range with its keys sliced to it, in
  global TxnId order; ``gid`` maps local rows to global ranks; a txn's home store is the store of its first
  key (the store that merges its deps).
* ``ShardStore`` — one store on one GPU (an ad_handle in sharded mode), driving the C-ABI protocol.
* transports — how stores exchange blobs and level arrays: ``RcclTransport`` (grouped ncclSend/ncclRecv
  all-to-all and ncclAllReduce on device buffers over xGMI, inside libaccord_deps; torch.distributed/gloo
  only carries the unique id, the per-destination byte counts and one scalar per level round),
  ``GlooTransport`` (host staging over a gloo group; used for tests and as the explicit host path),
  ``LocalTransport`` (several stores in one process, for tests).  Each store sends every other store only
  the deps rows of the txns homed there, and only rows that have deps.
* ``run_store`` — the per-store protocol: preaccept, export, exchange, merge, distributed levels, order.

Every computation runs on the GPU through the C-ABI; the transports only move bytes.
"""
import ctypes as C

import numpy as np

from . import abi, engine


def even_bounds(key_lo, key_hi, shards):
    """ShardDistributor.EvenSplit over [key_lo, key_hi): shards + 1 boundaries (last = 2^64-1)."""
    span = key_hi - key_lo
    b = [key_lo + (span * s) // shards for s in range(shards)]
    return np.array(b + [np.iinfo(np.uint64).max], np.uint64)


def _ranges(batch):
    ro = batch.get("range_off")
    if ro is None or int(ro[-1]) == 0:
        return None
    return (np.asarray(ro, np.int64), np.asarray(batch["range_start"], np.uint64), np.asarray(batch["range_end"], np.uint64))


def _clip_ranges(rs, re, lo, hi):
    """(start, end] ranges cut to the store owning keys [lo, hi): (max(start, lo - 1), min(end, hi - 1)] — the
    range commands' slice to the store's ranges (impl/InMemoryCommandStore.java:758-761, Ranges.slice)."""
    lo, hi = int(lo), int(hi)
    s = np.maximum(rs, np.uint64(lo - 1)) if lo > 0 else rs.copy()
    e = np.minimum(re, np.uint64(hi - 1))
    return s, e, s < e


def slice_for_shard(batch, lo, hi):
    """(local batch, gid, home) of the store owning keys [lo, hi): every txn with a key in range or a range
    meeting it, keys cut to the range and ranges sliced to it (_clip_ranges), TxnId order kept."""
    n = batch["n"]
    ko = batch["key_off"].astype(np.int64)
    keys = batch["keys"]
    inr = (keys >= np.uint64(lo)) & (keys < np.uint64(hi))
    owner = np.repeat(np.arange(n, dtype=np.int64), np.diff(ko))
    cnt = np.bincount(owner[inr], minlength=n)
    rg = _ranges(batch)
    if rg is not None:
        ro, rs, re = rg
        cs, ce, keep = _clip_ranges(rs, re, lo, hi)
        rowner = np.repeat(np.arange(n, dtype=np.int64), np.diff(ro))
        rcnt = np.bincount(rowner[keep], minlength=n)
    else:
        rcnt = np.zeros(n, np.int64)
    touch = (cnt > 0) | (rcnt > 0)
    gid = np.nonzero(touch)[0].astype(np.uint32)
    hs = home_stores(batch, np.array([lo, hi], np.uint64), clip=False)
    home = (hs[gid] == 0).astype(np.uint8)
    local = {"n": int(len(gid))}
    for f in ("txn_msb", "txn_lsb", "txn_node", "exec_msb", "exec_lsb", "exec_node", "status"):
        local[f] = np.ascontiguousarray(batch[f][gid])
    lk = np.zeros(len(gid) + 1, np.uint32)
    lk[1:] = np.cumsum(cnt[gid])
    local["key_off"] = lk
    local["keys"] = np.ascontiguousarray(keys[inr])
    if rg is not None and int(rcnt.sum()) > 0:
        lr = np.zeros(len(gid) + 1, np.uint32)
        lr[1:] = np.cumsum(rcnt[gid])
        local["range_off"] = lr
        local["range_start"] = np.ascontiguousarray(cs[keep])
        local["range_end"] = np.ascontiguousarray(ce[keep])
    else:
        local["range_off"] = local["range_start"] = local["range_end"] = None
    return local, gid, home


def home_stores(batch, bounds, clip=True):
    """Per global txn: the store owning its first key — for a range txn the first key its first range covers,
    start + 1 — (its home; merges its deps).  clip=False: -1 / len(bounds) - 1 outside the bounds."""
    ko = batch["key_off"].astype(np.int64)
    keys = batch["keys"]
    n = batch["n"]
    first = np.zeros(n, np.uint64)
    nz = ko[1:] > ko[:-1]
    first[nz] = keys[ko[:-1][nz]]
    rg = _ranges(batch)
    if rg is not None:
        ro, rs, _ = rg
        has = ro[1:] > ro[:-1]
        first[has & ~nz] = rs[ro[:-1][has & ~nz]] + np.uint64(1)
    hs = np.searchsorted(np.asarray(bounds, np.uint64), first, side="right") - 1
    if not clip:
        return hs
    return np.clip(hs, 0, len(bounds) - 2).astype(np.uint8)


def holder_masks(batch, bounds):
    """Per global txn: bitmask of the stores holding it (the stores owning any of its keys, or meeting any of
    its ranges).  A store's chains hold only its own txns, so in the level rounds a raised level travels only
    to the other holders (ShardStore.set_holders, the delta exchange)."""
    n = batch["n"]
    ko = batch["key_off"].astype(np.int64)
    keys = batch["keys"]
    b = np.asarray(bounds, np.uint64)
    S = len(b) - 1
    st = np.clip(np.searchsorted(b, keys, side="right") - 1, 0, S - 1)
    bits = (np.uint16(1) << st.astype(np.uint16)).astype(np.uint16)
    out = np.zeros(n, np.uint16)
    nz = ko[1:] > ko[:-1]
    if len(keys):
        red = np.bitwise_or.reduceat(bits, ko[:-1][nz])
        out[nz] = red
    rg = _ranges(batch)
    if rg is not None:
        ro, rs, re = rg
        first = np.clip(np.searchsorted(b, rs + np.uint64(1), side="right") - 1, 0, S - 1)
        last = np.clip(np.searchsorted(b, re, side="right") - 1, 0, S - 1)
        rb = np.zeros(len(rs), np.uint16)
        for k in range(S):
            rb |= (((first <= k) & (k <= last)).astype(np.uint16) << np.uint16(k)).astype(np.uint16)
        has = ro[1:] > ro[:-1]
        out[has] |= np.bitwise_or.reduceat(rb, ro[:-1][has])
    return out.astype(np.uint8)


def presplit(batch, bounds):
    """The global batch with every range cut at the store boundaries (each piece = one store's slice,
    _clip_ranges).  Its unsharded deps are what the sharded stores produce together: RangeDeps are keyed by
    the store-sliced ranges, while KeyDeps, TxnId sets, witnessedAt and levels do not depend on
    the split."""
    rg = _ranges(batch)
    if rg is None:
        return batch
    ro, rs, re = rg
    b = np.asarray(bounds, np.uint64)
    S = len(b) - 1
    n = batch["n"]
    rowner = np.repeat(np.arange(n, dtype=np.int64), np.diff(ro))
    ps, pe, po, pk = [], [], [], []
    for k in range(S):
        s, e, keep = _clip_ranges(rs, re, b[k], b[k + 1])
        idx = np.nonzero(keep)[0]
        ps.append(s[idx]); pe.append(e[idx]); po.append(rowner[idx]); pk.append(idx * (S + 1) + k)
    ps, pe, po, pk = (np.concatenate(x) for x in (ps, pe, po, pk))
    order = np.argsort(pk, kind="stable")                 # by (original range, store): ascending per txn
    out = dict(batch)
    out["range_start"] = np.ascontiguousarray(ps[order])
    out["range_end"] = np.ascontiguousarray(pe[order])
    cnt = np.bincount(po, minlength=n)
    out["range_off"] = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    return out


def reduce_witnessed(batch, parts):
    """PreAccept.reduce of the stores' witnessedAt proposals (messages/PreAccept.java:141-156: witnessedAt =
    Timestamp.mergeMax, Timestamp.java:273-279) for the global batch: parts = [(gid, max_rank, fast)] per
    store (ShardStore.max_conflicts).  Per view and global txn:
      rank   the txn whose executeAt wins mergeMax over the stores' answers: Timestamp.compareToWithoutEpoch
             (Timestamp.java:219-227: highHlc, lowHlc, identity flags, node), ties to the larger rank;
      fast   every store answered TxnId (fast path);
      epoch  mergeMax's withEpochAtLeast: the greatest epoch among the stores' answers (0 for Timestamp.NONE).
    In a single-epoch batch the winner's executeAt is exactly the merged witnessedAt; across epochs the merged
    value is the winner's (hlc, flags, node) at `epoch`.  A host-side fold of n x R integers, like the
    coordinator's fold over replica replies; the per-store work runs on the GPU."""
    n = batch["n"]
    R = parts[0][1].shape[0] if parts else 1
    j = np.arange(n, dtype=np.int64)
    msb, lsb = batch["exec_msb"], batch["exec_lsb"]
    # strict total order of (executeAt without epoch, rank): highHlc, lowHlc, identity flags, node signed, rank
    order = np.lexsort((j, batch["exec_node"].astype(np.int64), lsb & np.uint64(0x1E),
                        lsb >> np.uint64(16), msb & np.uint64(0x7FFF)))
    pos = np.empty(n, np.int64)
    pos[order] = j
    epoch_of = (msb >> np.uint64(15)).astype(np.int64)
    best = np.full((R, n), -1, np.int64)
    ep = np.zeros((R, n), np.int64)
    fast = np.ones((R, n), np.uint8)
    for gid, rank, f in parts:
        gid = np.asarray(gid, np.int64)
        has = rank != abi.AD_RANK_NONE
        safe = np.where(has, rank, 0).astype(np.int64)
        p = np.where(has, pos[safe], -1)
        e = np.where(has, epoch_of[safe], 0)
        for v in range(R):
            best[v, gid] = np.maximum(best[v, gid], p[v])
            ep[v, gid] = np.maximum(ep[v, gid], e[v])
            # fast only if every store answered TxnId; rejected (AD_FAST_REJECTED) if any store rejected it: mergeMax
            # keeps the REJECTED flag (Timestamp.mergeFlags, PreAccept.reduce :141-156)
            cur = fast[v, gid]
            fast[v, gid] = np.where((cur == 2) | (f[v] == 2), 2, cur & f[v])
    out = np.full((R, n), abi.AD_RANK_NONE, np.uint32)
    has = best >= 0
    out[has] = order[best[has]].astype(np.uint32)
    return out, fast, ep.astype(np.uint64)


def _u32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


class ShardStore:
    """One CommandStore of a key-range-sharded batch on one GPU."""

    def __init__(self, device, window=32, replicas=3, drop_p=0.1, seed=0xACC0D1):
        self.eng = engine.DepsEngine(device=device, window=window, replicas=replicas, drop_p=drop_p, seed=seed)
        self.replicas = replicas
        self.L = engine.lib()
        L = self.L
        vp = C.c_void_p
        u64p = C.POINTER(C.c_uint64)
        L.ad_shard_setup.argtypes = [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint8), C.c_uint32, C.c_uint32, C.c_size_t]
        L.ad_shard_export.argtypes = [vp, u64p]
        L.ad_shard_send_to_host.argtypes = [vp, C.c_void_p]
        L.ad_shard_import_host.argtypes = [vp, C.c_void_p, C.c_uint32, u64p]
        L.ad_comm_unique_id.argtypes = [C.POINTER(C.c_uint8)]
        L.ad_comm_init.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint8)]
        L.ad_comm_destroy.argtypes = [vp]
        L.ad_shard_query_positions.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.ad_shard_alltoall.argtypes = [vp, u64p]
        L.ad_shard_merge.argtypes = [vp, C.POINTER(abi.AdCsrSizes), C.POINTER(C.c_size_t)]
        L.ad_shard_fetch.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(abi.AdCsrOut), C.POINTER(C.c_uint32)]
        L.ad_shard_levels_round.argtypes = [vp, C.c_int, C.POINTER(C.c_uint32)]
        L.ad_shard_levels_get.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.ad_shard_levels_set.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.ad_shard_levels_allreduce.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.ad_shard_order.argtypes = [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.ad_shard_set_holders.argtypes = [vp, C.POINTER(C.c_uint8)]
        L.ad_shard_levels_deltas.argtypes = [vp, C.POINTER(C.c_uint32), u64p]
        L.ad_shard_levels_apply.argtypes = [vp, u64p, C.c_size_t]
        L.ad_shard_levels_exchange.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.ad_shard_level_edges.argtypes = [vp, C.POINTER(C.c_size_t), u64p]
        L.ad_shard_levels_solve.argtypes = [vp, u64p, C.c_size_t, C.POINTER(C.c_uint32)]
        L.ad_shard_levels_gather.argtypes = [vp, C.POINTER(C.c_uint32)]
        L.ad_shard_kahn_begin.argtypes = [vp]
        L.ad_shard_kahn_outbox.argtypes = [vp, C.POINTER(C.c_uint32), u64p]
        L.ad_shard_kahn_inbox.argtypes = [vp, u64p, C.c_size_t]
        L.ad_shard_kahn_exchange.argtypes = [vp, C.c_uint32, C.POINTER(C.c_uint32)]
        L.ad_shard_kahn_step.argtypes = [vp, C.c_uint32]
        L.ad_shard_kahn_finish.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.ad_shard_kahn_sent.argtypes = [vp, C.POINTER(C.c_uint64)]
        L.ad_shard_kahn_run.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]
        L.ad_shard_kahn_depth.argtypes = [vp, C.POINTER(C.c_uint32)]
        self.delta = False
        self.pairs_sent = 0

    def close(self):
        self.eng.close()

    def _check(self, rc, what):
        self.eng._check(rc, what)

    # ---- protocol steps
    def load(self, local_batch, gid, home_store, n_global, rank, world, holders=None):
        """home_store: per local row, the store of the txn's first key (home_stores(global)[gid]); holders
        (optional): per local row, the bitmask of stores holding the txn (holder_masks(global)[gid]) —
        given, the level rounds exchange only raised levels of shared txns (delta mode), else the whole
        global level array is all-reduced each round (dense mode)."""
        self.eng.load(local_batch)
        self.gid = np.ascontiguousarray(gid, np.uint32)
        self.home_store = np.ascontiguousarray(home_store, np.uint8)
        self.n_global = n_global
        self.rank, self.world = rank, world
        self._check(self.L.ad_shard_setup(self.eng.h, _u32p(self.gid), self.home_store.ctypes.data_as(C.POINTER(C.c_uint8)),
                                          rank, world, n_global), "ad_shard_setup")
        self.delta = holders is not None
        if self.delta:
            self.holders = np.ascontiguousarray(holders, np.uint8)
            self._check(self.L.ad_shard_set_holders(self.eng.h, self.holders.ctypes.data_as(C.POINTER(C.c_uint8))),
                        "ad_shard_set_holders")

    def accept(self, gq=None, bound_max=False):
        """Accept / GetDeps deps of the slice (bound = executeAt; gq = the global arrival positions of the local
        rows' executeAts, query_positions), or GetEphemeralReadDeps (bound = Timestamp.MAX)."""
        if bound_max:
            self.eng.ephemeral_read_deps()
            return
        g = np.ascontiguousarray(gq, np.uint32)
        self._check(self.L.ad_shard_query_positions(self.eng.h, _u32p(g)), "ad_shard_query_positions")
        self.eng.accept_deps()

    def preaccept(self):
        self._check(self.L.ad_preaccept_deps(self.eng.h, None), "ad_preaccept_deps")

    def max_conflicts(self):
        """This store's witnessedAt proposal per view for its local rows (ad_max_conflicts after the deps
        stage): (max_rank [R, n_local] as global ranks, fast [R, n_local])."""
        return self.eng.max_conflicts()

    def export(self):
        """Per-destination blobs on the device; returns their byte sizes (np.uint64[world])."""
        b = np.zeros(self.world, np.uint64)
        self._check(self.L.ad_shard_export(self.eng.h, b.ctypes.data_as(C.POINTER(C.c_uint64))), "ad_shard_export")
        self.send_sizes = b
        return b

    def send_buffer(self):
        """The blobs, concatenated in destination order (host copy)."""
        out = np.zeros(max(int(self.send_sizes.sum()), 1), np.uint8)
        self._check(self.L.ad_shard_send_to_host(self.eng.h, out.ctypes.data), "ad_shard_send_to_host")
        return out[:int(self.send_sizes.sum())]

    def import_host(self, recv, sizes):
        """Blobs received from every store (source order), sizes[s] bytes each."""
        recv = np.ascontiguousarray(recv, np.uint8)
        if recv.size == 0:
            recv = np.zeros(1, np.uint8)
        sizes = np.ascontiguousarray(sizes, np.uint64)
        self._check(self.L.ad_shard_import_host(self.eng.h, recv.ctypes.data, self.world,
                                                sizes.ctypes.data_as(C.POINTER(C.c_uint64))), "ad_shard_import_host")

    def alltoall(self, recv_sizes):
        rs = np.ascontiguousarray(recv_sizes, np.uint64)
        self._check(self.L.ad_shard_alltoall(self.eng.h, rs.ctypes.data_as(C.POINTER(C.c_uint64))), "ad_shard_alltoall")

    def comm_init(self, world, rank, uid):
        u = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._check(self.L.ad_comm_init(self.eng.h, world, rank, u), "ad_comm_init")

    def comm_destroy(self):
        self._check(self.L.ad_comm_destroy(self.eng.h), "ad_comm_destroy")


    def merge(self):
        sizes = (abi.AdCsrSizes * ((self.replicas + 1) * abi.NUM_CLASSES))()
        nh = C.c_size_t()
        self._check(self.L.ad_shard_merge(self.eng.h, sizes, C.byref(nh)), "ad_shard_merge")
        self._sizes = sizes
        self.n_home = nh.value
        return nh.value

    def fetch(self, view, cls):
        """Home txns' CSR of `view` (view == replicas: merged) and their global ranks."""
        s = self._sizes[view * abi.NUM_CLASSES + cls]
        out = abi.Csr.alloc(s, is_range=(cls == abi.CLASS_RANGE))
        hg = np.zeros(max(self.n_home, 1), np.uint32)
        o = out.as_out()
        self._check(self.L.ad_shard_fetch(self.eng.h, view, cls, C.byref(o), _u32p(hg)), "ad_shard_fetch")
        return out, hg[:self.n_home]

    def levels_round(self, first):
        ch = C.c_uint32()
        self._check(self.L.ad_shard_levels_round(self.eng.h, 1 if first else 0, C.byref(ch)), "ad_shard_levels_round")
        if self.delta:
            if first:
                self.pairs_sent = 0
            cnt = np.zeros(self.world, np.uint32)
            self._check(self.L.ad_shard_levels_deltas(self.eng.h, _u32p(cnt), None), "ad_shard_levels_deltas")
            self.pairs_sent += int(cnt.sum())       # level exchange volume of this batch: 8 B per pair
        return bool(ch.value)

    def levels_get(self):
        g = np.zeros(max(self.n_global, 1), np.uint32)
        self._check(self.L.ad_shard_levels_get(self.eng.h, _u32p(g)), "ad_shard_levels_get")
        return g[:self.n_global]

    def levels_set(self, g):
        g = np.ascontiguousarray(g, np.uint32)
        self._check(self.L.ad_shard_levels_set(self.eng.h, _u32p(g)), "ad_shard_levels_set")

    def levels_allreduce(self):
        """RCCL all-reduce(max) of the level array; returns whether any store raised a level this round."""
        ch = C.c_uint32()
        self._check(self.L.ad_shard_levels_allreduce(self.eng.h, C.byref(ch)), "ad_shard_levels_allreduce")
        return bool(ch.value)

    def level_deltas(self):
        """Delta mode: the last round's (gid << 32 | level) pairs per destination: (counts[world], pairs)."""
        cnt = np.zeros(self.world, np.uint32)
        self._check(self.L.ad_shard_levels_deltas(self.eng.h, _u32p(cnt), None), "ad_shard_levels_deltas")
        pairs = np.zeros(max(int(cnt.sum()), 1), np.uint64)
        self._check(self.L.ad_shard_levels_deltas(self.eng.h, _u32p(cnt), pairs.ctypes.data_as(C.POINTER(C.c_uint64))),
                    "ad_shard_levels_deltas")
        return cnt, pairs[:int(cnt.sum())]

    def levels_apply(self, pairs):
        p = np.ascontiguousarray(pairs, np.uint64)
        if p.size == 0:
            return
        self._check(self.L.ad_shard_levels_apply(self.eng.h, p.ctypes.data_as(C.POINTER(C.c_uint64)), p.size),
                    "ad_shard_levels_apply")

    def levels_exchange(self):
        """RCCL delta exchange; returns whether any store sent a pair this round."""
        ch = C.c_uint32()
        self._check(self.L.ad_shard_levels_exchange(self.eng.h, C.byref(ch)), "ad_shard_levels_exchange")
        return bool(ch.value)

    # ---- one-exchange levels (the default): this store's constraint edges, every store's edges solved
    def level_edges_compute(self):
        """This store's execution constraints as global-rank edges, kept on the device; returns their count."""
        m = C.c_size_t(0)
        self._check(self.L.ad_shard_level_edges(self.eng.h, C.byref(m), None), "ad_shard_level_edges")
        self.n_edges = m.value
        return m.value

    def level_edges(self):
        """The constraint edges as np.uint64 (global src << 32 | global dst), computed on the device."""
        m = self.level_edges_compute()
        out = np.zeros(max(m, 1), np.uint64)
        mm = C.c_size_t(m)
        self._check(self.L.ad_shard_level_edges(self.eng.h, C.byref(mm), out.ctypes.data_as(C.POINTER(C.c_uint64))),
                    "ad_shard_level_edges")
        return out[:m]

    def levels_solve(self, edges):
        """Levels of the whole batch from every store's edges (host array); returns the level count."""
        e = np.ascontiguousarray(edges, np.uint64)
        d = C.c_uint32()
        self._check(self.L.ad_shard_levels_solve(self.eng.h, e.ctypes.data_as(C.POINTER(C.c_uint64)) if e.size else None,
                                                 e.size, C.byref(d)), "ad_shard_levels_solve")
        return d.value

    def levels_gather(self):
        """RCCL: gather every store's edges (after level_edges_compute) and solve; returns the level count."""
        d = C.c_uint32()
        self._check(self.L.ad_shard_levels_gather(self.eng.h, C.byref(d)), "ad_shard_levels_gather")
        return d.value

    # ---- distributed Kahn waves (levels="kahn"; ad_shard_kahn_*)
    def kahn_begin(self):
        """The store's local constraint graph and wave 0's READY messages (needs holder masks)."""
        self._check(self.L.ad_shard_kahn_begin(self.eng.h), "ad_shard_kahn_begin")

    def kahn_outbox(self):
        """The current phase's messages per destination: (counts[world], messages in destination order)."""
        cnt = np.zeros(self.world, np.uint32)
        self._check(self.L.ad_shard_kahn_outbox(self.eng.h, _u32p(cnt), None), "ad_shard_kahn_outbox")
        msgs = np.zeros(max(int(cnt.sum()), 1), np.uint64)
        self._check(self.L.ad_shard_kahn_outbox(self.eng.h, _u32p(cnt), msgs.ctypes.data_as(C.POINTER(C.c_uint64))),
                    "ad_shard_kahn_outbox")
        return cnt, msgs[:int(cnt.sum())]

    def kahn_inbox(self, msgs):
        m = np.ascontiguousarray(msgs, np.uint64)
        self._check(self.L.ad_shard_kahn_inbox(self.eng.h, m.ctypes.data_as(C.POINTER(C.c_uint64)) if m.size else None,
                                               m.size), "ad_shard_kahn_inbox")

    def kahn_exchange(self):
        """RCCL: the outbox to the holders, theirs into the inbox; returns whether any store sent anything."""
        a = C.c_uint32()
        self._check(self.L.ad_shard_kahn_exchange(self.eng.h, 0, C.byref(a)), "ad_shard_kahn_exchange")
        return bool(a.value)

    def kahn_step(self, level):
        """One wave on the device: READYs counted, rows every holder reported released at `level`, their successors'
        READYs into the outbox (no host wait)."""
        self._check(self.L.ad_shard_kahn_step(self.eng.h, level), "ad_shard_kahn_step")

    def kahn_finish(self):
        """After the last wave: the local rows never released (a cycle if any)."""
        u = C.c_uint64()
        self._check(self.L.ad_shard_kahn_finish(self.eng.h, C.byref(u)), "ad_shard_kahn_finish")
        return u.value

    def kahn_run(self, slot=0, check_every=4, lag=2, wave_cap=1 << 16):
        """RCCL: the whole wave loop with fixed exchange slots and no host synchronisation between waves (every
        check_every waves an all-reduce of the READYs still queued, read lag checks later); returns the waves run.
        Raises LevelsNotConverged past wave_cap waves (every store together)."""
        w = C.c_uint32()
        rc = self.L.ad_shard_kahn_run(self.eng.h, slot, check_every, lag, wave_cap, C.byref(w))
        if rc == abi.AD_ERR_UNSUPPORTED:
            raise LevelsNotConverged("Kahn waves still releasing after %d waves" % w.value)
        self._check(rc, "ad_shard_kahn_run")
        return w.value

    def kahn_depth(self):
        """After the waves: the greatest level + 1 (the levels ride in the READYs)."""
        d = C.c_uint32()
        self._check(self.L.ad_shard_kahn_depth(self.eng.h, C.byref(d)), "ad_shard_kahn_depth")
        return d.value

    def kahn_sent(self):
        s_ = C.c_uint64()
        self._check(self.L.ad_shard_kahn_sent(self.eng.h, C.byref(s_)), "ad_shard_kahn_sent")
        return s_.value

    def order(self):
        lv = np.zeros(max(self.n_home, 1), np.uint32)
        od = np.zeros(max(self.n_home, 1), np.uint32)
        self._check(self.L.ad_shard_order(self.eng.h, _u32p(lv), _u32p(od)), "ad_shard_order")
        return lv[:self.n_home], od[:self.n_home]


def query_positions(batch):
    """Per txn of the global batch, the number of its TxnIds below the txn's executeAt under Timestamp.compareTo
    (Timestamp.java:208-217): where an Accept / GetDeps query with bound executeAt is answered."""
    def key(msb, lsb, node):
        return (int(msb), int(lsb) >> 16, int(lsb) & 0x1E, int(node))
    import bisect
    tx = [key(batch["txn_msb"][i], batch["txn_lsb"][i], batch["txn_node"][i]) for i in range(batch["n"])]
    return np.array([bisect.bisect_left(tx, key(batch["exec_msb"][i], batch["exec_lsb"][i], batch["exec_node"][i]))
                     for i in range(batch["n"])], np.uint32)


def unique_id():
    buf = (C.c_uint8 * 128)()
    rc = engine.lib().ad_comm_unique_id(buf)
    if rc != abi.AD_OK:
        raise engine.AccordDepsError(rc, "ad_comm_unique_id failed")
    return bytes(buf)


# ------------------------------------------------------------------------------------------------
# transports
# ------------------------------------------------------------------------------------------------
class GlooTransport:
    """Host staging over a torch.distributed (gloo) process group."""

    name = "host(gloo)"

    def __init__(self, dist, kahn_slot=None):
        self.dist = dist
        import torch
        self.torch = torch
        # Kahn waves: at most kahn_slot READYs per destination and wave (the rest wait in a per-destination backlog,
        # as in ad_shard_kahn_run's fixed slots; None: every queued READY each wave)
        self.kahn_slot = kahn_slot
        self._backlog = None

    def max_u64(self, x):
        t = self.torch.tensor([x], dtype=self.torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return int(t.item())

    def any(self, flag):
        return self.max_u64(1 if flag else 0) > 0

    def recv_sizes(self, send_sizes):
        """All-to-all of the per-destination byte counts: what every peer sends this store."""
        out = self.torch.zeros(len(send_sizes), dtype=self.torch.int64)
        self.dist.all_to_all_single(out, self.torch.from_numpy(np.asarray(send_sizes, np.int64)))
        return out.numpy().astype(np.uint64)

    def exchange_blobs(self, store):
        sizes = store.export()
        rsz = self.recv_sizes(sizes)
        send = self.torch.from_numpy(store.send_buffer().copy())
        recv = self.torch.zeros(int(rsz.sum()), dtype=self.torch.uint8)
        self.dist.all_to_all_single(recv, send, output_split_sizes=[int(x) for x in rsz],
                                    input_split_sizes=[int(x) for x in sizes])
        store.import_host(recv.numpy(), rsz)

    def gather_levels(self, store):
        """One-exchange levels: every store's constraint edges reach every store, then the store solves their
        union.  Returns the level count.  The edges travel as one broadcast per source store into its slice of
        one exactly sized buffer (no padding to the largest store: skewed stores would otherwise hold world x
        the largest edge list)."""
        edges = store.level_edges()
        cnt = self.torch.tensor([edges.size], dtype=self.torch.int64)
        world, me = self.dist.get_world_size(), self.dist.get_rank()
        counts = [self.torch.zeros(1, dtype=self.torch.int64) for _ in range(world)]
        self.dist.all_gather(counts, cnt)
        counts = [int(c.item()) for c in counts]
        allv = self.torch.empty(sum(counts), dtype=self.torch.int64)
        off = 0
        for r, c in enumerate(counts):
            part = allv.narrow(0, off, c)
            if r == me:
                part.copy_(self.torch.from_numpy(edges.view(np.int64)))
            if c:
                self.dist.broadcast(part, src=r)
            off += c
        return store.levels_solve(allv.numpy().view(np.uint64))

    def allreduce_levels(self, store, changed):
        """Delta mode: all-to-all of the raised levels of shared txns; dense mode: all-reduce(max) of the level
        array.  Returns whether any store raised a level another store needs (dense: raised any level)."""
        if store.delta:
            cnt, pairs = store.level_deltas()
            if not self.any(int(cnt.sum()) > 0):
                return False
            rcnt = self.recv_sizes(cnt.astype(np.uint64))
            recv = self.torch.zeros(int(rcnt.sum()), dtype=self.torch.int64)
            self.dist.all_to_all_single(recv, self.torch.from_numpy(pairs.view(np.int64).copy()),
                                        output_split_sizes=[int(x) for x in rcnt], input_split_sizes=[int(x) for x in cnt])
            store.levels_apply(recv.numpy().view(np.uint64))
            return True
        g = self.torch.from_numpy(store.levels_get().astype(np.int32))
        self.dist.all_reduce(g, op=self.dist.ReduceOp.MAX)
        store.levels_set(g.numpy().astype(np.uint32))
        return self.any(changed)


    def kahn_exchange(self, store):
        """One Kahn wave's exchange: every store's outbox to its destinations (all-to-all), the received READYs into the
        inbox; returns whether any store sent anything (the counts all-to-all already tells every store what it gets;
        one all-reduce of the sent totals ends the waves on every store together).  With kahn_slot, at most that many
        READYs per destination leave per wave, the rest the next waves (levels ride in the READYs)."""
        cnt, msgs = store.kahn_outbox()
        if self.kahn_slot is not None:
            world = len(cnt)
            if self._backlog is None or len(self._backlog) != world:
                self._backlog = [np.zeros(0, np.uint64) for _ in range(world)]
            o = np.concatenate([[0], np.cumsum(cnt.astype(np.int64))])
            send = []
            for d in range(world):
                q = np.concatenate([self._backlog[d], msgs[o[d]:o[d + 1]]])
                send.append(q[:self.kahn_slot])
                self._backlog[d] = q[self.kahn_slot:]
            cnt = np.array([len(x) for x in send], np.uint32)
            msgs = np.concatenate(send) if send else np.zeros(0, np.uint64)
        if not self.any(int(cnt.sum()) > 0):
            self._backlog = None
            return False
        rcnt = self.recv_sizes(cnt.astype(np.uint64))
        recv = self.torch.zeros(int(rcnt.sum()), dtype=self.torch.int64)
        self.dist.all_to_all_single(recv, self.torch.from_numpy(msgs.view(np.int64).copy()),
                                    output_split_sizes=[int(x) for x in rcnt], input_split_sizes=[int(x) for x in cnt])
        store.kahn_inbox(recv.numpy().view(np.uint64))
        return True


class RcclUnavailable(RuntimeError):
    """RCCL cannot be used by this group (decided identically on every rank, before any collective RCCL call)."""


class RcclTransport(GlooTransport):
    """Blobs and level arrays move over RCCL (grouped ncclSend/ncclRecv all-to-all, ncclAllReduce, on
    device buffers over xGMI); the gloo group carries the unique id, the byte counts and one scalar per
    level round.

    ncclCommInitRank is collective: a rank that fails before or inside it would leave its peers blocked in it.
    So the ranks first agree over gloo that RCCL is usable — every rank on a distinct (host, device) (RCCL
    refuses two ranks on one GPU) and rank 0 produced a unique id — and raise RcclUnavailable together
    otherwise; after the init an all-reduce(min) of the outcome makes a failure on any rank everyone's."""

    name = "rccl"

    def __init__(self, dist, store, rank, world):
        super().__init__(dist)
        import socket
        me = (socket.gethostname(), int(store.eng.device))
        everyone = [None] * world
        dist.all_gather_object(everyone, me)
        if len(set(everyone)) != world:
            raise RcclUnavailable("ranks share a GPU: %s" % (everyone,))
        uid = None
        if rank == 0:
            try:
                uid = unique_id()
            except engine.AccordDepsError:
                uid = None
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        if obj[0] is None:
            raise RcclUnavailable("ncclGetUniqueId failed on rank 0")
        err = None
        try:
            store.comm_init(world, rank, obj[0])
        except engine.AccordDepsError as e:
            err = e
        if not self.all_ok(err is None):
            if err is None:            # this rank's init succeeded, a peer's did not: drop the communicator
                store.comm_destroy()
            raise RcclUnavailable("ncclCommInitRank failed on some rank%s" % (": %s" % err if err else ""))

    def all_ok(self, ok):
        t = self.torch.tensor([1 if ok else 0], dtype=self.torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return bool(t.item())

    def exchange_blobs(self, store):
        sizes = store.export()
        store.alltoall(self.recv_sizes(sizes))

    def gather_levels(self, store):
        store.level_edges_compute()
        return store.levels_gather()       # counts all-gather + grouped edge send/recv over RCCL, then the solve

    def allreduce_levels(self, store, changed):
        if store.delta:
            return store.levels_exchange()   # counts all-gather + pair send/recv, all over RCCL
        return store.levels_allreduce()      # the round flags ride in the same RCCL all-reduce

    # Kahn waves: ad_shard_kahn_run (fixed slots, no host synchronisation between waves) unless kahn_run_loop is False
    kahn_run_loop = True
    kahn_slot, kahn_check_every, kahn_lag = 0, 4, 2

    def kahn_run(self, store, wave_cap=None):
        return store.kahn_run(self.kahn_slot or 0, self.kahn_check_every, self.kahn_lag,
                              wave_cap if wave_cap is not None else 1 << 16)

    def kahn_exchange(self, store):
        return store.kahn_exchange()         # counts all-gather (one host sync per wave), grouped send/recv over RCCL


class LevelsNotConverged(RuntimeError):
    """The distributed level rounds hit their cap while some store still raised a level: the levels are not
    final and must not be reported (every store raises it in the same round: the flag is all-reduced)."""


AUTO_ROUND_CAP = 128


def run_store(store, transport, max_rounds=1 << 16, timings=None, levels="auto", round_cap=AUTO_ROUND_CAP):
    """The per-store protocol after load(): returns the number of level exchanges (waves / rounds).
    levels="kahn": distributed Kahn waves (run_levels_kahn; holder masks needed): per txn one READY and one RELEASE
      message per holder over the whole batch, each store touching only its own constraint edges.
    levels="rounds": the per-round delta (holders set) / dense exchange, each store relaxing only its own key chains;
      raises LevelsNotConverged if the rounds reach max_rounds while levels are still changing.
    levels="gather": one exchange of every store's constraint edges, every store solving their union (returns 1).
    levels="auto" (default): the Kahn waves while the graph is shallow (at most round_cap waves: C5 takes ~60),
      else -- every store sees the same global release flag, so all switch together -- the one-exchange gather for
      deep graphs (C3-like hot keys: ~10^5 levels, one wave each); without holder masks the gather.  Returns
      round_cap + 1 when it fell back.
    timings (dict, optional) accumulates wall seconds per phase (each phase ends synchronised)."""
    import time
    clock = time.perf_counter
    t = [clock()]

    def lap(name):
        now = clock()
        if timings is not None:
            timings[name] = timings.get(name, 0.0) + now - t[0]
        t[0] = now

    store.preaccept()
    lap("deps")
    transport.exchange_blobs(store)
    lap("exchange")
    store.merge()
    lap("merge")
    if levels == "auto":
        if store.delta:
            return run_levels_auto(store, transport, round_cap, lap)
        levels = "gather"
    if levels == "gather":
        store.depth = transport.gather_levels(store)
        store.levels_via = "gather"
        lap("levels")
        return 1
    if levels == "kahn":
        return run_levels_kahn(store, transport, None, lap)
    return run_levels(store, transport, max_rounds, lap)


def run_levels_auto(store, transport, round_cap=AUTO_ROUND_CAP, lap=None):
    """levels="auto" of run_store: the Kahn waves, or -- when the graph is deeper than round_cap waves (every store
    sees the same global release flag, so all switch together) -- the one-exchange gather, which recomputes the
    levels from every store's constraint edges.  Returns the waves, or round_cap + 1 after the fallback."""
    lap = lap or (lambda name: None)
    # the previous batch's depth on this store (every store agrees: one all-reduce per batch): a deep graph goes
    # straight to the gather instead of spending round_cap waves to find out again
    if transport.any(getattr(store, "depth", 0) > round_cap):
        store.depth = transport.gather_levels(store)
        store.levels_via = "gather"
        lap("levels_gather")
        return round_cap + 1
    try:
        return run_levels_kahn(store, transport, round_cap, lap)
    except LevelsNotConverged:
        store.depth = transport.gather_levels(store)
        store.levels_via = "gather"
        lap("levels_gather")
        return round_cap + 1


def run_levels_kahn(store, transport, wave_cap=None, lap=None):
    """Distributed Kahn waves (ad_shard_kahn_*, csrc/kahn_shard_kernels.h): the READYs of the rows whose local
    predecessors are all released go to every holder of their txn with a level bound; every holder releases the txns all
    their holders reported (at the greatest bound) and frees their successors, whose READYs form the next wave.  Over
    RCCL the store runs the whole loop itself (ad_shard_kahn_run: fixed slots, no host synchronisation between waves);
    otherwise one exchange per wave until an exchange in which no store sent anything.  Raises LevelsNotConverged past
    wave_cap waves (all stores together).  Sets store.depth and store.kahn_bytes (8 B per message sent to another
    store); returns the exchanges (waves + 1 for the per-wave loop: the final, empty exchange)."""
    lap = lap or (lambda name: None)
    store.kahn_begin()
    lap("levels_local")
    if getattr(transport, "kahn_run_loop", False):
        try:
            # (a bounded slot spreads a wide level over several waves: the cap on waves is 4x the cap on levels)
            waves = transport.kahn_run(store, None if wave_cap is None else 4 * wave_cap)
        except LevelsNotConverged:
            store.kahn_finish()
            raise
        exchanges = waves
    else:
        level = 0
        while transport.kahn_exchange(store):
            store.kahn_step(level)
            level += 1
            if wave_cap is not None and level >= wave_cap:
                store.kahn_finish()
                raise LevelsNotConverged("Kahn waves still releasing after %d waves" % level)
        exchanges = level + 1
    unreleased = store.kahn_finish()
    lap("levels_waves")
    if unreleased:
        raise engine.AccordDepsError(abi.AD_ERR_ARGUMENT, "Kahn waves: %d rows never released (a cycle)" % unreleased)
    # the batch's depth: the greatest level over every store (one all-reduce per batch)
    store.depth = transport.max_u64(store.kahn_depth()) if hasattr(store, "kahn_depth") else exchanges - 1
    store.kahn_bytes = 8 * store.kahn_sent()
    store.levels_via = "kahn"
    return exchanges


def run_levels(store, transport, max_rounds=1 << 16, lap=None):
    """The distributed level fixpoint: local rounds over the store's own key chains, then the
    transport's exchange (delta pairs to the peers holding each raised txn, or the dense all-reduce), until no
    store has anything left to tell another.  Returns the number of rounds."""
    lap = lap or (lambda name: None)
    changed = store.levels_round(True)
    lap("levels_local")
    rounds = 1
    while True:
        any_changed = transport.allreduce_levels(store, changed)
        lap("levels_exchange")
        if not any_changed:
            break
        if rounds >= max_rounds:
            raise LevelsNotConverged("distributed execution levels still changing after %d rounds" % rounds)
        changed = store.levels_round(False)
        lap("levels_local")
        rounds += 1
    return rounds


class LocalTransport:
    """Several stores in one process (tests): the same protocol with in-process exchange."""

    @staticmethod
    def run(stores, max_rounds=1 << 16, levels="gather", deps="preaccept", gq=None, timings=None, kahn_slot=None):
        """deps: "preaccept", "accept" (gq: the global query positions, query_positions) or "ephemeral";
        kahn_slot: the Kahn waves' READYs per (source, destination) and wave (None: all);
        levels None: stop after the home merge.  timings (dict): seconds per phase, summed over the stores (the
        stores run one after another in this process: each phase's sum is what S GPUs would spend in parallel,
        times S)."""
        import time
        t = [time.perf_counter()]

        def lap(name):
            now = time.perf_counter()
            if timings is not None:
                timings[name] = timings.get(name, 0.0) + now - t[0]
            t[0] = now
        for s in stores:
            if deps == "preaccept":
                s.preaccept()
            else:
                s.accept(None if gq is None else gq[s.gid], bound_max=deps == "ephemeral")
        lap("deps")
        sizes = [s.export() for s in stores]
        bufs = [s.send_buffer() for s in stores]
        lap("export")
        offs = [np.concatenate([[0], np.cumsum(z)]).astype(np.int64) for z in sizes]
        for d, s in enumerate(stores):
            parts = [bufs[k][offs[k][d]:offs[k][d + 1]] for k in range(len(stores))]
            s.import_host(np.concatenate(parts) if parts else np.zeros(0, np.uint8),
                          np.array([sizes[k][d] for k in range(len(stores))], np.uint64))
            lap("exchange")
            s.merge()
            lap("home_merge")
        if levels is None:
            return 0
        fell_back = False
        if levels == "kahn":
            r = LocalTransport._kahn(stores, None, kahn_slot)
            lap("level_waves")
            return r
        if levels == "auto":
            if all(s.delta for s in stores):
                try:
                    r = LocalTransport._kahn(stores, AUTO_ROUND_CAP, kahn_slot)
                    lap("level_waves")
                    return r
                except LevelsNotConverged:
                    lap("level_waves")
            fell_back = True
            levels = "gather"
        if levels == "gather":
            edges = np.concatenate([s.level_edges() for s in stores])
            lap("level_edges")
            if timings is not None:
                timings["level_edges_count"] = int(len(edges))
            for s in stores:
                s.depth = s.levels_solve(edges)
            lap("level_solve")
            return AUTO_ROUND_CAP + 1 if fell_back else 1     # as run_levels_auto reports the fallback
        r = LocalTransport._rounds(stores, max_rounds)
        lap("level_rounds")
        return r

    @staticmethod
    def _kahn(stores, wave_cap, slot=None):
        """run_levels_kahn for stores in one process: each wave's outboxes routed to the inboxes (slot: at most that
        many READYs per (source, destination) and wave, the rest later, as ad_shard_kahn_run's fixed slots)."""
        W = len(stores)
        backlog = [[np.zeros(0, np.uint64) for _ in range(W)] for _ in range(W)]

        def route():
            moved = False
            inbox = [[] for _ in range(W)]
            for k, s in enumerate(stores):
                cnt, msgs = s.kahn_outbox()
                o = np.concatenate([[0], np.cumsum(cnt.astype(np.int64))])
                for d in range(W):
                    q = np.concatenate([backlog[k][d], msgs[o[d]:o[d + 1]]])
                    n = len(q) if slot is None else min(slot, len(q))
                    inbox[d].append(q[:n])
                    backlog[k][d] = q[n:]
                    moved |= n > 0
            if not moved:
                return False
            for d, s in enumerate(stores):
                s.kahn_inbox(np.concatenate(inbox[d]))
            return True
        for s in stores:
            s.kahn_begin()
        level = 0
        while route():
            for s in stores:
                s.kahn_step(level)
            level += 1
            if wave_cap is not None and level >= wave_cap:
                for s in stores:
                    s.kahn_finish()
                raise LevelsNotConverged("Kahn waves still releasing after %d waves" % level)
        if any(s.kahn_finish() for s in stores):
            raise engine.AccordDepsError(abi.AD_ERR_ARGUMENT, "Kahn waves: rows never released (a cycle)")
        depth = max(s.kahn_depth() for s in stores)
        for s in stores:
            s.depth = depth
            s.kahn_bytes = 8 * s.kahn_sent()
        return level + 1

    @staticmethod
    def _rounds(stores, max_rounds):
        changed = [s.levels_round(True) for s in stores]
        rounds = 1
        while True:
            if all(s.delta for s in stores):
                out = [s.level_deltas() for s in stores]
                for d, s in enumerate(stores):
                    parts = []
                    for k, (cnt, pairs) in enumerate(out):
                        o = np.concatenate([[0], np.cumsum(cnt.astype(np.int64))])
                        parts.append(pairs[o[d]:o[d + 1]])
                    s.levels_apply(np.concatenate(parts))
                if not any(int(c.sum()) for c, _ in out):
                    break
            else:
                g = np.maximum.reduce([s.levels_get() for s in stores])
                for s in stores:
                    s.levels_set(g)
                if not any(changed):
                    break
            if rounds >= max_rounds:
                raise LevelsNotConverged("distributed execution levels still changing after %d rounds" % rounds)
            changed = [s.levels_round(False) for s in stores]
            rounds += 1
        return rounds
