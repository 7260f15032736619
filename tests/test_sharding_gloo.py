"""The N>1 path on CPU: two processes over a gloo group (world_size 2, 127.0.0.1).

Each rank slices the batch to its key range (accord_amd.sharding.slice_for_shard), resolves its local batch
with the oracle (the test-only stand-in for the GPU engine; W = 0 and no drops so local ranks and global
ranks give the same answers), packs its fragments in the engine's own blob format (accord_amd.blob.export:
per destination store, the rows homed there with any deps, TxnIds as global ranks — byte-identical to
ad_shard_export, pinned by tests/test_gpu_sharding.py) and moves them with the product transport's
GlooTransport.exchange_blobs (all_to_all_single of the per-destination byte counts, then of the blobs).  Each
store decodes what it received and merges, for its home txns, every store's fragment (PreAccept.reduce =
Deps.with, messages/PreAccept.java:141-156).  The result must equal the unsharded oracle.  The transport's
scalar collectives (max / any) are exercised on the same group.
"""
import os
import socket
import sys

import numpy as np
import torch
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


def _relation(csr, i):
    ks, txns, k2t = csr.txn(i)
    return ks.copy(), txns.copy(), k2t.copy()


def _worker(rank, world, port, n):
    sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from accord_amd import abi, blob, sharding, workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = sharding.GlooTransport(dist)
        assert tr.max_u64(rank * 10 + 3) == (world - 1) * 10 + 3
        assert tr.any(rank == 1) and not tr.any(False)

        b = workload.config("C2", n=n)
        b["keys"] = b["keys"] % np.uint64(20000)                 # denser keys: plenty of cross-shard deps
        ko = b["key_off"]
        for t in range(n):                                        # re-sort / dedupe rows after the fold
            row = np.unique(b["keys"][ko[t]:ko[t + 1]])
            if len(row) != ko[t + 1] - ko[t]:
                row = np.arange(ko[t + 1] - ko[t], dtype=np.uint64) + np.uint64(20000 + 4 * t)
            b["keys"][ko[t]:ko[t + 1]] = np.sort(row)
        cfg = abi.make_config(0, 2, 0.0, 7)
        bounds = sharding.even_bounds(0, 20000, world)
        local, gid, home = sharding.slice_for_shard(b, bounds[rank], bounds[rank + 1])
        res = O.OracleResult(local, cfg, O.FLAG_MERGE)
        vcs = [(v, c) for v in range(2) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)]
        hs = sharding.home_stores(b, bounds)
        store = blob.HostFragmentStore(gid, hs[gid], [res.deps(v, c) for v, c in vcs], world)
        tr.exchange_blobs(store)                       # the product path: byte counts, then the blobs
        assert store.received is not None and len(store.received) == world
        homes = gid[home.astype(bool)]
        assert len(homes) > 0
        for src_gid, _ in store.received:              # every received row is homed here
            assert np.isin(src_gid, homes).all()

        ref = O.OracleResult(b, cfg, O.FLAG_MERGE)
        rowpos = [{int(g): i for i, g in enumerate(src_gid)} for src_gid, _ in store.received]
        for k, (v, c) in enumerate(vcs):
            want = ref.deps(v, c)
            for g in homes:
                acc = O.EMPTY_RELATION
                for s, (_, csrs) in enumerate(store.received):
                    r = rowpos[s].get(int(g))
                    if r is not None:
                        acc = O.union_relation(acc, _relation(csrs[k], r))
                wk, wt, wm = want.txn(int(g))
                assert np.array_equal(acc[0], wk) and np.array_equal(acc[1], wt) and np.array_equal(acc[2], wm), \
                    "rank %d view %d class %d txn %d" % (rank, v, c, g)
        # every txn is homed exactly once across the stores
        counts = torch.zeros(n, dtype=torch.int64)
        counts[torch.from_numpy(homes.astype(np.int64))] = 1
        dist.all_reduce(counts)
        assert (counts.numpy() == 1).all()
    finally:
        dist.destroy_process_group()


def test_two_stores_over_gloo_equal_unsharded():
    mp.spawn(_worker, args=(2, _free_port(), 1500), nprocs=2, join=True)
