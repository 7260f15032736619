"""Range txns across key-range stores, on the CPU ("Range txns are split at shard boundaries,
exactly as range commands are sliced to store ranges", impl/InMemoryCommandStore.java:758-761).

The host slicing (sharding.slice_for_shard / home_stores / holder_masks / presplit) and the claim the GPU
sharding tests rest on: the stores' PartialDeps, resolved independently on their slices with global arrival
ranks and united per txn (PreAccept.reduce -> PartialDeps.with, messages/PreAccept.java:141-156), equal the
unsharded deps of the batch whose ranges are cut at the store boundaries (presplit) — checked here with the
oracle on both sides, every view and class, and the merged Deps.
"""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, blob, sharding, workload
from batchkit import deps_of


def mixed(n, keyspace, seed, width=20000, range_frac=0.15):
    return workload.generate(n, 3, keyspace, "uniform", range_frac=range_frac, range_width_max=width, seed=seed)


def test_presplit_pieces_are_store_slices():
    b = mixed(2000, 100_000, 3)
    bounds = sharding.even_bounds(0, 100_000, 4)
    ps = sharding.presplit(b, bounds)
    ro, pro = b["range_off"].astype(np.int64), ps["range_off"].astype(np.int64)
    crossing = 0
    for t in range(b["n"]):
        pieces = list(zip(ps["range_start"][pro[t]:pro[t + 1]].tolist(), ps["range_end"][pro[t]:pro[t + 1]].tolist()))
        want = []
        for s, e in zip(b["range_start"][ro[t]:ro[t + 1]].tolist(), b["range_end"][ro[t]:ro[t + 1]].tolist()):
            cut = [s] + [int(x) - 1 for x in bounds[1:-1] if s < int(x) - 1 < e] + [e]
            want += list(zip(cut[:-1], cut[1:]))
            crossing += len(cut) > 2
        assert pieces == want
        # sorted, disjoint (touching at most), non-empty
        assert all(p[0] < p[1] for p in pieces) and all(a[1] <= c[0] for a, c in zip(pieces, pieces[1:]))
    assert crossing > 20
    # every piece lies in one store; the union of the stores' slices is the presplit batch
    for k in range(4):
        local, gid, home = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
        lo, hi = int(bounds[k]), int(bounds[k + 1])
        assert (local["range_start"] >= max(lo - 1, 0)).all() and (local["range_end"] <= hi - 1).all()
        lro = local["range_off"].astype(np.int64)
        for r, g in enumerate(gid):
            got = list(zip(local["range_start"][lro[r]:lro[r + 1]].tolist(), local["range_end"][lro[r]:lro[r + 1]].tolist()))
            allp = list(zip(ps["range_start"][pro[g]:pro[g + 1]].tolist(), ps["range_end"][pro[g]:pro[g + 1]].tolist()))
            assert got == [p for p in allp if p[0] >= max(lo - 1, 0) and p[1] <= hi - 1]


def test_homes_and_holders_with_ranges():
    b = mixed(3000, 100_000, 4)
    bounds = sharding.even_bounds(0, 100_000, 3)
    hs = sharding.home_stores(b, bounds)
    masks = sharding.holder_masks(b, bounds)
    held = np.zeros(b["n"], np.uint8)
    for k in range(3):
        local, gid, home = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
        held[gid] |= np.uint8(1 << k)
        assert np.array_equal(home, (hs[gid] == k).astype(np.uint8))
    touched = (np.diff(b["key_off"]) > 0) | (np.diff(b["range_off"]) > 0)
    assert np.array_equal(held[touched], masks[touched])
    # a txn's home holds it
    assert ((masks[touched] >> hs[touched]) & 1).all()


def _union(rels):
    out = {}
    for r in rels:
        for k, v in r.items():
            out[k] = sorted(set(out.get(k, [])) | set(v))
    return out


@pytest.mark.parametrize("shards,window,drop,seed", [(2, 32, 0.1, 5), (3, 8, 0.3, 6), (4, 0, 0.0, 7)])
def test_stores_united_equal_presplit_unsharded(shards, window, drop, seed):
    n, ks = 2500, 60_000
    kinds = np.random.default_rng(seed).choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT], size=n, p=[0.45, 0.45, 0.1])
    b = workload.generate(n, 3, ks, "uniform", range_frac=0.2, range_width_max=15000, kinds=kinds, seed=seed)
    bounds = sharding.even_bounds(0, ks, shards)
    cfg = abi.make_config(window, 3, drop, 0xACC0D1)
    want = O.OracleResult(sharding.presplit(b, bounds), cfg, O.FLAG_MERGE)
    got = {}     # (view or 'merged', class) -> per global txn list of relations
    for k in range(shards):
        local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
        res = O.OracleResult(local, cfg, O.FLAG_MERGE, gid=gid)
        for c in range(3):
            for v in list(range(3)) + ["m"]:
                csr = res.merged(c) if v == "m" else res.deps(v, c)
                for r, g in enumerate(gid):
                    rel = {key: [int(gid[x]) for x in txs] for key, txs in deps_of(csr, r).items()}
                    got.setdefault((v, c), {}).setdefault(int(g), []).append(rel)
    nonempty = 0
    for c in range(3):
        for v in list(range(3)) + ["m"]:
            csr = want.merged(c) if v == "m" else want.deps(v, c)
            for t in range(n):
                w = deps_of(csr, t)
                g = _union(got.get((v, c), {}).get(t, []))
                assert g == w, "view %s class %d txn %d" % (v, c, t)
                nonempty += bool(w) and c == abi.CLASS_RANGE
    assert nonempty > 100


def test_blob_codec_carries_range_classes():
    b = mixed(800, 50_000, 9)
    bounds = sharding.even_bounds(0, 50_000, 2)
    local, gid, _ = sharding.slice_for_shard(b, bounds[0], bounds[1])
    res = O.OracleResult(local, abi.make_config(16, 2, 0.1, 1), O.FLAG_MERGE, gid=gid)
    csrs = [res.deps(v, c) for v in range(2) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)] + [res.deps(v, abi.CLASS_RANGE) for v in range(2)]
    hs = sharding.home_stores(b, bounds)[gid]
    buf, sizes = blob.export(gid, hs, csrs, 2)
    parts = blob.split(buf, sizes)
    assert sum(int(np.diff(p[1][4].txn_off).sum()) for p in parts) > 0
    for d, (g, back) in enumerate(parts):
        assert len(back) == 6 and [c.is_range for c in back] == [False] * 4 + [True] * 2
        rows = np.searchsorted(gid, g)
        for c, (x, y) in enumerate(zip(back, csrs)):
            for i, r in enumerate(rows):
                assert deps_of(x, i) == {k: [int(gid[t]) for t in v] for k, v in deps_of(y, int(r)).items()}
    # header word: nvc | nr << 16
    h = buf[:24].view(np.uint64)
    assert int(h[2]) == 6 | (2 << 16)


def test_clip_edges():
    # (start, end] against the store owning keys [lo, hi): boundary keys belong to exactly one store
    rs = np.array([0, 9, 10, 5, 19, 0], np.uint64)
    re = np.array([10, 10, 11, 25, 20, 2**64 - 2], np.uint64)
    bounds = np.array([0, 10, 20, 2**64 - 1], np.uint64)
    pieces = []
    for k in range(3):
        s, e, keep = sharding._clip_ranges(rs, re, bounds[k], bounds[k + 1])
        pieces.append([(int(a), int(b)) if m else None for a, b, m in zip(s, e, keep)])
    # keys 1..10 of (0, 10]: 1..9 in store 0, 10 in store 1
    assert pieces[0][0] == (0, 9) and pieces[1][0] == (9, 10) and pieces[2][0] is None
    assert pieces[0][1] is None and pieces[1][1] == (9, 10)           # (9, 10] = key 10 only
    assert pieces[1][2] == (10, 11) and pieces[0][2] is None
    assert pieces[0][3] == (5, 9) and pieces[1][3] == (9, 19) and pieces[2][3] == (19, 25)
    assert pieces[1][4] is None and pieces[2][4] == (19, 20)          # (19, 20] = key 20, store 2
    assert pieces[2][5] == (19, 2**64 - 2)
    # every covered key lands in exactly one piece
    for t in range(5):
        keys = set(range(int(rs[t]) + 1, int(re[t]) + 1))
        got = set()
        for k in range(3):
            if pieces[k][t]:
                a, b = pieces[k][t]
                part = set(range(a + 1, b + 1))
                assert not (got & part)
                assert all(int(bounds[k]) <= x < int(bounds[k + 1]) for x in part)
                got |= part
        assert got == keys
