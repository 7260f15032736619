"""The cross-store fragment blob codec (accord_amd.blob) on the CPU: round trips, the export rule (rows homed
at the destination with any deps, TxnIds as global ranks) on oracle-resolved fragments, and rejection of
malformed blobs.  tests/test_gpu_sharding.py pins the codec to the engine's own bytes."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, blob, sharding, workload


def _local_fragments(b, lo, hi, replicas=2):
    cfg = abi.make_config(0, replicas, 0.0, 7)
    local, gid, home = sharding.slice_for_shard(b, lo, hi)
    res = O.OracleResult(local, cfg, O.FLAG_MERGE)
    csrs = [res.deps(v, c) for v in range(replicas) for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY)]
    return local, gid, csrs


def test_encode_decode_round_trip():
    b = workload.generate(800, keys_per_txn=3, keyspace=300, seed=3)
    local, gid, csrs = _local_fragments(b, 0, 150)
    glob = [abi.Csr(c.key_off, c.keys, c.k2t_off, c.k2t, c.txn_off, gid[c.txns].astype(np.uint32)) for c in csrs]
    buf = blob.encode(gid, glob)
    assert buf.nbytes % 8 == 0
    g2, back = blob.decode(buf)
    assert np.array_equal(g2, gid)
    for a, c in zip(back, glob):
        assert a.equal(c)


def test_export_rows_by_home_store():
    b = workload.generate(1200, keys_per_txn=4, keyspace=500, seed=5)
    world = 3
    bounds = sharding.even_bounds(0, 500, world)
    hs = sharding.home_stores(b, bounds)
    local, gid, csrs = _local_fragments(b, bounds[1], bounds[2])
    buf, sizes = blob.export(gid, hs[gid], csrs, world)
    assert int(sizes.sum()) == buf.nbytes
    parts = blob.split(buf, sizes)
    has = np.zeros(len(gid), bool)
    for c in csrs:
        has |= np.diff(c.txn_off) > 0
    for d, (g, sub) in enumerate(parts):
        rows = np.nonzero(has & (hs[gid] == d))[0]
        assert np.array_equal(g, gid[rows])
        for c, s in zip(csrs, sub):
            for k, r in enumerate(rows):
                ks, tx, m = c.txn(r)
                ks2, tx2, m2 = s.txn(k)
                assert np.array_equal(ks, ks2) and np.array_equal(gid[tx], tx2) and np.array_equal(m, m2)
    assert sum(len(p[0]) for p in parts) == int(has.sum())


def test_empty_and_malformed():
    buf = blob.encode(np.zeros(0, np.uint32), [abi.Csr(np.zeros(1, np.uint32), np.zeros(0, np.uint64),
                                                       np.zeros(1, np.uint32), np.zeros(0, np.int32),
                                                       np.zeros(1, np.uint32), np.zeros(0, np.uint32))] * 2)
    g, c = blob.decode(buf)
    assert len(g) == 0 and len(c) == 2
    with pytest.raises(ValueError):
        blob.decode(buf[:16])
    bad = buf.copy()
    bad[0] ^= 1
    with pytest.raises(ValueError):
        blob.decode(bad)
    with pytest.raises(ValueError):
        blob.decode(buf[:-8] if buf.nbytes > 48 else buf[:40])
