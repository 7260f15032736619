"""Seeded synthetic transaction batches (SURVEY §8d / BASELINE.md §2).

A batch is a dict of numpy arrays in the ad_batch layout (include/accord_deps.h):

* TxnIds: epoch, hlc strictly increasing with random gaps 1..8, node in [1, nodes], flags =
  kind << 1 | domain (TxnId.java:132-165); msb = epoch << 15 | hlc >>> 48, lsb = hlc << 16 | flags
  (Timestamp.java:81-89).  Arrival order == TxnId order (the batch is CommandsForKey.byId order).
* executeAt: == TxnId on the fast path; with probability ``slow_frac`` bumped by 1..``bump_max``
  hlc and witnessed by a replica node id (101..103) so that every executeAt is a distinct Timestamp.
* Keys: ``keys_per_txn`` distinct keys per key txn, ascending (Keys is a sorted set), uniform or Zipf(s) over ``keyspace`` (Zipf ranks are
  scattered over the key space by an affine bijection so hot keys do not cluster in one shard).
* Kinds: key txns Write with probability ``write_frac`` else Read (BurnTest.java:161-164); range
  txns (``range_frac``) carry 1-2 disjoint ranges of width U[1, range_width_max] (BurnTest.randomRange
  :242-258) and kind ``range_kind``.
* status: the final InternalStatus (APPLIED) each txn has once it leaves the in-flight window.

The configs of BASELINE.json are exposed as ``config(name)``.
"""
import numpy as np

from . import abi

SEEDS = {"C2": 0xACC0D1, "C3": 0xACC0D2, "C4": 0xACC0D3, "C5": 0xACC0D4}


def _hlc_to_bits(epoch, hlc, flags):
    hlc = hlc.astype(np.uint64)
    msb = (np.uint64(epoch) << np.uint64(15)) | (hlc >> np.uint64(48))
    lsb = (hlc << np.uint64(16)) | flags.astype(np.uint64)
    return msb, lsb


def _distinct_rows(rng, draw, n, k):
    """n rows of k distinct values; ``draw(m)`` returns m candidates."""
    out = draw(n * k).reshape(n, k)
    while True:
        s = np.sort(out, axis=1)
        bad = np.nonzero((s[:, 1:] == s[:, :-1]).any(axis=1))[0] if k > 1 else np.zeros(0, np.int64)
        if len(bad) == 0:
            return out
        out[bad] = draw(len(bad) * k).reshape(len(bad), k)


class _Zipf:
    def __init__(self, keyspace, s):
        r = np.arange(1, keyspace + 1, dtype=np.float64)
        cdf = np.cumsum(r ** -s)
        self.cdf = cdf / cdf[-1]
        self.keyspace = keyspace
        # affine bijection rank -> key id (a coprime with keyspace)
        a = 2654435761 % keyspace
        while np.gcd(a, keyspace) != 1:
            a += 1
        self.a, self.b = a, 7919 % keyspace

    def __call__(self, rng, m):
        ranks = np.searchsorted(self.cdf, rng.random(m), side="right")
        ranks = np.minimum(ranks, self.keyspace - 1).astype(np.int64)
        return ((ranks * self.a + self.b) % self.keyspace).astype(np.uint64)


_ZIPF_CACHE = {}


def generate(n, keys_per_txn=4, keyspace=10_000_000, dist="uniform", zipf_s=0.99, write_frac=0.5,
             range_frac=0.0, range_width_max=1 << 13, range_kind=abi.KIND_READ, slow_frac=0.1, bump_max=16,
             nodes=8, epoch=1, seed=0xACC0D1, hlc_start=1_000_000, kinds=None, status=None):
    rng = np.random.default_rng(seed)
    hlc = hlc_start + np.cumsum(rng.integers(1, 9, size=n, dtype=np.int64))
    node = rng.integers(1, nodes + 1, size=n, dtype=np.int64).astype(np.int32)
    is_range = rng.random(n) < range_frac if range_frac > 0 else np.zeros(n, bool)
    if kinds is None:
        kinds = np.where(rng.random(n) < write_frac, abi.KIND_WRITE, abi.KIND_READ).astype(np.int64)
        kinds[is_range] = range_kind
    kinds = np.asarray(kinds, np.int64)
    domain = is_range.astype(np.int64)
    flags = (kinds << 1) | domain
    txn_msb, txn_lsb = _hlc_to_bits(epoch, hlc, flags)

    # executeAt: fast path == TxnId; slow path bumped hlc, replica node id
    slow = rng.random(n) < slow_frac
    bump = rng.integers(1, bump_max + 1, size=n, dtype=np.int64)
    enode = rng.integers(101, 104, size=n, dtype=np.int64).astype(np.int32)
    ehlc = np.where(slow, hlc + bump, hlc)
    # re-draw colliding slow executeAts (same hlc, identity flags, node)
    for _ in range(100):
        sl = np.nonzero(slow)[0]
        key = (ehlc[sl] << 12) ^ ((flags[sl] & 0x1E) << 7) ^ enode[sl]
        _, first = np.unique(key, return_index=True)
        dup = np.setdiff1d(np.arange(len(sl)), first)
        if len(dup) == 0:
            break
        ehlc[sl[dup]] += rng.integers(1, bump_max + 1, size=len(dup))
    exec_msb, exec_lsb = _hlc_to_bits(epoch, ehlc, flags)
    exec_node = np.where(slow, enode, node).astype(np.int32)
    exec_msb = np.where(slow, exec_msb, txn_msb)
    exec_lsb = np.where(slow, exec_lsb, txn_lsb)

    # key footprints
    nkey_txn = int((~is_range).sum())
    if dist == "uniform":
        draw = lambda m: rng.integers(0, keyspace, size=m, dtype=np.int64).astype(np.uint64)  # noqa: E731
    elif dist == "zipf":
        zk = (keyspace, zipf_s)
        if zk not in _ZIPF_CACHE:
            _ZIPF_CACHE[zk] = _Zipf(keyspace, zipf_s)
        z = _ZIPF_CACHE[zk]
        draw = lambda m: z(rng, m)  # noqa: E731
    else:
        raise ValueError(dist)
    kk = _distinct_rows(rng, draw, nkey_txn, keys_per_txn) if nkey_txn else np.zeros((0, keys_per_txn), np.uint64)
    kk = np.sort(kk, axis=1)                   # Keys are a sorted set (primitives/Keys.java)
    cnt = np.where(is_range, 0, keys_per_txn).astype(np.int64)
    key_off = np.zeros(n + 1, np.uint32)
    key_off[1:] = np.cumsum(cnt)
    keys = kk.reshape(-1).astype(np.uint64)

    # range footprints: 1-2 disjoint (start, end] ranges per range txn
    rcnt = np.where(is_range, rng.integers(1, 3, size=n), 0).astype(np.int64)
    range_off = np.zeros(n + 1, np.uint32)
    range_off[1:] = np.cumsum(rcnt)
    nr = int(range_off[-1])
    rs = rng.integers(0, max(1, keyspace - range_width_max - 1), size=nr, dtype=np.int64)
    rw = rng.integers(1, range_width_max + 1, size=nr, dtype=np.int64)
    if nr:
        # make each txn's ranges sorted & disjoint: second range starts after the first ends
        owner = np.repeat(np.arange(n), rcnt)
        second = np.zeros(nr, bool)
        second[1:] = owner[1:] == owner[:-1]
        idx = np.nonzero(second)[0]
        rs[idx] = rs[idx - 1] + rw[idx - 1] + 1 + (rs[idx] % max(1, range_width_max))
    range_start = rs.astype(np.uint64)
    range_end = (rs + rw).astype(np.uint64)

    if status is None:
        status = np.full(n, abi.ST_APPLIED, np.uint8)
    return {
        "n": n, "txn_msb": txn_msb, "txn_lsb": txn_lsb, "txn_node": node,
        "exec_msb": exec_msb.astype(np.uint64), "exec_lsb": exec_lsb.astype(np.uint64), "exec_node": exec_node,
        "status": np.asarray(status, np.uint8), "key_off": key_off, "keys": keys,
        "range_off": range_off if nr else None,
        "range_start": range_start if nr else None, "range_end": range_end if nr else None,
    }


def config(name, n=None, seed=None):
    """BASELINE.json configs (C2..C5) at full or reduced size."""
    if name == "C2":
        return generate(n or 1 << 20, 4, 10_000_000, "uniform", seed=seed or SEEDS["C2"])
    if name == "C3":
        return generate(n or 1 << 20, 4, 10_000_000, "zipf", 0.99, seed=seed or SEEDS["C3"])
    if name == "C4":
        return generate(n or 1 << 22, 4, 10_000_000, "uniform", range_frac=0.1, seed=seed or SEEDS["C4"])
    if name == "C5":
        return generate(n or 1 << 24, 4, 10_000_000, "uniform", seed=seed or SEEDS["C5"])
    raise ValueError(name)


def slice_batch(b, lo, hi):
    """Rows [lo, hi) of a batch (re-based CSR offsets)."""
    out = {"n": hi - lo}
    for f in ("txn_msb", "txn_lsb", "txn_node", "exec_msb", "exec_lsb", "exec_node", "status"):
        out[f] = np.ascontiguousarray(b[f][lo:hi])
    ko = b["key_off"]
    out["key_off"] = (ko[lo:hi + 1] - ko[lo]).astype(np.uint32)
    out["keys"] = np.ascontiguousarray(b["keys"][ko[lo]:ko[hi]])
    if b.get("range_off") is not None:
        ro = b["range_off"]
        out["range_off"] = (ro[lo:hi + 1] - ro[lo]).astype(np.uint32)
        out["range_start"] = np.ascontiguousarray(b["range_start"][ro[lo]:ro[hi]])
        out["range_end"] = np.ascontiguousarray(b["range_end"][ro[lo]:ro[hi]])
    else:
        out["range_off"] = out["range_start"] = out["range_end"] = None
    return out
