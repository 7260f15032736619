"""Host codec of the cross-store fragment blob (the bytes ad_shard_export writes and ad_shard_import_host /
ad_shard_alltoall read; engine.hip blob_layout, shard_kernels.h k_export_fill).

PreAccept.reduce across CommandStores (messages/PreAccept.java:141-156) needs, at each txn's home store, the
PartialDeps every other store computed for it.  A store packs, per destination store, the rows of the local
txns homed there that have any deps, with TxnIds rewritten to global arrival ranks.  One blob per destination:

    u64 header[3 + 3*nvc] = {MAGIC, rows, nvc | nr << 16, per (view, class) vc: (keys, keysToTxnIds, TxnIds) counts}
    u32 gid[rows]                                      global rank of each row (ascending)
    per vc:  u32 key_off[rows+1]  u32 k2t_off[rows+1]  u32 ent_off[rows+1]  u32 tcnt[rows]
             u64 keys[keys * w]   i32 k2t[k2t]         u32 txns[TxnIds]
    every section 8-byte aligned, padding zero; vc = view * 2 + class (keyDeps, directKeyDeps) for vc < 2R, then,
    when the store holds range txns, nr = R RangeDeps classes (one per view) whose keys are (start, end] ranges
    (w = 2 words; RangeDeps.SerializerSupport.create's Range[], primitives/RangeDeps.java:100-103)

The per-row arrays are exactly KeyDeps.SerializerSupport.create's arguments (primitives/KeyDeps.java:69-72)
per txn; ent_off is compact (ent_off[i+1] - ent_off[i] == tcnt[i]).  A host that resolves a store's fragments
elsewhere (or a test) produces byte-identical blobs with ``export`` and reads received ones with ``decode``;
tests/test_gpu_sharding.py pins this codec to the engine's own bytes.
"""
import numpy as np

from . import abi

MAGIC = 0xAD5EC0DF


def _align8(x):
    return (x + 7) & ~7


def layout(rows, nvc, counts, nr=0):
    """Byte offsets of the sections of one blob and its total size.  counts[vc] = (keys, k2t, txns); the last nr
    classes are RangeDeps (two words per key).  Returns (gid offset, [vc][7] section offsets, total bytes) —
    engine.hip blob_layout."""
    off = _align8((3 + 3 * nvc) * 8)
    gid_off = off
    off = _align8(off + rows * 4)
    secs = []
    for c in range(nvc):
        nk, nm, nt = counts[c]
        w = 2 if c >= nvc - nr else 1
        sizes = ((rows + 1) * 4, (rows + 1) * 4, (rows + 1) * 4, rows * 4, nk * 8 * w, nm * 4, nt * 4)
        s = []
        for z in sizes:
            s.append(off)
            off = _align8(off + z)
        secs.append(s)
    return gid_off, secs, off


def _rows_of(csr, rows):
    """The sub-CSR of `rows` (ascending row indices) of a compacted abi.Csr, vectorised."""
    rows = np.asarray(rows, np.int64)

    def take(off, data, width=1):
        lo, hi = off[rows].astype(np.int64), off[rows + 1].astype(np.int64)
        cnt = hi - lo
        new_off = np.zeros(len(rows) + 1, np.uint32)
        new_off[1:] = np.cumsum(cnt)
        total = int(new_off[-1])
        if total == 0:
            return new_off, data[:0]
        idx = np.repeat(lo - new_off[:-1].astype(np.int64), cnt) + np.arange(total, dtype=np.int64)
        if width == 1:
            return new_off, data[idx]
        return new_off, data.reshape(-1, width)[idx].reshape(-1)

    ko, keys = take(csr.key_off, csr.keys, 2 if csr.is_range else 1)
    mo, k2t = take(csr.k2t_off, csr.k2t)
    to, txns = take(csr.txn_off, csr.txns)
    return abi.Csr(ko, keys, mo, k2t, to, txns, csr.is_range)


def encode(gid, csrs):
    """One blob: rows with global ranks `gid` (ascending), csrs[vc] = abi.Csr over exactly those rows with
    TxnIds already global.  Returns np.uint8 bytes (zero padding, as the engine's memset send buffer)."""
    gid = np.ascontiguousarray(gid, np.uint32)
    rows, nvc = len(gid), len(csrs)
    nr = sum(1 for c in csrs if c.is_range)
    if any(c.is_range for c in csrs[:nvc - nr]):
        raise ValueError("RangeDeps classes go last")
    counts = [(int(c.key_off[-1]), int(c.k2t_off[-1]), int(c.txn_off[-1])) for c in csrs]
    gid_off, secs, total = layout(rows, nvc, counts, nr)
    buf = np.zeros(total, np.uint8)
    hdr = np.zeros(3 + 3 * nvc, np.uint64)
    hdr[0], hdr[1], hdr[2] = MAGIC, rows, nvc | (nr << 16)
    for c, (nk, nm, nt) in enumerate(counts):
        hdr[3 + 3 * c:6 + 3 * c] = (nk, nm, nt)
    buf[:hdr.nbytes] = hdr.view(np.uint8)

    def put(off, arr):
        b = np.ascontiguousarray(arr).view(np.uint8)
        buf[off:off + b.nbytes] = b

    put(gid_off, gid)
    for c, csr in enumerate(csrs):
        s = secs[c]
        tcnt = np.diff(csr.txn_off).astype(np.uint32)
        put(s[0], csr.key_off.astype(np.uint32))
        put(s[1], csr.k2t_off.astype(np.uint32))
        put(s[2], csr.txn_off.astype(np.uint32))
        put(s[3], tcnt)
        put(s[4], csr.keys.astype(np.uint64))
        put(s[5], csr.k2t.astype(np.int32))
        put(s[6], csr.txns.astype(np.uint32))
    return buf


def decode(buf):
    """(gid, [abi.Csr] * nvc) of one blob; raises ValueError on a malformed blob (the checks of
    engine.hip parse_recv)."""
    buf = np.ascontiguousarray(buf, np.uint8)
    if buf.nbytes < 24:
        raise ValueError("shard blob truncated")
    h0 = buf[:24].view(np.uint64)
    if int(h0[0]) != MAGIC:
        raise ValueError("shard blob: bad magic")
    rows, nvc, nr = int(h0[1]), int(h0[2]) & 0xFFFF, int(h0[2]) >> 16
    if nr > nvc:
        raise ValueError("shard blob: bad class counts")
    if buf.nbytes < (3 + 3 * nvc) * 8:
        raise ValueError("shard blob truncated")
    hdr = buf[:(3 + 3 * nvc) * 8].view(np.uint64)
    counts = [tuple(int(x) for x in hdr[3 + 3 * c:6 + 3 * c]) for c in range(nvc)]
    gid_off, secs, total = layout(rows, nvc, counts, nr)
    if total > buf.nbytes:
        raise ValueError("shard blob exceeds its size")

    def get(off, count, dt):
        return buf[off:off + count * np.dtype(dt).itemsize].view(dt).copy()

    gid = get(gid_off, rows, np.uint32)
    out = []
    for c in range(nvc):
        nk, nm, nt = counts[c]
        s = secs[c]
        w = 2 if c >= nvc - nr else 1
        out.append(abi.Csr(get(s[0], rows + 1, np.uint32), get(s[4], nk * w, np.uint64), get(s[1], rows + 1, np.uint32),
                           get(s[5], nm, np.int32), get(s[2], rows + 1, np.uint32), get(s[6], nt, np.uint32), w == 2))
    return gid, out


def export(gid, home_store, csrs, world):
    """ad_shard_export on the host: csrs[vc] = abi.Csr over the store's local rows with TxnIds as local ranks,
    gid = local row -> global rank, home_store[row] = the row's home store.  Per destination d: the rows homed
    at d with any deps, TxnIds rewritten to global ranks.  Returns (concatenated blobs, sizes[world])."""
    gid = np.asarray(gid, np.uint32)
    home_store = np.asarray(home_store, np.int64)
    has = np.zeros(len(gid), bool)
    for c in csrs:
        has |= np.diff(c.txn_off) > 0
    blobs = []
    for d in range(world):
        rows = np.nonzero(has & (home_store == d))[0]
        sub = []
        for c in csrs:
            s = _rows_of(c, rows)
            s.txns = gid[s.txns].astype(np.uint32) if len(s.txns) else s.txns.astype(np.uint32)
            sub.append(s)
        blobs.append(encode(gid[rows], sub))
    sizes = np.array([b.nbytes for b in blobs], np.uint64)
    return (np.concatenate(blobs) if blobs else np.zeros(0, np.uint8)), sizes


def split(buf, sizes):
    """Concatenated blobs (source order) -> list of per-source decoded (gid, csrs)."""
    out, o = [], 0
    for z in np.asarray(sizes, np.int64):
        out.append(decode(buf[o:o + int(z)]))
        o += int(z)
    return out


class HostFragmentStore:
    """A CommandStore whose fragments were resolved on the host: the export / send_buffer / import_host
    surface of sharding.ShardStore, so the same transports (GlooTransport.exchange_blobs) move its bytes."""

    def __init__(self, gid, home_store, csrs, world):
        self._buf, self.send_sizes = export(gid, home_store, csrs, world)
        self.received = None

    def export(self):
        return self.send_sizes

    def send_buffer(self):
        return self._buf

    def import_host(self, recv, sizes):
        self.received = split(np.ascontiguousarray(recv, np.uint8), sizes)
