"""Hand-built batches for known-answer tests (TEST INFRASTRUCTURE)."""
import numpy as np

from accord_amd import abi

EPOCH = 1


def ts_bits(hlc, flags, epoch=EPOCH):
    msb = (epoch << 15) | (hlc >> 48)
    lsb = ((hlc << 16) & 0xFFFFFFFFFFFFFFFF) | flags
    return msb, lsb


class T:
    """One transaction: TxnId (hlc, kind, domain, node), footprint, final executeAt and status."""

    def __init__(self, hlc, kind, keys=(), ranges=(), node=1, exec_hlc=None, exec_node=None, status=abi.ST_APPLIED):
        self.hlc, self.kind, self.node = hlc, kind, node
        self.keys, self.ranges = list(keys), list(ranges)
        self.domain = abi.DOMAIN_RANGE if ranges else abi.DOMAIN_KEY
        self.exec_hlc = hlc if exec_hlc is None else exec_hlc
        self.exec_node = node if exec_node is None else exec_node
        self.status = status


def make_batch(txns):
    txns = sorted(txns, key=lambda t: (t.hlc, t.node))
    n = len(txns)
    b = {"n": n}
    tm, tl, em, el = [], [], [], []
    for t in txns:
        flags = (t.kind << 1) | t.domain
        m, l = ts_bits(t.hlc, flags)
        tm.append(m); tl.append(l)
        m, l = ts_bits(t.exec_hlc, flags)
        em.append(m); el.append(l)
    b["txn_msb"], b["txn_lsb"] = np.array(tm, np.uint64), np.array(tl, np.uint64)
    b["exec_msb"], b["exec_lsb"] = np.array(em, np.uint64), np.array(el, np.uint64)
    b["txn_node"] = np.array([t.node for t in txns], np.int32)
    b["exec_node"] = np.array([t.exec_node for t in txns], np.int32)
    b["status"] = np.array([t.status for t in txns], np.uint8)
    ko = np.zeros(n + 1, np.uint32)
    ko[1:] = np.cumsum([len(t.keys) for t in txns])
    b["key_off"] = ko
    b["keys"] = np.array([k for t in txns for k in t.keys], np.uint64)
    if any(t.ranges for t in txns):
        ro = np.zeros(n + 1, np.uint32)
        ro[1:] = np.cumsum([len(t.ranges) for t in txns])
        b["range_off"] = ro
        b["range_start"] = np.array([r[0] for t in txns for r in t.ranges], np.uint64)
        b["range_end"] = np.array([r[1] for t in txns for r in t.ranges], np.uint64)
    else:
        b["range_off"] = b["range_start"] = b["range_end"] = None
    return b


def deps_of(csr, i):
    """{key: [dep ranks]} of txn i from a batched CSR (RangeDeps: key = (start, end))."""
    ks, txns, k2t = csr.txn(i)
    nk = len(ks)
    out = {}
    start = nk
    for ki in range(nk):
        end = int(k2t[ki])
        key = tuple(int(x) for x in ks[ki]) if csr.is_range else int(ks[ki])
        out[key] = [int(txns[int(x)]) for x in k2t[start:end]]
        start = end
    return out
