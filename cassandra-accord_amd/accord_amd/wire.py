"""Deps wire formats at the host boundary.

* The zero-copy form is the C-ABI's own: a batched per-txn CSR = the arguments of KeyDeps.SerializerSupport.create
  (primitives/KeyDeps.java:55-73) / RangeDeps.SerializerSupport.create (primitives/RangeDeps.java:86-104) for every
  row, with TxnIds as batch ranks; ``ad_fetch_rows`` pages it out, ``ad_merge_host`` takes it in (validated).
* The Maelstrom JSON form is ``Json.DEPS_ADAPTER`` (accord-maelstrom/.../Json.java:316-428):
  ``{"keyDeps": [[key, txnId], ...], "rangeDeps": [[start, end, txnId], ...], "directKeyDeps": [[key, txnId], ...]}``
  with one entry per (key, TxnId) in the Deps iteration order (keys ascending, each key's TxnIds ascending; RangeDeps
  by Range order), a TxnId as ``[msb, lsb, node]`` (Json.writeTimestamp :138-150: Java longs, the node id as
  ``"n<id>"`` / ``"c<id>"`` or null for id 0, Json.ID_ADAPTER :58-96) and keys / range bounds as the Datum LONG
  values the host encodes them by (this engine's u64 keys, as signed Java longs).  Reading is
  ``KeyDeps.Builder`` / ``RangeDeps.Builder`` (entries in any order, duplicates folded).

``to_json`` renders one row of a fetched batched CSR triple; ``from_json`` builds canonical rows back, and
``relations_to_csr`` packs rows into the batched CSR ``ad_merge_host`` accepts.
"""
import json

import numpy as np

from . import abi

_M64 = (1 << 64) - 1


def _signed(x):
    x = int(x) & _M64
    return x - (1 << 64) if x >> 63 else x


def _unsigned(x):
    return int(x) & _M64


def node_to_json(node):
    node = int(node)
    if node == 0:
        return None
    return ("c%d" if node < 0 else "n%d") % node


def node_from_json(v):
    if v is None:
        return 0
    if v[0] not in "cn":
        raise ValueError("node id %r" % (v,))
    return int(v[1:])


def ts_to_json(msb, lsb, node):
    return [_signed(msb), _signed(lsb), node_to_json(node)]


def ts_from_json(v):
    return _unsigned(v[0]), _unsigned(v[1]), node_from_json(v[2])


class TxnTable:
    """Batch ranks <-> TxnIds (msb, lsb, node) for the batch a CSR's ranks refer to."""

    def __init__(self, batch):
        self.msb, self.lsb, self.node = batch["txn_msb"], batch["txn_lsb"], batch["txn_node"]
        self._rank = {(int(m), int(l), int(nd)): r for r, (m, l, nd) in enumerate(zip(self.msb, self.lsb, self.node))}

    def txn_id(self, r):
        return ts_to_json(self.msb[r], self.lsb[r], self.node[r])

    def rank(self, v):
        key = ts_from_json(v)
        if key not in self._rank:
            raise ValueError("TxnId %r is not in the batch" % (v,))
        return self._rank[key]


def to_json(txns, key_csr, direct_csr, range_csr, row):
    """Json.DEPS_ADAPTER.write of row `row` of three fetched classes (abi.Csr; range_csr may be None)."""
    def entries(csr):
        out = []
        if csr is None or csr.n == 0:
            return out
        ks, tx, k2t = csr.txn(row)
        nk = len(ks)
        for k in range(nk):
            lo = nk if k == 0 else int(k2t[k - 1])
            hi = int(k2t[k])
            for x in range(lo, hi):
                t = txns.txn_id(int(tx[int(k2t[x])]))
                if csr.is_range:
                    out.append([_signed(ks[k][0]), _signed(ks[k][1]), t])
                else:
                    out.append([_signed(ks[k]), t])
        return out
    return {"keyDeps": entries(key_csr), "rangeDeps": entries(range_csr), "directKeyDeps": entries(direct_csr)}


def dumps(obj):
    return json.dumps(obj, separators=(",", ":"))


def _relation(pairs):
    """KeyDeps.Builder / RangeDeps.Builder: (key, rank) pairs in any order -> canonical (keys, txns, keysToTxnIds)."""
    by_key = {}
    for k, r in pairs:
        by_key.setdefault(k, set()).add(r)
    keys = sorted(by_key)
    txns = sorted(set(r for v in by_key.values() for r in v))
    pos = {r: i for i, r in enumerate(txns)}
    heads, body = [], []
    for k in keys:
        body.extend(pos[r] for r in sorted(by_key[k]))
        heads.append(len(keys) + len(body))
    return keys, txns, heads + body


def from_json(obj, txns):
    """Json.DEPS_ADAPTER.read -> {"key": rel, "direct": rel, "range": rel}, rel = (keys, txn ranks, keysToTxnIds)
    canonical as SerializerSupport.create takes them; unknown names are refused as the adapter does (:420)."""
    out = {"key": _relation([]), "direct": _relation([]), "range": _relation([])}
    for name, arr in obj.items():
        if name == "keyDeps":
            out["key"] = _relation([(_unsigned(e[0]), txns.rank(e[1])) for e in arr])
        elif name == "directKeyDeps":
            out["direct"] = _relation([(_unsigned(e[0]), txns.rank(e[1])) for e in arr])
        elif name == "rangeDeps":
            out["range"] = _relation([((_unsigned(e[0]), _unsigned(e[1])), txns.rank(e[2])) for e in arr])
        else:
            raise ValueError("Unknown name: %s" % name)
    return out


def relations_to_csr(rels, is_range=False):
    """Per-row canonical relations -> one batched abi.Csr (the layout ad_merge_host takes)."""
    ko, mo, to = [0], [0], [0]
    for k, v, m in rels:
        ko.append(ko[-1] + len(k)); mo.append(mo[-1] + len(m)); to.append(to[-1] + len(v))
    if is_range:
        keys = np.array([x for r in rels for kk in r[0] for x in kk], np.uint64)
    else:
        keys = np.array([kk for r in rels for kk in r[0]], np.uint64)
    k2t = np.array([x for r in rels for x in r[2]], np.int32)
    txns = np.array([x for r in rels for x in r[1]], np.uint32)
    return abi.Csr(np.array(ko, np.uint32), keys, np.array(mo, np.uint32), k2t, np.array(to, np.uint32), txns, is_range)
