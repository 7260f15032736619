"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; it is the
checker (and the timed "port" CPU baseline), never part of the product path.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(_HERE), "cassandra-accord_amd"))
from accord_amd import abi  # noqa: E402

_LIB = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.oracle_run.restype = C.c_void_p
        L.oracle_run.argtypes = [C.POINTER(abi.AdBatch), C.POINTER(abi.ModelConfig), C.c_uint32, C.c_uint32]
        L.oracle_run_masked.restype = C.c_void_p
        L.oracle_run_masked.argtypes = [C.POINTER(abi.AdBatch), C.POINTER(abi.ModelConfig), C.c_uint32, C.c_uint32, C.c_void_p]
        L.oracle_run_gid.restype = C.c_void_p
        L.oracle_run_gid.argtypes = [C.POINTER(abi.AdBatch), C.POINTER(abi.ModelConfig), C.c_uint32, C.c_void_p]
        L.oracle_error.restype = C.c_char_p
        L.oracle_error.argtypes = [C.c_void_p]
        L.oracle_sizes.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.c_uint32, C.POINTER(abi.AdCsrSizes)]
        L.oracle_fetch.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.c_uint32, C.POINTER(abi.AdCsrOut)]
        L.oracle_levels.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.oracle_stats.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
        L.oracle_free.argtypes = [C.c_void_p]
        L.oracle_max_conflicts.argtypes = [C.POINTER(abi.AdBatch), C.POINTER(abi.ModelConfig), C.POINTER(C.c_uint32),
                                           C.POINTER(C.c_uint8)]
        vp = C.c_void_p
        L.oracle_max_conflicts_ts.argtypes = [C.POINTER(abi.AdBatch), C.POINTER(abi.ModelConfig), C.c_size_t, vp, vp, vp, vp,
                                              vp, vp, vp, vp]
        L.oracle_max_conflicts_export.argtypes = [C.POINTER(abi.AdBatch), C.c_size_t, vp, vp, vp, vp, C.POINTER(C.c_size_t),
                                                  vp, vp, vp, vp]
        L.oracle_max_conflicts_ts_ranges.argtypes = [C.POINTER(abi.AdBatch), C.POINTER(abi.ModelConfig), C.c_size_t, vp, vp, vp,
                                                     vp, C.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.oracle_max_conflicts_export_ranges.argtypes = [C.POINTER(abi.AdBatch), C.c_size_t, vp, vp, vp, vp, vp,
                                                         C.POINTER(C.c_size_t), vp, vp, vp, vp, vp]
        L.oracle_build.argtypes = [C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.c_size_t,
                                   C.POINTER(C.c_uint64), C.POINTER(C.c_size_t), C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_size_t), C.POINTER(C.c_int32), C.POINTER(C.c_size_t)]
        u64p, u32p, i32p, szp = C.POINTER(C.c_uint64), C.POINTER(C.c_uint32), C.POINTER(C.c_int32), C.POINTER(C.c_size_t)
        L.oracle_union.argtypes = [u64p, C.c_size_t, u32p, C.c_size_t, i32p, C.c_size_t,
                                   u64p, C.c_size_t, u32p, C.c_size_t, i32p, C.c_size_t,
                                   u64p, szp, u32p, szp, i32p, szp]
        L.oracle_set_preaccept_expiry.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, vp, vp, vp, vp, vp]
        L.oracle_invert.argtypes = [i32p, C.c_size_t, C.c_size_t, C.c_size_t, i32p]
        L.oracle_recover.restype = C.c_void_p
        L.oracle_recover.argtypes = [C.POINTER(abi.AdBatch), C.c_void_p, C.c_void_p, C.c_size_t]
        L.oracle_recovery_error.restype = C.c_char_p
        L.oracle_recovery_error.argtypes = [C.c_void_p]
        L.oracle_recovery_entries.restype = C.c_size_t
        L.oracle_recovery_entries.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.oracle_recovery_fetch.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, vp, vp, vp]
        L.oracle_recovery_flags.argtypes = [C.c_void_p, vp]
        L.oracle_recovery_free.argtypes = [C.c_void_p]
        _LIB = L
    return _LIB


FLAG_PRUNE, FLAG_MERGE, FLAG_LEVELS, FLAG_ACCEPT = 1, 2, 4, 8
FLAG_DONE = 16     # levels over a CFK history batch: APPLIED / INVALID txns are done (AD_LEVEL_DONE)
FLAG_BOUND_MAX = 32  # deps with bound Timestamp.MAX (GetEphemeralReadDeps), answered after every arrival
FLAG_KEY_SHARDS = 64  # threads > 1: key-range-sharded stores + PreAccept.reduce (default: TxnId ranges, shared index)


class OracleResult:
    def __init__(self, batch, cfg, flags=FLAG_MERGE | FLAG_LEVELS, threads=1, view_mask=None, gid=None):
        """view_mask ([replicas, n] uint8, optional): per txn, the replies the merge folds (the coordinator's
        fast-path merge: only replies with witnessedAt == TxnId).  gid ([n] uint32, optional): global arrival rank
        of every row (a batch carrying earlier batches' kept CFK rows first); window and drops use it."""
        self._b = abi.make_batch(batch)
        self._cfg = cfg
        self.n = batch["n"]
        self.replicas = cfg.replicas
        if gid is not None:
            self._gid = np.ascontiguousarray(gid, np.uint32)
            self.h = lib().oracle_run_gid(C.byref(self._b), C.byref(cfg), flags, self._gid.ctypes.data)
        elif view_mask is None:
            self.h = lib().oracle_run(C.byref(self._b), C.byref(cfg), flags, threads)
        else:
            self._mask = np.ascontiguousarray(view_mask, np.uint8)
            self.h = lib().oracle_run_masked(C.byref(self._b), C.byref(cfg), flags, threads, self._mask.ctypes.data)
        err = lib().oracle_error(self.h)
        if err:
            msg = err.decode()
            lib().oracle_free(self.h)
            self.h = None
            raise ValueError(msg)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_free(self.h)
            self.h = None

    def _csr(self, stage, view, cls):
        s = abi.AdCsrSizes()
        rc = lib().oracle_sizes(self.h, stage, view, cls, C.byref(s))
        if rc != abi.AD_OK:
            raise ValueError("oracle_sizes rc=%d" % rc)
        out = abi.Csr.alloc(s, is_range=(cls == abi.CLASS_RANGE))
        o = out.as_out()
        lib().oracle_fetch(self.h, stage, view, cls, C.byref(o))
        return out

    def deps(self, view, cls):
        return self._csr(0, view, cls)

    def merged(self, cls):
        return self._csr(1, 0, cls)

    def levels(self):
        lv = np.zeros(self.n, np.uint32)
        order = np.zeros(self.n, np.uint32)
        rc = lib().oracle_levels(self.h, lv.ctypes.data_as(C.POINTER(C.c_uint32)), order.ctypes.data_as(C.POINTER(C.c_uint32)))
        if rc != abi.AD_OK:
            raise ValueError("no levels computed")
        return lv, order

    def stats(self):
        t = (C.c_double * 3)()
        e = (C.c_uint64 * 2)()
        lib().oracle_stats(self.h, t, e)
        return {"t_deps": t[0], "t_merge": t[1], "t_levels": t[2], "deps_entries": e[0], "merged_entries": e[1]}


def max_conflicts(batch, cfg):
    """CommandStore.preaccept's maxConflicts.get(keys) per view (oracle.cpp Oracle::max_conflict) ->
    (max_rank [R, n] uint32, AD_RANK_NONE = 0xFFFFFFFF; fast [R, n] uint8: TxnId >= that executeAt)."""
    b = abi.make_batch(batch)
    n, R = batch["n"], cfg.replicas
    rank = np.zeros((R, max(n, 1)), np.uint32)
    fast = np.zeros((R, max(n, 1)), np.uint8)
    rc = lib().oracle_max_conflicts(C.byref(b), C.byref(cfg), _p(rank, C.c_uint32), _p(fast, C.c_uint8))
    if rc != abi.AD_OK:
        raise ValueError("oracle_max_conflicts rc=%d" % rc)
    return rank[:, :n].copy(), fast[:, :n].copy()


EMPTY_CARRY = (np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.int32))


def _carry(table):
    table = EMPTY_CARRY if table is None else table
    return tuple(np.ascontiguousarray(a, dt) for a, dt in zip(table, (np.uint64, np.uint64, np.uint64, np.int32)))


EMPTY_CARRY_RANGES = (np.zeros(0, np.uint64),) * 4 + (np.zeros(0, np.int32),)


def _carry_ranges(table):
    table = EMPTY_CARRY_RANGES if table is None else table
    return tuple(np.ascontiguousarray(a, dt) for a, dt in zip(table, (np.uint64,) * 4 + (np.int32,)))


NO_TIMEOUT = 0xFFFFFFFFFFFFFFFF


def set_preaccept_expiry(now=0, timeout=NO_TIMEOUT, reject_before=None):
    """The store state of CommandStore.preaccept's expiry test (oracle.cpp preaccept_rules) for the following
    max_conflicts / max_conflicts_ts calls: the clock's now (hlc), preAcceptTimeout (NO_TIMEOUT: no timeout test) and
    rejectBefore as (starts, ends, msb, lsb, node) intervals (s, e] (None: empty)."""
    s, e, m, l, nd = _carry_ranges(reject_before)
    lib().oracle_set_preaccept_expiry(now, timeout, len(s), s.ctypes.data, e.ctypes.data, m.ctypes.data, l.ctypes.data,
                                      nd.ctypes.data)


def max_conflicts_ts(batch, cfg, carry=None, carry_ranges=None):
    """maxConflicts.get(keys or ranges) over a carried MaxConflicts map (key table + interval table) + the batch, as
    timestamps: (msb [R, n], lsb [R, n], node [R, n], fast [R, n])."""
    b = abi.make_batch(batch)
    n, R = batch["n"], cfg.replicas
    ck, cm, cl, cn = _carry(carry)
    rs, re_, rm, rl, rn = _carry_ranges(carry_ranges)
    om = np.zeros((R, max(n, 1)), np.uint64)
    ol = np.zeros((R, max(n, 1)), np.uint64)
    on = np.zeros((R, max(n, 1)), np.int32)
    fa = np.zeros((R, max(n, 1)), np.uint8)
    rc = lib().oracle_max_conflicts_ts_ranges(C.byref(b), C.byref(cfg), len(ck), ck.ctypes.data, cm.ctypes.data,
                                              cl.ctypes.data, cn.ctypes.data, len(rs), rs.ctypes.data, re_.ctypes.data,
                                              rm.ctypes.data, rl.ctypes.data, rn.ctypes.data, om.ctypes.data,
                                              ol.ctypes.data, on.ctypes.data, fa.ctypes.data)
    if rc != abi.AD_OK:
        raise ValueError("oracle_max_conflicts_ts rc=%d" % rc)
    return om[:, :n].copy(), ol[:, :n].copy(), on[:, :n].copy(), fa[:, :n].copy()


def max_conflicts_export(batch, carry=None):
    """The MaxConflicts table after the batch: (keys, msb, lsb, node)."""
    b = abi.make_batch(batch)
    ck, cm, cl, cn = _carry(carry)
    m = C.c_size_t()
    rc = lib().oracle_max_conflicts_export(C.byref(b), len(ck), ck.ctypes.data, cm.ctypes.data, cl.ctypes.data,
                                           cn.ctypes.data, C.byref(m), None, None, None, None)
    if rc != abi.AD_OK:
        raise ValueError("oracle_max_conflicts_export rc=%d" % rc)
    out = (np.zeros(max(m.value, 1), np.uint64), np.zeros(max(m.value, 1), np.uint64), np.zeros(max(m.value, 1), np.uint64),
           np.zeros(max(m.value, 1), np.int32))
    lib().oracle_max_conflicts_export(C.byref(b), len(ck), ck.ctypes.data, cm.ctypes.data, cl.ctypes.data, cn.ctypes.data,
                                      C.byref(m), *(a.ctypes.data for a in out))
    return tuple(a[:m.value].copy() for a in out)


def max_conflicts_export_ranges(batch, carry_ranges=None):
    """The interval part of the MaxConflicts map after the batch: (starts, ends, msb, lsb, node), pieces (s, e]."""
    b = abi.make_batch(batch)
    rs, re_, rm, rl, rn = _carry_ranges(carry_ranges)
    args = (len(rs), rs.ctypes.data, re_.ctypes.data, rm.ctypes.data, rl.ctypes.data, rn.ctypes.data)
    m = C.c_size_t()
    rc = lib().oracle_max_conflicts_export_ranges(C.byref(b), *args, C.byref(m), None, None, None, None, None)
    if rc != abi.AD_OK:
        raise ValueError("oracle_max_conflicts_export_ranges rc=%d" % rc)
    k = max(m.value, 1)
    out = (np.zeros(k, np.uint64),) + tuple(np.zeros(k, np.uint64) for _ in range(3)) + (np.zeros(k, np.int32),)
    lib().oracle_max_conflicts_export_ranges(C.byref(b), *args, C.byref(m), *(a.ctypes.data for a in out))
    return tuple(a[:m.value].copy() for a in out)


def build_relation(keys, vals):
    """RelationMultiMap.AbstractBuilder over (key, value-rank) pairs in add order -> (keys, vals, k2t)."""
    keys = np.ascontiguousarray(keys, np.uint64)
    vals = np.ascontiguousarray(vals, np.uint32)
    n = len(keys)
    ok = np.zeros(max(n, 1), np.uint64)
    ov = np.zeros(max(n, 1), np.uint32)
    om = np.zeros(max(2 * n, 1), np.int32)
    nk, nv, nm = C.c_size_t(), C.c_size_t(), C.c_size_t()
    rc = lib().oracle_build(keys.ctypes.data_as(C.POINTER(C.c_uint64)), vals.ctypes.data_as(C.POINTER(C.c_uint32)), n,
                            ok.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(nk),
                            ov.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(nv),
                            om.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(nm))
    if rc != abi.AD_OK:
        raise ValueError("builder rejected input (rc=%d)" % rc)
    return ok[:nk.value].copy(), ov[:nv.value].copy(), om[:nm.value].copy()


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def union_relation(left, right):
    """RelationMultiMap.linearUnion of two canonical (keys, vals, k2t) relations -> (keys, vals, k2t)."""
    lk, lv, lm = (np.ascontiguousarray(left[0], np.uint64), np.ascontiguousarray(left[1], np.uint32),
                  np.ascontiguousarray(left[2], np.int32))
    rk, rv, rm = (np.ascontiguousarray(right[0], np.uint64), np.ascontiguousarray(right[1], np.uint32),
                  np.ascontiguousarray(right[2], np.int32))
    cap = len(lk) + len(rk) + 1
    ok = np.zeros(cap, np.uint64)
    ov = np.zeros(len(lv) + len(rv) + 1, np.uint32)
    om = np.zeros(len(lm) + len(rm) + 1, np.int32)
    nk, nv, nm = C.c_size_t(), C.c_size_t(), C.c_size_t()
    lib().oracle_union(_p(lk, C.c_uint64), len(lk), _p(lv, C.c_uint32), len(lv), _p(lm, C.c_int32), len(lm),
                       _p(rk, C.c_uint64), len(rk), _p(rv, C.c_uint32), len(rv), _p(rm, C.c_int32), len(rm),
                       _p(ok, C.c_uint64), C.byref(nk), _p(ov, C.c_uint32), C.byref(nv), _p(om, C.c_int32), C.byref(nm))
    return ok[:nk.value].copy(), ov[:nv.value].copy(), om[:nm.value].copy()


def invert(k2t, n_keys, n_vals):
    """RelationMultiMap.invert (oracle.cpp oracle_invert): keysToTxnIds of n_keys keys over n_vals TxnIds ->
    txnIdsToKeys (KeyDeps.txnIdsToKeys / RangeDeps.txnIdsToRanges)."""
    src = np.ascontiguousarray(k2t, np.int32)
    out = np.zeros(max(n_vals + len(src) - n_keys, 1), np.int32)
    rc = lib().oracle_invert(_p(src, C.c_int32), len(src), n_keys, n_vals, _p(out, C.c_int32))
    if rc != abi.AD_OK:
        raise ValueError("invert rejected input (rc=%d)" % rc)
    return out[:n_vals + len(src) - n_keys].copy()


EMPTY_RELATION = (np.zeros(0, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.int32))


def recover(batch, merged, rows):
    """BeginRecovery's store queries (oracle.cpp oracle_recover) for the recovering rows, over the batch whose txns hold
    the Deps `merged` ([key, direct, range] abi.Csr) -> (out, reject): out[which][cls] = (off [nq+1], keys [E] or
    [E, 2], txns [E]) with which 0 = earlierCommittedWitness, 1 = earlierAcceptedNoWitness; reject [nq] uint8 =
    rejectsFastPath."""
    b = abi.make_batch(batch)
    rows = np.ascontiguousarray(rows, np.uint32)
    parts = (abi.AdCsrIn * 3)()
    for c in range(3):
        parts[c] = merged[c].as_in()
    h = lib().oracle_recover(C.byref(b), C.cast(parts, C.c_void_p), rows.ctypes.data, len(rows))
    try:
        err = lib().oracle_recovery_error(h)
        if err:
            raise ValueError(err.decode())
        out = []
        for w in range(2):
            cl = []
            for c in range(3):
                e = lib().oracle_recovery_entries(h, w, c)
                w2 = 2 if c == abi.CLASS_RANGE else 1
                off = np.zeros(len(rows) + 1, np.uint32)
                keys = np.zeros(max(e * w2, 1), np.uint64)
                txns = np.zeros(max(e, 1), np.uint32)
                lib().oracle_recovery_fetch(h, w, c, off.ctypes.data, keys.ctypes.data, txns.ctypes.data)
                keys = keys[:e * w2].reshape(-1, 2) if w2 == 2 else keys[:e]
                cl.append((off, keys.copy(), txns[:e].copy()))
            out.append(cl)
        rej = np.zeros(max(len(rows), 1), np.uint8)
        lib().oracle_recovery_flags(h, rej.ctypes.data)
        return out, rej[:len(rows)].copy()
    finally:
        lib().oracle_recovery_free(h)
