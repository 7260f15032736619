"""Host model of the device-resident CFK store's event application (csrc/cfk_store_kernels.h k_cfk_apply) — TEST
INFRASTRUCTURE.  It restates the kernel's own data layout (byId rows with insertion slots, missing() as a bitmap over
slots) step for step, so a CPU test can check that the kernel's algorithm, replayed over the event log of the restated
CommandsForKeyTest harness (tests/cfk_canon.py, CFK.log), reproduces the harness's CommandsForKey rows and missing()
arrays at every sampled event; the -m gpu test then compares the device with the same snapshots.

Events: (txnId, InternalStatus, executeAt, deps) — CommandsForKey.update of a managed command
(local/cfk/CommandsForKey.java:987-1057, Updating.insertOrUpdate :99-358) or, with status TRANSITIVELY_KNOWN, the
insertAdditionsOnly path of Updating.updateUnmanaged (:452-514)."""
import bisect

import numpy as np

import cfk_canon as K


def has_deps(s):
    return s in (K.ACC, K.COMMITTED, K.STABLE, K.APPLIED)


def decided(s):
    return s in (K.COMMITTED, K.STABLE, K.APPLIED)


class StoreModel:
    def __init__(self):
        self.ids = []            # byId TxnIds
        self.row = []            # per byId row: [status, executeAt, slot]
        self.bits = []           # per slot: missing bitmap over slots (python int)
        self.slot_txn = []       # per slot: its TxnId

    def _find(self, t):
        p = bisect.bisect_left(self.ids, t)
        return p, p < len(self.ids) and self.ids[p] == t

    def _insert(self, p, t, status, ex):
        s = len(self.slot_txn)
        self.ids.insert(p, t)
        self.row.insert(p, [status, ex, s])
        self.bits.append(0)
        self.slot_txn.append(t)
        return s

    def _dkb(self, r):
        st, ex, _ = self.row[r]
        return ex if decided(st) else self.ids[r]

    def _add_missing(self, t, ts, skip):
        kt = K.kind_of(t)
        for r, u in enumerate(self.ids):
            st, _, s = self.row[r]
            if s == ts or s == skip or not has_deps(st) or not K.witnesses(K.kind_of(u), kt):
                continue
            if self._dkb(r) > t:
                self.bits[s] |= 1 << ts

    def _remove_missing(self, ts):
        for s in range(len(self.bits)):
            self.bits[s] &= ~(1 << ts)

    def apply(self, ev):
        t, ns, ex, deps = ev
        p, found = self._find(t)
        cur = self.row[p][0] if found else None
        if found and ns <= cur:
            return
        if has_deps(ns):
            dkb = ex if decided(ns) else t
            kt = K.kind_of(t)
            dset = set(deps)
            miss = 0
            for r, u in enumerate(self.ids):
                st, _, s = self.row[r]
                if st >= K.COMMITTED or not K.witnesses(kt, K.kind_of(u)) or u >= dkb or u == t or u in dset:
                    continue
                miss |= 1 << s
            adds = []
            for d in deps:
                q, f = self._find(d)
                if not f:
                    adds.append(self._insert(q, d, K.TK, d))
            p2, f2 = self._find(t)
            if not f2:
                ts = self._insert(p2, t, ns, ex)
            else:
                ts = self.row[p2][2]
                self.row[p2][0], self.row[p2][1] = ns, ex
            self.bits[ts] = miss
            for s in adds:
                self._add_missing(self.slot_txn[s], s, ts)
            if not found and ns < K.COMMITTED:
                self._add_missing(t, ts, None)
            if found and cur < K.COMMITTED and ns >= K.COMMITTED:
                self._remove_missing(ts)
        else:
            if not found:
                ts = self._insert(p, t, ns, t)
                if ns != K.INVALID:
                    self._add_missing(t, ts, None)
            else:
                ts = self.row[p][2]
                self.row[p][0], self.row[p][1] = ns, t
                self.bits[ts] = 0
                if cur < K.COMMITTED and ns == K.INVALID:
                    self._remove_missing(ts)

    def rows(self):
        """(txnId, status, executeAt, missing as byId row indices ascending) per byId row."""
        pos = {s: r for r, (_, _, s) in enumerate(self.row)}
        out = []
        for r, t in enumerate(self.ids):
            st, ex, s = self.row[r]
            b, m = self.bits[s], []
            while b:
                low = b & -b
                m.append(pos[low.bit_length() - 1])
                b ^= low
            out.append((t, st, ex, sorted(m)))
        return out


def pack_events(per_key, domains):
    """Per key a list of events -> the ad_cfk_events arrays (grouped by key)."""
    ev_off, tm, tl, tn, st, em, el, en, doff, dm, dl, dn = [0], [], [], [], [], [], [], [], [0], [], [], []
    for evs in per_key:
        for t, s, ex, deps in evs:
            m, l, n = K.ts_bits(t, domains[t])
            tm.append(m); tl.append(l); tn.append(n); st.append(s)
            m, l, n = K.ts_bits(ex, domains[t]) if ex == t else K.ts_bits(ex)   # executeAt = TxnId keeps its flags
            em.append(m); el.append(l); en.append(n)
            for d in deps:
                m, l, n = K.ts_bits(d, domains[d])
                dm.append(m); dl.append(l); dn.append(n)
            doff.append(len(dm))
        ev_off.append(len(st))
    return {"ev_off": np.array(ev_off, np.uint32), "txn_msb": np.array(tm, np.uint64), "txn_lsb": np.array(tl, np.uint64),
            "txn_node": np.array(tn, np.int32), "status": np.array(st, np.uint8), "exec_msb": np.array(em, np.uint64),
            "exec_lsb": np.array(el, np.uint64), "exec_node": np.array(en, np.int32),
            "deps_off": np.array(doff, np.uint32), "deps_msb": np.array(dm, np.uint64), "deps_lsb": np.array(dl, np.uint64),
            "deps_node": np.array(dn, np.int32)}
