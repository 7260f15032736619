"""Host model of the device-resident CFK store's event application (csrc/cfk_store_kernels.h k_cfk_apply) — TEST
INFRASTRUCTURE.  It restates the kernel's own data layout (byId rows with insertion slots, missing() as a bitmap over
slots) step for step, so a CPU test can check that the kernel's algorithm, replayed over the event log of the restated
CommandsForKeyTest harness (tests/cfk_canon.py, CFK.log), reproduces the harness's CommandsForKey rows and missing()
arrays at every sampled event; the -m gpu test then compares the device with the same snapshots.

Events: (txnId, InternalStatus, executeAt, deps[, op[, interval, hlcDelta]]) —
* op UPDATE (absent): CommandsForKey.update of a managed command (local/cfk/CommandsForKey.java:987-1057,
  Updating.insertOrUpdate :99-358) or, with status TRANSITIVELY_KNOWN, the insertAdditionsOnly path of
  Updating.updateUnmanaged (:452-514); deps below prunedBefore that the rows lack become loadingPruned entries witnessed
  by the command (Utils.removePrunedAdditions :229-244);
* op LOAD: CommandsForKey.updatePruned (:998-1005) of a loaded pruned command (TxnInfo.create: no missing(), and the
  TxnId joins the other rows' missing() except its loadingPruned witnesses, Updating.java:289-358); an UPDATE of a TxnId
  that is in loadingPruned takes this path too (:1015-1016);
* op PRUNE: Pruning.maybePrune(interval, hlcDelta) (Pruning.java:164-331);
* op LOADING: the pruned deps of an unmanaged command join loadingPruned, witnessed by it (Updating.java:806-815).
The loading table keeps per entry its TxnId and its witnesses as a bitmap over slots (witnesses that are not rows of
the key are never read: isWaitingOnPruned asks about rows, addToMissingArrays skips rows)."""
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
        self.pruned_before = K.NONE
        self.lp_id = []          # loading table: TxnIds (in insertion order, swap-removed)
        self.lp_bits = []        # their witnesses as slot bitmaps

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

    def _lp_find(self, t):
        return self.lp_id.index(t) if t in self.lp_id else -1

    def _lp_add(self, t, wbits):
        j = self._lp_find(t)
        if j < 0:
            self.lp_id.append(t)
            self.lp_bits.append(wbits)
        else:
            self.lp_bits[j] |= wbits

    def _lp_remove(self, j):
        self.lp_id[j], self.lp_bits[j] = self.lp_id[-1], self.lp_bits[-1]
        self.lp_id.pop()
        self.lp_bits.pop()

    def _add_missing(self, t, ts, skip, dont=0):
        kt = K.kind_of(t)
        for r, u in enumerate(self.ids):
            st, _, s = self.row[r]
            if s == ts or s == skip or not has_deps(st) or not K.witnesses(K.kind_of(u), kt) or (dont >> s) & 1:
                continue
            if self._dkb(r) > t:
                self.bits[s] |= 1 << ts

    def _remove_missing(self, ts):
        for s in range(len(self.bits)):
            self.bits[s] &= ~(1 << ts)

    def apply(self, ev):
        t, ns, ex, deps = ev[:4]
        op = ev[4] if len(ev) > 4 else K.OP_UPDATE
        if op == K.OP_PRUNE:
            self.maybe_prune(ev[5], ev[6])
            return
        if op in (K.OP_UNMANAGED, K.OP_UNMANAGED_RECHECK):   # the registry is not modelled here (no row changes)
            return
        if op == K.OP_LOADING:
            w = 0
            for d in deps:
                q, f = self._find(d)
                if f:
                    w |= 1 << self.row[q][2]
            self._lp_add(t, w)
            return
        p, found = self._find(t)
        cur = self.row[p][0] if found else None
        if found and ns <= cur:
            return
        j = self._lp_find(t)
        if op == K.OP_LOAD or j >= 0:
            dont = 0
            if j >= 0:
                dont = self.lp_bits[j]
                self._lp_remove(j)
            if not found:
                ts = self._insert(p, t, ns, ex)
            else:
                ts = self.row[p][2]
                self.row[p][0], self.row[p][1] = ns, ex
                self.bits[ts] = 0
            if decided(ns) and not (found and decided(cur)):
                self._remove_missing(ts)
            elif found and cur < K.COMMITTED and ns == K.INVALID:
                self._remove_missing(ts)
            elif not found and ns != K.INVALID:
                self._add_missing(t, ts, None, dont)
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
            adds, pruned = [], []
            for d in deps:
                q, f = self._find(d)
                if not f:
                    if d < self.pruned_before:
                        pruned.append(d)
                    else:
                        adds.append(self._insert(q, d, K.TK, d))
            p2, f2 = self._find(t)
            if not f2:
                ts = self._insert(p2, t, ns, ex)
            else:
                ts = self.row[p2][2]
                self.row[p2][0], self.row[p2][1] = ns, ex
            self.bits[ts] = miss
            for d in pruned:
                self._lp_add(d, 1 << ts)
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

    def maybe_prune(self, interval, delta):
        """Pruning.maybePrune as the kernel computes it: order statistics over the committed rows instead of a
        committedByExecuteAt array, then pruneBefore's sequential byId scan with missing() as bitmaps, then compaction
        of rows and slots (every removed row is Applied or invalidated, so no missing bit names it)."""
        com = [r for r in range(len(self.ids)) if decided(self.row[r][0])]
        aw = [r for r in com if self.row[r][0] == K.APPLIED and K.kind_of(self.ids[r]) == K.WRITE]
        if not aw:
            return
        maw = max(aw, key=lambda r: self.row[r][1])
        mex = self.row[maw][1]
        rank = sum(1 for r in com if self.row[r][1] < mex)
        if rank < interval:
            return
        lim = mex[1] - delta
        cand = [r for r in aw if self.row[r][1] < mex and self.row[r][1][1] <= lim]
        if not cand:
            return
        npb = max(cand, key=lambda r: self.row[r][1])
        if self.ids[npb] <= self.pruned_before or npb == 0:
            return
        pex = self.row[npb][1]
        merged = self.bits[self.row[npb][2]]
        gone = []
        for r in range(npb):
            st, ex, s = self.row[r]
            if st == K.INVALID:
                gone.append(r)
            elif st == K.APPLIED and ex < pex:
                b = self.bits[s]
                if b & ~merged == 0:
                    gone.append(r)
                elif ex == self.ids[r]:
                    merged |= b
        if not gone:
            return
        self.pruned_before = self.ids[npb]
        gset = set(gone)
        dead = {self.row[r][2] for r in gone}
        remap, k = {}, 0
        for s in range(len(self.slot_txn)):
            if s not in dead:
                remap[s] = k
                k += 1

        def rebits(b):
            out = 0
            while b:
                low = b & -b
                s = low.bit_length() - 1
                assert s in remap, "a missing bit names a pruned row"
                out |= 1 << remap[s]
                b ^= low
            return out
        self.ids = [t for r, t in enumerate(self.ids) if r not in gset]
        self.row = [[st, ex, remap[s]] for r, (st, ex, s) in enumerate(self.row) if r not in gset]
        nb, nt = [0] * k, [None] * k
        for s, ns in remap.items():
            nb[ns] = rebits(self.bits[s])
            nt[ns] = self.slot_txn[s]
        self.bits, self.slot_txn = nb, nt
        self.lp_bits = [rebits(b & ~sum(1 << s for s in dead)) for b in self.lp_bits]

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
    """Per key a list of events -> the ad_cfk_events arrays (grouped by key).  A PRUNE event carries its interval in
    exec_node and its minHlcDelta in exec_msb."""
    ev_off, tm, tl, tn, st, em, el, en, doff, dm, dl, dn, ops = [0], [], [], [], [], [], [], [], [0], [], [], [], []
    for evs in per_key:
        for ev in evs:
            t, s, ex, deps = ev[:4]
            op = ev[4] if len(ev) > 4 else K.OP_UPDATE
            ops.append(op)
            if op == K.OP_PRUNE:
                tm.append(0); tl.append(0); tn.append(0); st.append(0)
                em.append(ev[6]); el.append(0); en.append(ev[5])
                doff.append(len(dm))
                continue
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
            "deps_node": np.array(dn, np.int32), "op": np.array(ops, np.uint8)}
