"""Host side of the replica's witnessedAt proposal (the part of CommandStore.preaccept that is not data-parallel).

The engine answers maxConflicts.get(keys) per txn and view on the device (ad_max_conflicts); what remains is a
clock read and a comparison, restated here from the reference:

* ``Timestamp`` order / bits        primitives/Timestamp.java:81-96, 208-227, 328-336
* ``NodeClock.unique_now``          Node.uniqueNow / uniqueNow(atLeast) / nowAtLeast, local/Node.java:335-375
* ``preaccept_witnessed_at``        CommandStore.preaccept, local/CommandStore.java:322-347: TxnId on the fast
                                    path (TxnId >= maxConflict and the txn's epoch is current), else
                                    time.uniqueNow(maxConflict).
* ``preaccept``                     the whole of CommandStore.preaccept (:322-347): the expiry test
                                    (preAcceptTimeout, :326) and the rejectBefore fold (:327-328) ->
                                    uniqueNow(TxnId).asRejected(); ExclusiveSyncPoint -> markExclusiveSyncPoint +
                                    TxnId (:333-337); else the fast-path test above.  The device applies the same
                                    rules to its fast flags (ad_preaccept_expiry; AD_FAST_REJECTED).
* ``RejectBefore``                  CommandStore.rejectBefore, the ReducingRangeMap<Timestamp> markExclusiveSyncPoint
                                    builds (:300-306), as sorted disjoint (start, end] intervals.

Timestamps are (msb, lsb, node) int triples (Accord's raw bits, as the C-ABI passes them).
"""
IDENTITY_FLAGS = 0x1E
NONE = (0, 0, 0)                       # Timestamp.NONE = fromValues(0, 0, 0, Id.NONE)


def from_values(epoch, hlc, flags, node):
    """Timestamp.fromValues(epoch, hlc, flags, node) bits (Timestamp.java:81-89)."""
    return ((epoch << 15) | (hlc >> 48), ((hlc << 16) & 0xFFFFFFFFFFFFFFFF) | flags, node)


def epoch(t):
    return t[0] >> 15


def hlc(t):
    return ((t[0] & 0x7FFF) << 48) | (t[1] >> 16)


def flags(t):
    return t[1] & 0xFFFF


def order_key(t):
    """Timestamp.compareTo (:208-217): msb unsigned, lowHlc, identity flags, node."""
    return (t[0], t[1] >> 16, t[1] & IDENTITY_FLAGS, t[2])


IDENTITY_LSB = 0xFFFFFFFFFFFF001E


def equals(a, b):
    """Timestamp.equals (:244-249): msb, the identity bits of lsb (hlc and kind flags; not the domain bit or
    REJECTED) and node."""
    return a[0] == b[0] and (a[1] & IDENTITY_LSB) == (b[1] & IDENTITY_LSB) and a[2] == b[2]


def compare(a, b):
    ka, kb = order_key(a), order_key(b)
    return (ka > kb) - (ka < kb)


def with_next_hlc(t, hlc_at_least):
    """Timestamp.withNextHlc (:149-153)."""
    return from_values(epoch(t), max(hlc_at_least, hlc(t) + 1), flags(t), t[2])


def with_epoch_at_least(t, min_epoch):
    """Timestamp.withEpochAtLeast (:155-158)."""
    return t if min_epoch <= epoch(t) else from_values(min_epoch, hlc(t), flags(t), t[2])


def with_hlc_at_least(t, min_hlc):
    return t if min_hlc <= hlc(t) else from_values(epoch(t), min_hlc, flags(t), t[2])


class NodeClock:
    """Node.now + nowSupplier + topology epoch (local/Node.java:161, 188, 335-375)."""

    def __init__(self, node, epoch_, hlc_now, now_epoch=None):
        """now_epoch: the topology epoch when the node was built (Node.java:188 builds `now` from topology.epoch()
        then: 0 before the configuration service has reported any topology); default epoch_."""
        self.node = node
        self.topology_epoch = epoch_
        self.clock = hlc_now                                      # nowSupplier.getAsLong()
        self.now = from_values(epoch_ if now_epoch is None else now_epoch, hlc_now, 0, node)

    def unique_now(self, at_least=None):
        if at_least is not None and compare(self.now, at_least) < 0:
            cur = self.now
            if not (epoch(cur) >= epoch(at_least) and hlc(cur) >= hlc(at_least)):     # nowAtLeast
                p = with_hlc_at_least(with_epoch_at_least(at_least, epoch(at_least)), hlc(cur))
                self.now = (p[0], p[1], cur[2])
        nxt = with_epoch_at_least(with_next_hlc(self.now, self.clock), self.topology_epoch)
        self.now = nxt
        return nxt


def preaccept_witnessed_at(txn_id, max_conflict, clock, permit_fast_path=True):
    """CommandStore.preaccept's decision (:335-346) given maxConflicts.get(keys) (None / NONE when the store
    recorded nothing on the keys)."""
    mc = NONE if max_conflict is None else max_conflict
    if permit_fast_path and compare(txn_id, mc) >= 0 and epoch(txn_id) >= clock.topology_epoch:
        return txn_id
    return clock.unique_now(mc)


REJECTED_FLAG = 0x8000                 # Timestamp.REJECTED_FLAG (:32)
KIND_SYNC_POINT, KIND_EXCLUSIVE_SYNC_POINT = 3, 4


def as_rejected(t):
    """Timestamp.asRejected (:144-147)."""
    return (t[0], t[1] | REJECTED_FLAG, t[2])


def kind(t):
    return (t[1] >> 1) & 7


class RejectBefore:
    """CommandStore.rejectBefore: ReducingRangeMap<Timestamp> of the greatest ExclusiveSyncPoint TxnId marked over
    each range (markExclusiveSyncPoint, CommandStore.java:300-306: ReducingRangeMap.add(.., Timestamp::max)), held as
    sorted disjoint intervals (s, e] -> Timestamp in normal form (adjacent equal values coalesced).  A key k is the
    interval (k - 1, k]."""

    def __init__(self):
        self.iv = []                   # [(s, e, ts)]

    def add(self, ranges, ts):
        pts = sorted({p for s, e, _ in self.iv for p in (s, e)} | {p for s, e in ranges for p in (s, e)})
        out = []
        for a, b in zip(pts, pts[1:]):
            best = None
            for s, e, t in self.iv:
                if s <= a and b <= e:
                    best = t
            if any(s <= a and b <= e for s, e in ranges) and (best is None or compare(ts, best) > 0):
                best = ts
            if best is None:
                continue
            if out and out[-1][1] == a and out[-1][2] == best:
                out[-1] = (out[-1][0], b, best)
            else:
                out.append((a, b, best))
        self.iv = out

    def rejects(self, txn_id, keys=(), ranges=()):
        """rejectBefore.foldl(keys, rejectIfBefore.compareTo(test) > 0 ? null : test, txnId, isNull) == null."""
        for s, e, t in self.iv:
            if any(s < k <= e for k in keys) or any(s < qe and e > qs for qs, qe in ranges):
                if compare(t, txn_id) > 0:
                    return True
        return False

    def table(self):
        """(starts, ends, msb, lsb, node) arrays for ad_preaccept_expiry / the oracle."""
        import numpy as np
        iv = self.iv
        return (np.array([x[0] for x in iv], np.uint64), np.array([x[1] for x in iv], np.uint64),
                np.array([x[2][0] for x in iv], np.uint64), np.array([x[2][1] for x in iv], np.uint64),
                np.array([x[2][2] for x in iv], np.int32))


def preaccept(txn_id, max_conflict, clock, keys=(), ranges=(), reject_before=None, pre_accept_timeout=None,
              permit_fast_path=True):
    """CommandStore.preaccept (local/CommandStore.java:322-347) given maxConflicts.get(keys or ranges): the witnessedAt
    the replica answers.  keys / ranges: the txn's footprint sliced to the store (ranges as (start, end] pairs);
    reject_before: the store's RejectBefore (marked here when txn_id is an ExclusiveSyncPoint, as the reference does);
    pre_accept_timeout: Agent.preAcceptTimeout in hlc units (None: no timeout test)."""
    expired = (pre_accept_timeout is not None and clock.clock - hlc(txn_id) >= pre_accept_timeout
               and kind(txn_id) not in (KIND_SYNC_POINT, KIND_EXCLUSIVE_SYNC_POINT))
    if reject_before is not None and not expired:
        expired = reject_before.rejects(txn_id, keys, ranges)
    if expired:
        return as_rejected(clock.unique_now(txn_id))
    if kind(txn_id) == KIND_EXCLUSIVE_SYNC_POINT:
        if reject_before is not None:
            reject_before.add(list(ranges) + [(k - 1, k) for k in keys], txn_id)
        return txn_id
    return preaccept_witnessed_at(txn_id, max_conflict, clock, permit_fast_path)
