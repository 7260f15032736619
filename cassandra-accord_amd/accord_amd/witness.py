"""Host side of the replica's witnessedAt proposal (the part of CommandStore.preaccept that is not data-parallel).

The engine answers maxConflicts.get(keys) per txn and view on the device (ad_max_conflicts); what remains is a
clock read and a comparison, restated here from the reference:

* ``Timestamp`` order / bits        primitives/Timestamp.java:81-96, 208-227, 328-336
* ``NodeClock.unique_now``          Node.uniqueNow / uniqueNow(atLeast) / nowAtLeast, local/Node.java:335-375
* ``preaccept_witnessed_at``        CommandStore.preaccept, local/CommandStore.java:322-347: TxnId on the fast
                                    path (TxnId >= maxConflict and the txn's epoch is current), else
                                    time.uniqueNow(maxConflict).  The expiry / rejectBefore test and the
                                    ExclusiveSyncPoint branch (:326-333) are not modelled.

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
