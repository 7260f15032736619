"""CommandsForKeyTest.Canon + test(seed, minCount) restated — TEST INFRASTRUCTURE (the oracle for evolving CFK state).

The reference's only harness for CommandsForKey's execution-order release is a randomized canonical model driven by
DefaultRandom (test/local/cfk/CommandsForKeyTest.java:120-357 Canon, :590-646 test).  This module restates it
literally, RNG call for RNG call, over a restatement of the CommandsForKey state machine it drives:

* DefaultRandom / RandomSource        java.util.Random via tests/refgen.JavaRandom (WrappedRandomSource: nextInt(n),
                                      nextFloat, nextBoolean, nextLong from java.util.Random; nextInt(min, max) and
                                      nextLong(min, max) are RandomSource's defaults, utils/RandomSource.java:81-186)
* Canon                               CommandsForKeyTest.java:120-571 (TRANSITIONS :235-246 exactly, as SaveStatus)
* CommandsForKey.update               local/cfk/CommandsForKey.java:987-1057 + Updating.insertOrUpdate
                                      (local/cfk/Updating.java:99-358): byId, statuses, executeAt, the missing arrays
                                      (kept to their invariant: CommandsForKey.java:101-113, Utils.validateMissing
                                      Utils.java:42-63 — every uncommitted TxnId below depsKnownBefore the txn witnesses
                                      and does not have as a dependency), transitively known additions
* postProcess / notifyManaged         CommandsForKey.java:1121-1330 (the event-driven release: kinds, bounds, counters)
* registerUnmanaged / notifyUnmanaged Updating.updateUnmanaged :715-849, PostProcess.notifyUnmanaged :143-244,
                                      Utils.findCommit / findFirstApply / findApply :363-393
* WaitingOn                           local/Command.java:1225-1560 (key bit + direct range / key TxnId bits)

* Pruning (Run(prune=True), the reference's test(seed)): CommandsForKey.maybePrune / pruneBefore
                                      (local/cfk/Pruning.java:164-331) on rnd.decide(pruneChance) and after a loaded
                                      Applied command (SafeCommandsForKey.update :66-83); prunedBefore; loadingPruned
                                      (Pruning.LoadingPruned :50-114: pruned additions of an update, Updating.java:111-117,
                                      and pruned deps of an unmanaged, :803-815); the test's task queue
                                      (TestCommandStore.queue / runOneTask, CommandsForKeyTest.java:917-953) holding
                                      PostProcess.LoadPruned loads (-> CommandsForKey.updatePruned :998-1005) and
                                      Updating.updateUnmanagedAsync (:690-700) for unmanageds below prunedBefore;
                                      isWaitingOnPruned in notifyManaged (:1222), isAnyPredecessorWaitingOnPruned for
                                      sync points (Updating.java:796), loadingPruned's first TxnId bounding the commit
                                      notifications (PostProcess.java:171).
Deliberate limits, stated where they act:
* Run(prune=False) (the default, kept for the earlier tests) draws every rnd.decide(pruneChance) but never prunes, so no
  TxnId is ever below prunedBefore and the task queue stays empty.
* Order inside one harness step: CommandsForKeyUpdate.postProcess runs notifyManaged on the PRE-prune CFK and the
  notifier chain on the current (post-prune) one.  The restatement prunes after notifyManaged: pruning removes only
  Applied rows executing before the new prunedBefore (at or below maxAppliedWriteByExecuteAt) and invalidated rows, none
  of which notifyManaged reads (it starts after maxAppliedWrite, counts undecided rows, and reads missing() sets, which
  hold no committed TxnId), so its notifications are the same either way.
* Ballots are all ZERO (as in Canon), so the ballot-ordered CFK updates reduce to "the InternalStatus must rise".
No JVM exists here, so the stream cannot be compared with a Java run: parity of the stream itself is unpinned; what is
pinned is that the restated harness satisfies the reference's own invariants (:175-180, :208-218) on every seed run.
"""
import bisect
import collections

import numpy as np

import refgen

# ---- kinds, statuses ---------------------------------------------------------------------------------------------
READ, WRITE, EPH, SYNC, ESP = 0, 1, 2, 3, 4                   # Txn.Kind ordinals
KEY, RANGE = 0, 1
KINDS = (READ, WRITE, EPH, SYNC, ESP)                         # Canon.KINDS :125
_WITNESSES = {READ: {WRITE}, EPH: {WRITE}, WRITE: {READ, WRITE}, SYNC: {READ, WRITE},
              ESP: {READ, WRITE, SYNC, ESP}}                  # Txn.Kind.witnesses :221-235
_WITNESSED_BY = {EPH: set(), READ: {WRITE, SYNC, ESP}, WRITE: {READ, WRITE, SYNC, ESP},
                 SYNC: {ESP}, ESP: {ESP}}                     # Txn.Kind.witnessedBy :247-262
ANY_GLOBALLY_VISIBLE = {READ, WRITE, SYNC, ESP}


def witnesses(q, d):
    return d in _WITNESSES[q]


# SaveStatus (local/SaveStatus.java:55-87, the members Canon uses) -> Status ordinal (local/Status.java:49-...)
NOT_DEFINED, PRE_ACCEPTED, ACCEPTED_INVALIDATE, ACCEPTED_INVALIDATE_WD, ACCEPTED_SS, ACCEPTED_WD, COMMITTED_SS, \
    STABLE_SS, APPLIED_SS, INVALIDATED = range(10)
S_NOT_DEFINED, S_PRE_ACCEPTED, S_ACCEPTED_INVALIDATE, S_ACCEPTED, S_PRE_COMMITTED, S_COMMITTED, S_STABLE, \
    S_PRE_APPLIED, S_APPLIED, S_TRUNCATED, S_INVALIDATED = range(11)
STATUS_OF = {NOT_DEFINED: S_NOT_DEFINED, PRE_ACCEPTED: S_PRE_ACCEPTED, ACCEPTED_INVALIDATE: S_ACCEPTED_INVALIDATE,
             ACCEPTED_INVALIDATE_WD: S_ACCEPTED_INVALIDATE, ACCEPTED_SS: S_ACCEPTED, ACCEPTED_WD: S_ACCEPTED,
             COMMITTED_SS: S_COMMITTED, STABLE_SS: S_STABLE, APPLIED_SS: S_APPLIED, INVALIDATED: S_INVALIDATED}
# SaveStatus enum order for compareTo (Applied < ... < Invalidated)
SS_ORDER = {NOT_DEFINED: 1, PRE_ACCEPTED: 2, ACCEPTED_INVALIDATE: 3, ACCEPTED_INVALIDATE_WD: 4, ACCEPTED_SS: 5,
            ACCEPTED_WD: 6, COMMITTED_SS: 11, STABLE_SS: 12, APPLIED_SS: 15, INVALIDATED: 21}

# CommandsForKeyTest.Canon.TRANSITIONS :235-246, exactly
TRANSITIONS = {
    NOT_DEFINED: (PRE_ACCEPTED, ACCEPTED_INVALIDATE, ACCEPTED_INVALIDATE_WD, ACCEPTED_SS, ACCEPTED_WD, COMMITTED_SS,
                  STABLE_SS, INVALIDATED),
    PRE_ACCEPTED: (ACCEPTED_INVALIDATE_WD, ACCEPTED_WD, COMMITTED_SS, STABLE_SS, INVALIDATED),
    ACCEPTED_INVALIDATE: (INVALIDATED,),
    ACCEPTED_INVALIDATE_WD: (INVALIDATED,),
    ACCEPTED_SS: (COMMITTED_SS, STABLE_SS, INVALIDATED),
    ACCEPTED_WD: (COMMITTED_SS, STABLE_SS, INVALIDATED),
    COMMITTED_SS: (STABLE_SS,),
    STABLE_SS: (APPLIED_SS,),
}

# CommandsForKey.InternalStatus :493-528 (ordinals = the C-ABI's AD_ST_*)
TK, HISTORICAL, PREACC, ACC, COMMITTED, STABLE, APPLIED, INVALID = range(8)
_INTERNAL = {PRE_ACCEPTED: PREACC, ACCEPTED_INVALIDATE_WD: PREACC, ACCEPTED_SS: ACC, ACCEPTED_WD: ACC,
             COMMITTED_SS: COMMITTED, STABLE_SS: STABLE, APPLIED_SS: APPLIED, INVALIDATED: INVALID}


def has_deps(st):                                   # InternalStatus.hasExecuteAtOrDeps
    return st in (ACC, COMMITTED, STABLE, APPLIED)


# ---- timestamps ----------------------------------------------------------------------------------------------------
# A Timestamp / TxnId is (epoch, hlc, identity flags, node): tuple order == Timestamp.compareTo (:208-217) and tuple
# equality == Timestamp.equals (identity bits only).  TxnId domains live in DOMAIN (identity excludes the domain bit).
NONE = (0, 0, 0, 0)
MAX = (1 << 49, 0, 0, 1 << 62)


def txn_id(epoch, hlc, kind, domain, node, domains):
    t = (epoch, hlc, kind << 1, node)
    domains[t] = domain
    return t


def ts_from_values(epoch, hlc, node):               # Timestamp.fromValues: flags 0
    return (epoch, hlc, 0, node)


def kind_of(t):
    return t[2] >> 1


class Rnd:
    """DefaultRandom (utils/DefaultRandom.java:23-38) = WrappedRandomSource over java.util.Random."""

    def __init__(self, seed):
        self.r = refgen.JavaRandom(seed)

    def next_float(self):
        return refgen.next_float(self.r)

    def decide(self, chance):                         # RandomSource.decide(float) :63-66
        return self.next_float() < chance

    def next_boolean(self):
        return self.r.nextBoolean()

    def next_int(self, a, b=None):
        return self.r.nextInt(a) if b is None else self.r.nextInt(a, b)

    def _next_long_signed(self):
        v = self.r.nextLong()
        return v - (1 << 64) if v >= 1 << 63 else v

    def next_long(self, lo, hi):                      # RandomSource.nextLong(min, max) :150-176
        M = 1 << 64

        def s64(x):
            x &= M - 1
            return x - M if x >= 1 << 63 else x

        result = self._next_long_signed()
        delta = s64(hi - lo)
        mask = s64(delta - 1)
        if delta & mask == 0:
            return s64((result & mask) + lo)
        if delta > 0:
            u = (result & (M - 1)) >> 1
            while True:
                result = u % delta
                if s64(u + mask - result) >= 0:
                    return result + lo
                u = (self._next_long_signed() & (M - 1)) >> 1
        while result < lo or result >= hi:
            result = self._next_long_signed()
        return result

    def pick(self, seq):
        return seq[self.r.nextInt(len(seq))]


class SortedMap:
    """The TreeMap / TreeSet operations Canon uses, over tuple keys."""

    def __init__(self):
        self.keys = []
        self.vals = {}

    def __contains__(self, k):
        return k in self.vals

    def __len__(self):
        return len(self.keys)

    def get(self, k):
        return self.vals.get(k)

    def put(self, k, v=True):
        if k not in self.vals:
            bisect.insort(self.keys, k)
        self.vals[k] = v

    def remove(self, k):
        if k in self.vals:
            del self.vals[k]
            self.keys.pop(bisect.bisect_left(self.keys, k))

    def last_key(self):
        return self.keys[-1]

    def first_key(self):
        return self.keys[0]

    def floor(self, k):
        i = bisect.bisect_right(self.keys, k)
        return self.keys[i - 1] if i else None

    def head(self, k, inclusive=False):               # headMap(k, inclusive) keys, ascending
        return self.keys[:bisect.bisect_right(self.keys, k) if inclusive else bisect.bisect_left(self.keys, k)]

    def tail(self, k, inclusive=False):               # tailMap(k, inclusive)
        return self.keys[bisect.bisect_left(self.keys, k) if inclusive else bisect.bisect_right(self.keys, k):]

    def sub(self, lo, hi):                            # subMap(lo, false, hi, false)
        return self.keys[bisect.bisect_right(self.keys, lo):bisect.bisect_left(self.keys, hi)]


# ---- commands ------------------------------------------------------------------------------------------------------
class WaitingOn:
    """Command.WaitingOn restricted to Canon's one key: the key bit + the direct range / key TxnId bits."""
    __slots__ = ("has_key", "key", "txns")

    def __init__(self, has_key, key, txns):
        self.has_key = has_key        # keyDeps has the key (keys.size() > 0)
        self.key = key                # waiting on the key
        self.txns = txns              # frozenset of TxnIds still waited on

    def waiting(self):
        return self.key or bool(self.txns)


class Command:
    __slots__ = ("txn", "ss", "execute_at", "deps", "waiting_on")

    def __init__(self, txn, ss, execute_at, deps=None, waiting_on=None):
        self.txn, self.ss, self.execute_at, self.deps, self.waiting_on = txn, ss, execute_at, deps, waiting_on

    def status(self):
        return STATUS_OF[self.ss]

    def has_been(self, s):
        return STATUS_OF[self.ss] >= s

    def execute_at_if_known(self, or_else):          # Command.executeAtIfKnown :552-557 (ExecuteAtKnown)
        return self.execute_at if self.ss in (COMMITTED_SS, STABLE_SS, APPLIED_SS) else or_else


class Canon:
    """CommandsForKeyTest.Canon (:120-571), the NotifySink of the CFK."""
    MIN_ARGS = (1, 1, READ, KEY, 1)

    def __init__(self, rnd, domains):
        self.rnd = rnd
        self.domains = domains
        self.node_ids = list(range(1, 11))
        self.MIN = txn_id(*self.MIN_ARGS, domains)
        self.unwitnessed = SortedMap()
        self.undecided = SortedMap()
        self.candidates = SortedMap()
        self.unfinished = SortedMap()
        self.by_id = SortedMap()
        self.committed_by_execute_at = SortedMap()
        self.execute_ats = set()
        self.closing = False
        self.undecided_count = 0          # declared in the reference and never assigned (:137): always 0
        self.notified = []                # (txnId, key-bit cleared?) of every notWaiting call, in order
        self.ready_events = []            # txnIds that readyToExecute admitted

    def domain(self, t):
        return self.domains[t]

    def manages(self, t):                 # CommandsForKey.manages :185-188
        return self.domains[t] == KEY and kind_of(t) in ANY_GLOBALLY_VISIBLE

    def manages_execution(self, t):       # CommandsForKey.managesExecution :196-199
        return self.domains[t] == KEY and kind_of(t) in (READ, WRITE)

    # -- set / readyToExecute / removeWaitingOn / notWaiting (:141-222)
    def set(self, prev, nxt):
        self.by_id.put(nxt.txn, nxt)
        if nxt.has_been(S_COMMITTED):
            self.undecided.remove(nxt.txn)
            self.committed_by_execute_at.put(nxt.execute_at, nxt)
            if nxt.has_been(S_STABLE):
                if prev.ss != nxt.ss:
                    self.candidates.remove(nxt.txn)
                if nxt.has_been(S_APPLIED):
                    self.unfinished.remove(nxt.txn)
                    if not self.manages_execution(nxt.txn):
                        self.remove_waiting_on(nxt.txn, MAX)
                else:
                    if not nxt.waiting_on.waiting() and (not prev.has_been(S_STABLE) or prev.waiting_on.waiting()):
                        self.ready_to_execute(nxt)
            if nxt.has_been(S_COMMITTED) and not prev.has_been(S_COMMITTED) and not nxt.has_been(S_INVALIDATED):
                if nxt.execute_at != nxt.txn and not self.manages(nxt.txn):
                    self.remove_waiting_on(nxt.txn, nxt.execute_at)

    def ready_to_execute(self, committed):
        for ex in self.committed_by_execute_at.head(committed.execute_at):
            pred = self.committed_by_execute_at.get(ex)
            assert pred.has_been(S_APPLIED) or not witnesses(kind_of(committed.txn), kind_of(pred.txn)), \
                "readyToExecute invariant (:177-178): %s before %s" % (pred.txn, committed.txn)
        self.candidates.put(committed.txn)
        self.ready_events.append(committed.txn)

    def remove_waiting_on(self, waiting_id, until):
        for ex in list(self.committed_by_execute_at.sub(waiting_id, until)):
            command = self.committed_by_execute_at.get(ex)
            if not command.has_been(S_STABLE):
                continue
            w = command.waiting_on
            if waiting_id in w.txns:
                self.set(command, Command(command.txn, command.ss, command.execute_at, command.deps,
                                          WaitingOn(w.has_key, w.key, w.txns - {waiting_id})))

    def not_waiting(self, txn):
        prev = self.by_id.get(txn)
        w = prev.waiting_on
        cleared = w.key
        self.notified.append((txn, cleared))
        if not cleared:
            return
        pk = kind_of(txn)
        if pk not in (ESP, EPH):                       # !awaitsOnlyDeps (:208-212)
            for ex in self.committed_by_execute_at.head(prev.execute_at):
                c = self.committed_by_execute_at.get(ex)
                assert self.domains[c.txn] == RANGE or not witnesses(pk, kind_of(c.txn)) \
                    or SS_ORDER[c.ss] >= SS_ORDER[APPLIED_SS], "notWaiting invariant (:211): %s before %s" % (c.txn, txn)
        if self.domains[txn] == KEY:                  # (:214-218)
            for ex in self.committed_by_execute_at.tail(prev.execute_at):
                c = self.committed_by_execute_at.get(ex)
                if kind_of(c.txn) in (ESP, EPH) or not witnesses(kind_of(c.txn), pk) or SS_ORDER[c.ss] < SS_ORDER[STABLE_SS]:
                    continue
                assert c.waiting_on.has_key, "isWaitingOnKey(0) on a command without keys"
                assert c.waiting_on.key, "notWaiting invariant (:217): %s after %s released" % (c.txn, txn)
        self.set(prev, Command(prev.txn, prev.ss, prev.execute_at, prev.deps, WaitingOn(w.has_key, False, w.txns)))

    # -- the generator (:264-571)
    def is_done(self):
        return self.closing and len(self.unfinished) == 0

    def close(self):
        self.closing = True

    def update(self, has_waiting_tasks):
        rnd = self.rnd
        generate = (not self.closing) and rnd.decide(np.float32(1.0) / np.float32(1 + self.undecided_count))
        if not generate and len(self.candidates) == 0 and has_waiting_tasks:
            return None
        assert len(self.candidates) > 0 or len(self.unfinished) == len(self.unwitnessed)
        prev = self.unwitnessed_cmd(self.generate_id()) if generate or len(self.candidates) == 0 \
            else self.select_one(self.candidates)
        invalidate = False
        if kind_of(prev.txn) == ESP and not prev.has_been(S_COMMITTED):
            for t in self.by_id.tail(prev.txn):
                c = self.by_id.get(t)
                if c.has_been(S_COMMITTED) and witnesses(kind_of(c.txn), kind_of(prev.txn)):
                    invalidate = True
                    break
        nxt = self.update_to(prev, INVALIDATED) if invalidate else self.update_cmd(prev)
        self.set(prev, nxt)
        self.unwitnessed.remove(nxt.txn)
        return prev, nxt

    def update_cmd(self, prev):
        cands = TRANSITIONS[prev.ss]
        return self.update_to(prev, cands[self.rnd.next_int(len(cands))])

    def update_to(self, prev, new):
        t = prev.txn
        if new == PRE_ACCEPTED:
            return Command(t, PRE_ACCEPTED, t)
        if new in (ACCEPTED_SS, ACCEPTED_WD):
            ex = self.generate_execute_at(t)
            return self.accepted(t, ex, new)
        if new in (ACCEPTED_INVALIDATE, ACCEPTED_INVALIDATE_WD):
            return Command(t, new, t)
        if new == COMMITTED_SS:
            ex = prev.execute_at_if_known(self.generate_execute_at(t))
            return Command(t, COMMITTED_SS, ex, self.generate_deps(t, ex, S_COMMITTED))
        if new == STABLE_SS:
            ex = prev.execute_at_if_known(self.generate_execute_at(t))
            committed = prev if prev.has_been(S_COMMITTED) else None
            deps = self.generate_deps(t, ex, S_STABLE) if committed is None else committed.deps
            return Command(t, STABLE_SS, ex, deps, self.initialise_waiting_on(t, ex, deps))
        if new == APPLIED_SS:
            ex = prev.execute_at_if_known(self.generate_execute_at(t))
            committed = prev if prev.has_been(S_COMMITTED) else None
            deps = self.generate_deps(t, ex, S_APPLIED) if committed is None else committed.deps
            w = self.initialise_waiting_on(t, ex, deps) if committed is None or committed.waiting_on is None \
                else committed.waiting_on
            return Command(t, APPLIED_SS, ex, deps, w)
        if new == INVALIDATED:
            return Command(t, INVALIDATED, NONE)
        raise AssertionError(new)

    def accepted(self, t, ex, ss):
        return Command(t, ss, ex, self.generate_deps(t, t, S_ACCEPTED))

    def generate_deps(self, t, execute_at, for_status):
        self.maybe_generate_unwitnessed()
        need = S_COMMITTED if for_status <= S_ACCEPTED else S_ACCEPTED
        deps = []
        for d in self.by_id.head(execute_at):
            if d == t or not witnesses(kind_of(t), kind_of(d)):
                continue
            c = self.by_id.get(d)
            if c.has_been(need) or self.rnd.next_boolean():
                self.unwitnessed.remove(d)
                deps.append(d)
        return tuple(deps)

    def generate_execute_at(self, t):
        if kind_of(t) in (ESP, EPH):                  # awaitsOnlyDeps
            return t
        lo = NONE
        if len(self.committed_by_execute_at):
            last = self.committed_by_execute_at.get(self.committed_by_execute_at.last_key()).execute_at
            lo = ts_from_values(last[0], last[1] + 1, last[3])
        if lo <= t and self.rnd.next_boolean():
            return t
        lo = max(lo, ts_from_values(t[0], t[1] + 1, t[3]))
        hi = ts_from_values(lo[0], lo[1] + 100, lo[3])
        ex = self.generate_timestamp(lo, hi)
        assert ex >= t
        self.execute_ats.add(ex)
        return ex

    def maybe_generate_unwitnessed(self):
        chance = np.float32(1.0) / np.float32(1 + len(self.unwitnessed))          # 1 / (1f + size), in float
        count = self.rnd.next_int(0, 3) if self.rnd.decide(chance) else 0
        while count > 0:
            count -= 1
            nxt = self.generate_id()
            self.by_id.put(nxt, self.unwitnessed_cmd(nxt))

    def generate_id(self):
        lo = self.MIN
        if len(self.by_id) == 0:
            hi = txn_id(1, 100, READ, KEY, self.node_ids[0], self.domains)
        else:
            hi = self.by_id.get(self.by_id.last_key()).txn
            case = self.rnd.next_int(3)
            if case == 2:
                lo = hi
            if case >= 1:
                hi = txn_id(hi[0], hi[1] + 100, kind_of(hi), self.domains[hi], hi[3], self.domains)
        return self.generate_id_between(lo, hi, True)

    def generate_id_between(self, lo, hi, unique):
        r = self._generate_id(lo, hi)
        while unique and (r in self.by_id or r in self.execute_ats):
            r = self._generate_id(lo, hi)
        return r

    def _pick_node(self, lo, hi, hlc):
        if hlc == lo[1]:
            return lo[3] if lo[3] == len(self.node_ids) + 1 else self.node_ids[self.rnd.next_int(lo[3] - 1, len(self.node_ids))]
        if hlc == hi[1]:
            return hi[3] if hi[3] == 1 else self.node_ids[self.rnd.next_int(0, hi[3] - 1)]
        return self.rnd.pick(self.node_ids)

    def _generate_id(self, lo, hi):
        rnd = self.rnd
        epoch = lo[0] if lo[0] == hi[0] else rnd.next_long(lo[0], hi[0])
        hlc = lo[1] if lo[1] == hi[1] else rnd.next_long(lo[1], hi[1])
        node = self._pick_node(lo, hi, hlc)
        if hlc == lo[1]:
            kind = kind_of(lo)
        elif hlc == hi[1]:
            kind = kind_of(hi)
        else:
            kind = rnd.pick(KINDS)
        if hlc == lo[1] and self.domains[lo] == RANGE:
            dom = RANGE
        elif hlc == hi[1] and self.domains[hi] == KEY:
            dom = KEY
        else:
            dom = KEY if rnd.next_boolean() else RANGE
        t = (epoch, hlc, kind << 1, node)
        # identity excludes the domain bit: an id equal to a known txn keeps that txn's domain (the caller then
        # regenerates it, or uses it only as a floor() bound)
        if t not in self.by_id:
            self.domains[t] = dom
        return t

    def generate_timestamp(self, lo, hi):
        r = self._generate_timestamp(lo, hi)
        while r in self.by_id or r in self.execute_ats:
            r = self._generate_timestamp(lo, hi)
        return r

    def _generate_timestamp(self, lo, hi):
        rnd = self.rnd
        epoch = lo[0] if lo[0] == hi[0] else rnd.next_long(lo[0], hi[0])
        hlc = lo[1] if lo[1] == hi[1] else rnd.next_long(lo[1], hi[1])
        node = self._pick_node(lo, hi, hlc)
        r = ts_from_values(epoch, hlc, node)
        assert r >= lo
        return r

    def unwitnessed_cmd(self, t):
        for s in (self.unwitnessed, self.undecided, self.candidates, self.unfinished):
            s.put(t)
        return Command(t, NOT_DEFINED, None)

    def initialise_waiting_on(self, t, execute_at, deps):
        """WaitingOn.Update.initialise (Command.java:1427-1435) over Canon's one key / one range, then Canon's removal of
        applied deps and of deps committed to execute after (:547-558)."""
        has_key = any(self.manages_execution(d) for d in deps)        # keyDeps.keys() holds KEY
        direct = [d for d in deps if not self.manages_execution(d)]   # rangeDeps + directKeyDeps
        waiting = set(direct)
        for d in direct:
            c = self.by_id.get(d)
            if c.has_been(S_APPLIED) or (c.has_been(S_COMMITTED) and c.execute_at > execute_at):
                waiting.discard(d)
        return WaitingOn(has_key, has_key, frozenset(waiting))

    def select_one(self, frm):
        bound = self.generate_id_between(frm.first_key(), frm.last_key(), False)
        return self.by_id.get(frm.floor(bound))


# ---- CommandsForKey --------------------------------------------------------------------------------------------------
class Info:
    __slots__ = ("txn", "status", "execute_at", "missing", "deps")

    def __init__(self, txn, status, execute_at, missing=None, deps=None):
        self.txn, self.status, self.execute_at = txn, status, execute_at
        self.missing = missing if missing is not None else set()
        self.deps = deps

    def deps_known_before(self):                      # InternalStatus.depsKnownBefore :561-580
        return self.execute_at if self.status in (COMMITTED, STABLE, APPLIED) else self.txn


COMMIT_P, APPLY_P = 0, 1                              # Unmanaged.Pending
# ops of the device event log (CFK.log entries (txnId, InternalStatus, executeAt, deps[, op[, interval, hlcDelta]]))
OP_UPDATE, OP_LOAD, OP_PRUNE, OP_LOADING, OP_UNMANAGED, OP_UNMANAGED_RECHECK = 0, 1, 2, 3, 4, 5


class CFK:
    """One key's CommandsForKey: byId Infos, unmanageds, prunedBefore, loadingPruned; the derived committedByExecuteAt,
    minUndecidedById and maxAppliedWriteByExecuteAt are recomputed from byId as the constructor does (:642-681)."""

    def __init__(self, domains):
        self.domains = domains
        self.ids = []
        self.info = {}
        self.unmanageds = []                          # sorted (pending, waitingUntil, txnId)
        self.log = None                               # list: the CommandsForKey.update calls as device events
        self.notes = None                             # with log: the unmanaged notifications, (tag, TxnId) in order —
                                                      # 0 notifyUnmanaged commit, 1 notifyUnmanaged applied, 2 ready
        self.pruned_before = NONE                     # prunedBefore's TxnId (NO_INFO: TxnId.NONE)
        self.loading = {}                             # loadingPruned: TxnId -> witnessedBy (sorted tuple)
        self.last_load = ()                           # the TxnIds the last update / updateUnmanaged asked to load
        self.prunes = 0                               # pruneBefore calls that removed rows

    def copy(self):
        c = CFK(self.domains)
        c.ids = list(self.ids)
        c.info = {t: Info(i.txn, i.status, i.execute_at, set(i.missing), i.deps) for t, i in self.info.items()}
        c.unmanageds = list(self.unmanageds)
        c.pruned_before, c.loading = self.pruned_before, dict(self.loading)
        return c

    def manages(self, t):                             # CommandsForKey.manages :185-188
        return self.domains[t] == KEY and kind_of(t) in ANY_GLOBALLY_VISIBLE

    def _load_pruned(self, ids, witness):             # Pruning.loadPruned :79-94 (witnessedBy merged by linearUnion)
        for d in ids:
            w = set(self.loading.get(d, ()))
            if witness is not None:
                w.add(witness)
            self.loading[d] = tuple(sorted(w))

    def waiting_on_pruned(self, waiting, execute_at):  # Pruning.isWaitingOnPruned :119-135
        return any(lid < execute_at and self.me(lid) and waiting in w for lid, w in self.loading.items())

    def any_predecessor_waiting_on_pruned(self, waiting):   # Pruning.isAnyPredecessorWaitingOnPruned :140-157
        return any(lid < waiting and self.me(lid) and w and waiting >= w[0] for lid, w in self.loading.items())

    def me(self, t):
        return self.domains[t] == KEY and kind_of(t) in (READ, WRITE)

    def committed(self):
        c = [self.info[t] for t in self.ids if self.info[t].status in (COMMITTED, STABLE, APPLIED)]
        c.sort(key=lambda i: i.execute_at)
        return c

    def min_undecided(self):
        for idx, t in enumerate(self.ids):
            i = self.info[t]
            if i.status < COMMITTED and self.me(t):
                return idx
        return -1

    @staticmethod
    def max_applied_write(committed):
        for k in range(len(committed) - 1, -1, -1):
            if committed[k].status == APPLIED and kind_of(committed[k].txn) == WRITE:
                return k
        return -1

    def _insert(self, info):
        bisect.insort(self.ids, info.txn)
        self.info[info.txn] = info

    def _add_missing_everywhere(self, a, skip=None, do_not_insert=()):
        """a (uncommitted, newly known) joins the missing array of every txn with deps that witnesses it and whose
        depsKnownBefore is above it (Utils.addToMissingArrays :97-172, Updating.insertOrUpdateWithAdditions :385-450),
        except the members of do_not_insert (a loaded pruned TxnId's witnessedBy, Updating.java:351)."""
        ka = kind_of(a)
        for u in self.info.values():
            if u.txn == a or u.txn == skip or not has_deps(u.status) or u.txn in do_not_insert:
                continue
            if witnesses(kind_of(u.txn), ka) and u.deps_known_before() > a:
                u.missing.add(a)

    def _remove_missing_everywhere(self, a):           # Utils.removeFromMissingArrays :70-95
        for u in self.info.values():
            u.missing.discard(a)

    def update(self, cmd, was_pruned=False):
        """CommandsForKey.update (:987-1057) for a managed command, or updatePruned (:998-1005) for a loaded pruned one
        -> (changed, curInfo status, newInfo); self.last_load = the pruned additions to load (LoadPruned)."""
        self.last_load = ()
        new = _INTERNAL.get(cmd.ss)
        t = cmd.txn
        if was_pruned:
            if new is None:
                new = TK
            if not self.manages(t):
                new = TK if new < COMMITTED else INVALID
        elif new is None:
            return False, None, None
        loading_for = self.loading.get(t)             # loadingPrunedFor(loadingPruned, txnId, null)
        was_pruned = was_pruned or loading_for is not None
        if self.log is not None:                      # (txnId, InternalStatus, executeAt, deps) as ad_cfk_store_apply takes it
            if was_pruned:
                self.log.append((t, new, cmd.execute_at if has_deps(new) else t, (), OP_LOAD))
            else:
                self.log.append((t, new, cmd.execute_at if has_deps(new) else t, tuple(cmd.deps) if has_deps(new) else ()))
        cur = self.info.get(t)
        if cur is not None and new <= cur.status:      # ballots ZERO: only a higher InternalStatus updates
            return False, None, None
        cur_status = cur.status if cur is not None else None
        if was_pruned:                                # TxnInfo.create: no missing(), no additions (:1024, :1053)
            ex = cmd.execute_at if has_deps(new) else t
            if loading_for is not None:               # insertOrUpdate :295
                del self.loading[t]
            if cur is None:
                self._insert(Info(t, new, ex))
            else:
                cur.status, cur.execute_at, cur.missing, cur.deps = new, ex, set(), None
            was_committed = cur_status is not None and cur_status in (COMMITTED, STABLE, APPLIED)
            if new in (COMMITTED, STABLE, APPLIED) and not was_committed:          # :340-343
                self._remove_missing_everywhere(t)
            elif cur is not None and cur_status < COMMITTED and new == INVALID:
                self._remove_missing_everywhere(t)
            elif cur is None and new != INVALID:
                self._add_missing_everywhere(t, do_not_insert=loading_for or ())
            return True, cur_status, self.info[t]
        if has_deps(new):
            ex = cmd.execute_at
            deps = cmd.deps
            dkb = ex if new in (COMMITTED, STABLE, APPLIED) else t
            dep_set = set(deps)
            kt = kind_of(t)
            missing = set()
            for u in self.ids:
                if u == t or u >= dkb:
                    continue
                iu = self.info[u]
                if iu.status < COMMITTED and witnesses(kt, kind_of(u)) and u not in dep_set:
                    missing.add(u)
            additions = [d for d in deps if d not in self.info]
            pruned = [d for d in additions if d < self.pruned_before]       # Utils.removePrunedAdditions :229-244
            if pruned:
                additions = [d for d in additions if d >= self.pruned_before]
                self._load_pruned(pruned, t)
                self.last_load = tuple(pruned)
            for a in additions:                       # TRANSITIVELY_KNOWN additions (:178-227)
                self._insert(Info(a, TK, a))
            if cur is None:
                self._insert(Info(t, new, ex, missing, deps))
            else:
                cur.status, cur.execute_at, cur.missing, cur.deps = new, ex, missing, deps
            for a in additions:
                self._add_missing_everywhere(a, skip=t)
            if cur is None and new < COMMITTED:        # insertSelfMissing
                self._add_missing_everywhere(t)
            if cur is not None and cur_status < COMMITTED and new >= COMMITTED:     # removeSelfMissing
                self._remove_missing_everywhere(t)
            new_info = self.info[t]
        else:
            if cur is None:
                self._insert(Info(t, new, t))
                if new != INVALID:
                    self._add_missing_everywhere(t)
            else:
                cur.status, cur.execute_at, cur.missing, cur.deps = new, t, set(), None
                if cur_status < COMMITTED and new == INVALID:
                    self._remove_missing_everywhere(t)
            new_info = self.info[t]
        return True, cur_status, new_info

    # -- CommandsForKey.mapReduceActive (:925-983), as PreAccept.calculatePartialDeps asks it (PreAccept.java:245-267)
    def map_reduce_active(self, started_before, kinds, exclude=None):
        """The TxnIds mapReduceActive hands the builder for a query with bound `started_before` witnessing `kinds`,
        minus `exclude` (calculatePartialDeps' own TxnId when the bound is its executeAt), ascending and unique (the
        Deps.Builder's sorted set)."""
        end = bisect.bisect_left(self.ids, started_before)            # insertPos :1373-1378
        committed = self.committed()                                  # committedByExecuteAt :660-667
        maw = self.max_applied_write(committed)
        i = bisect.bisect_left([c.execute_at for c in committed], started_before) - 1   # :930-941 (last < bound)
        while i >= 0 and kind_of(committed[i].txn) != WRITE:
            i -= 1
        mcwb = committed[i].execute_at if i >= 0 else None
        out = set()
        for t in self.ids[:end]:                                      # :945-965
            if kind_of(t) not in kinds:
                continue
            inf = self.info[t]
            if inf.status in (COMMITTED, STABLE, APPLIED):
                if mcwb is not None and inf.execute_at < mcwb and kind_of(t) in (READ, WRITE):
                    continue                                          # ELIDE_TRANSITIVE_DEPENDENCIES, Write.witnesses
            elif inf.status in (TK, INVALID):
                continue
            out.add(t)
        if started_before <= self.pruned_before and maw >= 0:          # :967-980
            j = bisect.bisect_left([c.execute_at for c in committed[:maw]], started_before)
            while kind_of(committed[j].txn) != WRITE:
                j += 1
            out.add(committed[j].txn)
        out.discard(exclude)
        return sorted(out)

    # -- Pruning.maybePrune / pruneBefore (Pruning.java:164-331)
    def maybe_prune(self, prune_interval, min_hlc_delta):
        if self.log is not None:
            self.log.append((NONE, 0, NONE, (), OP_PRUNE, prune_interval, min_hlc_delta))
        committed = self.committed()
        i = self.max_applied_write(committed)
        if i < prune_interval:                        # maxAppliedWriteByExecuteAt < pruneInterval (-1 when none)
            return False
        max_prune_hlc = committed[i].execute_at[1] - min_hlc_delta
        i -= 1
        while i >= 0:
            x = committed[i]
            if kind_of(x.txn) == WRITE and x.execute_at[1] <= max_prune_hlc and x.status == APPLIED:
                break
            i -= 1
        if i < 0:
            return False
        npb = committed[i]
        if npb.txn <= self.pruned_before:
            return False
        pos = bisect.bisect_left(self.ids, npb.txn)   # insertPos
        if pos == 0:
            return False
        return self._prune_before(npb, pos)

    def _prune_before(self, npb, pos):
        """Removes the Applied rows before npb (in TxnId and executeAt) whose missing() the later retained rows cover, and
        the invalidated rows before it (:199-297); prunedBefore = npb."""
        merged = set(npb.missing)
        remove = []
        for k in range(pos):
            x = self.info[self.ids[k]]
            if x.status == INVALID:
                remove.append(x.txn)
            elif x.status == APPLIED and x.execute_at < npb.execute_at:
                if not x.missing or x.missing <= merged:
                    remove.append(x.txn)
                elif x.execute_at == x.txn:
                    merged |= x.missing
        if not remove:                                # pos == retainCount: unchanged (prunedBefore not advanced)
            return False
        gone = set(remove)
        self.ids = [t for t in self.ids if t not in gone]
        for t in remove:
            del self.info[t]
        self.pruned_before = npb.txn
        self.prunes += 1
        return True

    # -- notifyUnmanaged (PostProcess.java:143-244)
    def notify_unmanaged(self, cur_status, new_info):
        commit_notify, apply_notify = [], []
        mu = self.min_undecided()
        bound = self.ids[mu] if mu >= 0 else MAX
        if self.loading:                              # PostProcess.java:171
            bound = min(bound, min(self.loading))
        end = 0
        while end < len(self.unmanageds) and self.unmanageds[end][0] == COMMIT_P and bound > self.unmanageds[end][1]:
            end += 1
        if end > 0:
            commit_notify = [u[2] for u in self.unmanageds[:end]]
            self.unmanageds = self.unmanageds[end:]
            if self.notes is not None:
                self.notes.extend((0, u) for u in commit_notify)
        if new_info.status >= APPLIED:
            committed = self.committed()
            k = self.max_applied_write(committed) + 1
            while k < len(committed) and (committed[k].status == APPLIED or not self.me(committed[k].txn)):
                k += 1
            mca = committed[k - 1] if k - 1 >= 0 else None
            if mca is not None and mca.execute_at < new_info.execute_at:
                mca = None
            if mca is not None:
                start = 0
                while start < len(self.unmanageds) and self.unmanageds[start][0] == COMMIT_P:
                    start += 1
                e = start
                while e < len(self.unmanageds) and mca.execute_at >= self.unmanageds[e][1]:
                    e += 1
                if start != e:
                    apply_notify = [u[2] for u in self.unmanageds[start:e]]
                    self.unmanageds = self.unmanageds[:start] + self.unmanageds[e:]
                    if self.notes is not None:
                        self.notes.extend((1, u) for u in apply_notify)
        assert not (new_info.status == INVALID and cur_status is not None and cur_status in (COMMITTED, STABLE, APPLIED))
        return commit_notify, apply_notify

    # -- notifyManaged (CommandsForKey.java:1121-1289)
    def post_process(self, prev_status, cmd, sink):
        if cmd is None or not cmd.has_been(S_COMMITTED) or not self.me(cmd.txn):
            return
        t = cmd.txn
        new_info = self.info[t]
        new_status = new_info.status
        prev_status = TK if prev_status is None else prev_status
        committed = self.committed()
        idx = -1 if new_status == INVALID else committed.index(new_info)
        any_at = -1
        if prev_status < COMMITTED:
            kinds = _WITNESSED_BY[kind_of(t)]
            if new_status in (INVALID, APPLIED):
                to = len(committed)
            elif new_status == COMMITTED:
                to = idx
            elif new_status == STABLE:
                to, any_at = idx + 1, idx
            else:
                raise AssertionError("committed command with InternalStatus %d" % new_status)
        elif new_status == APPLIED:
            kinds, to = _WITNESSED_BY[kind_of(t)], len(committed)
        elif new_status == INVALID and prev_status != INVALID:
            kinds, to = ANY_GLOBALLY_VISIBLE, len(committed)
        else:
            if new_status != STABLE:
                return
            any_at, kinds, to = idx, ANY_GLOBALLY_VISIBLE, idx + 1
        self.notify_managed(committed, kinds, to, any_at, sink)

    def notify_managed(self, committed, kinds, to, any_at, sink):
        mu = self.min_undecided()
        undecided_index = len(self.ids) if mu < 0 else mu
        min_undecided = self.ids[mu] if mu >= 0 else None
        counters = 0
        for i in range(self.max_applied_write(committed) + 1, to):
            txn = committed[i]
            if txn.status == APPLIED or not self.me(txn.txn):
                continue
            kind = kind_of(txn.txn)
            if (kind in kinds or i == any_at) and not self.waiting_on_pruned(txn.txn, txn.execute_at):
                if txn.status == STABLE:
                    if undecided_index < len(self.ids):
                        nxt = bisect.bisect_left(self.ids, txn.execute_at, undecided_index)
                        while undecided_index < nxt:
                            b = self.info[self.ids[undecided_index]]
                            undecided_index += 1
                            if b.status >= COMMITTED or not self.me(b.txn):
                                continue
                            counters += unapplied_delta(kind_of(b.txn))
                    expect = unapplied_count(counters, kind)
                    if missing_count(txn, min_undecided, self.me) == expect:
                        sink(txn.txn)
            counters += unapplied_delta(kind)
            if kind == WRITE:
                return

    # -- updateUnmanaged (Updating.java:715-849)
    def update_unmanaged(self, cmd, sink, register, add_list=None):
        self.last_load = ()
        if cmd.has_been(S_TRUNCATED):
            return
        wt, wex = cmd.txn, cmd.execute_at
        wk = kind_of(wt)
        tx = [d for d in cmd.deps if self.me(d)]      # partialDeps.keyDeps.txnIds(key)
        missing = []
        if tx:
            ready_to_apply = waiting_to_apply = True
            executes_at = None
            i = 0
            j = bisect.bisect_left(self.ids, tx[0])

            def consider(t):
                nonlocal ready_to_apply, waiting_to_apply, executes_at
                if t.status < COMMITTED:
                    waiting_to_apply = ready_to_apply = False
                elif t.status != INVALID and (t.execute_at < wex or wk == EPH or (wk == ESP and t.txn < wt)):
                    ready_to_apply &= t.status == APPLIED
                    executes_at = t.execute_at if executes_at is None else max(executes_at, t.execute_at)

            while i < len(tx):
                c = -1 if j == len(self.ids) else (0 if tx[i] == self.ids[j] else (1 if tx[i] > self.ids[j] else -1))
                if c == 0:
                    consider(self.info[self.ids[j]])
                    i += 1
                    j += 1
                elif c > 0:
                    if wk in (SYNC, ESP):
                        t = self.info[self.ids[j]]
                        if self.me(t.txn):
                            consider(t)
                    j += 1
                elif not self.me(tx[i]):
                    i += 1
                elif register:
                    ready_to_apply = waiting_to_apply = False
                    missing.append(tx[i])
                    i += 1
                else:
                    assert tx[i] < self.pruned_before, "unmanaged dependency %s unknown to the CFK" % (tx[i],)
                    i += 1
            if wk in (SYNC, ESP) and self.any_predecessor_waiting_on_pruned(wt):      # :796-797
                ready_to_apply = waiting_to_apply = False
            if not ready_to_apply:
                pruned = [a for a in missing if a < self.pruned_before]            # :806-815
                if pruned:
                    missing = missing[len(pruned):]
                    self._load_pruned(pruned, wt)
                    if self.log is not None:
                        for a in pruned:
                            self.log.append((a, 0, a, (wt,), OP_LOADING))
                    self.last_load = tuple(pruned)
                for a in missing:                     # insertAdditionsOnly (:452-514)
                    self._insert(Info(a, TK, a))
                    if self.log is not None:
                        self.log.append((a, TK, a, ()))
                for a in missing:
                    self._add_missing_everywhere(a)
                if self.log is not None:              # the registration itself (the device evaluates it after the above)
                    self.log.append((wt, 0, wex, tuple(tx), OP_UNMANAGED if register else OP_UNMANAGED_RECHECK))
                rec = (APPLY_P, executes_at, wt) if waiting_to_apply else (COMMIT_P, tx[-1], wt)
                if add_list is not None:
                    add_list.append(rec)
                    return
                k = bisect.bisect_left(self.unmanageds, rec)
                if k == len(self.unmanageds) or self.unmanageds[k] != rec:
                    self.unmanageds.insert(k, rec)
                return
        if self.log is not None:
            self.log.append((wt, 0, wex, tuple(tx), OP_UNMANAGED if register else OP_UNMANAGED_RECHECK))
            self.notes.append((2, wt))
        sink(wt)


def unapplied_delta(kind):                            # CommandsForKey.unappliedCountersDelta :1291-1310
    return (1 << 32) + 1 if kind == WRITE else (1 if kind == READ else 0)


def unapplied_count(counters, kind):                  # CommandsForKey.unappliedCount :1312-1330
    return counters >> 32 if kind == READ else counters & 0xFFFFFFFF


def missing_count(txn, min_undecided, me):            # :1256-1272
    missing = sorted(txn.missing)
    n = len(missing)
    if n > 0:
        frm = 0
        if min_undecided is not None:
            frm = bisect.bisect_left(missing, min_undecided)
            n -= frm
        for j in range(frm, len(missing)):
            if not me(missing[j]):
                n -= 1
    return n


def full_scan_ready(cfk):
    """notifyManaged over the whole of committedByExecuteAt with every kind admitted: the STABLE managed txns the
    release rule lets go at this state.  This is what ad_cfk_notify computes on the device (one workgroup per key)."""
    committed = cfk.committed()
    out = []
    cfk.notify_managed(committed, ANY_GLOBALLY_VISIBLE, len(committed), -1, out.append)
    return out


def canon_view(canon):
    """Canon's committedByExecuteAt as the release invariants read it: (executeAt, txnId, SaveStatus order, domain,
    still waiting on the key) per committed command, executeAt ascending."""
    out = []
    for ex in canon.committed_by_execute_at.head(MAX):
        c = canon.committed_by_execute_at.get(ex)
        w = c.waiting_on
        out.append((ex, c.txn, SS_ORDER[c.ss], canon.domains[c.txn], bool(w is not None and w.key)))
    return out


def release_invariant_violations(view, released):
    """The reference's execution-order invariants, applied to a release set (txns let go at this state): for each
    released T, (:175-180 / :208-212) every committed command executing before T that T witnesses (key domain) has
    Applied (ExclusiveSyncPoints / EphemeralReads await only their deps); (:214-218) no Stable command executing after T
    that witnesses T (and awaits more than its deps) has been let go — neither earlier (its key bit cleared) nor in
    the same set.  Returns the violations."""
    rel = set(released)
    by_txn = {t: (ex, so, dom, waiting) for ex, t, so, dom, waiting in view}
    bad = []
    for t in rel:
        if t not in by_txn:
            bad.append(("not committed", t))
            continue
        tex = by_txn[t][0]
        pk = kind_of(t)
        for ex, c, so, dom, waiting in view:
            if ex < tex:
                if pk not in (ESP, EPH) and dom != RANGE and witnesses(pk, kind_of(c)) and so < SS_ORDER[APPLIED_SS]:
                    bad.append(("unapplied predecessor", t, c))
            elif ex > tex and by_txn[t][2] == KEY:
                if kind_of(c) in (ESP, EPH) or not witnesses(kind_of(c), pk) or so < SS_ORDER[STABLE_SS]:
                    continue
                if not waiting or c in rel:
                    bad.append(("successor released first", t, c))
    return bad


# ---- CommandsForKeyTest.test(seed, minCount) (:590-646) --------------------------------------------------------------
class Run:
    """One seed of the restated harness.  events: per update, (txnId, SaveStatus) and the managed notifications it
    caused; snapshots: the CFK after events chosen by `snapshot_every` (and every event with a notification)."""

    def __init__(self, seed, min_count, snapshot_every=0, check_full_scan=False, count_gating=False, log=False,
                 prune=False, keep_states_every=0, snapshot_lag=False):
        self.seed = seed
        self.states = {}                              # event -> CFK copy (keep_states_every: mapReduceActive probes)
        self.canon_views = {}                         # snapshot event -> canon_view(canon) (release invariants)
        self.lag_events = 0
        self.event_log = [] if log else None          # per harness event: the CFK update calls it made (CFK.log)
        self.note_log = [] if log else None           # per harness event: its unmanaged notifications (CFK.notes)
        rnd = Rnd(seed)
        self.run_task_chance = max(0.01, float(rnd.next_float()))
        import numpy as np
        f = np.float32
        self.prune_chance = float(rnd.next_float() * (f(0.1) if rnd.next_boolean() else f(0.01)))
        self.prune_hlc_delta = 1 << rnd.next_int(10)
        self.prune_interval = 1 << rnd.next_int(5)
        self.domains = {}
        canon = Canon(rnd, self.domains)
        cfk = CFK(self.domains)
        if log:
            cfk.log = []
            cfk.notes = []
        self.canon, self.cfk = canon, cfk
        self.snapshots = []                           # (event, rows, notified-and-STABLE set, full-scan release set)
        self.events = 0
        self.notified = set()
        self.full_scan_mismatches = []
        self.gated_events = 0                         # events after which some STABLE txn is held by an undecided dep
        queue = collections.deque()                   # TestCommandStore.queue: ('load' | 'unmanaged', TxnId)
        self.tasks_run = 0
        self.max_rows = 0
        self.loads = 0
        sink = canon.not_waiting

        def run_one_task():                           # TestCommandStore.runOneTask (:932-939)
            if not queue:
                return
            self.tasks_run += 1
            what, t = queue.popleft()
            cmd = canon.by_id.get(t)
            if what == 'load':                        # PostProcess.LoadPruned.load -> SafeCommandsForKey.updatePruned
                changed, cur_status, new_info = cfk.update(cmd, was_pruned=True)
                if not changed:                       # updateCfk == prevCfk: nothing to post-process
                    return
                self.loads += 1
                self._post_update(cfk, canon, queue, cur_status, new_info, cmd, True, sink,
                                  prune_now=cmd.has_been(S_APPLIED))
            else:                                     # Updating.updateUnmanagedAsync (:690-700)
                cfk.update_unmanaged(cmd, sink, False)

        c = 0
        while not canon.is_done():
            c += 1
            if c >= min_count:
                canon.close()
            rtc = np.float32(self.run_task_chance)
            if rnd.decide(rtc - rtc / np.float32(1 + len(queue))):
                run_one_task()
            up = canon.update(len(queue) > 0)
            if up is None:
                run_one_task()
                continue
            prev, nxt = up
            before = len(canon.notified)
            if canon.manages(nxt.txn):
                changed, cur_status, new_info = cfk.update(nxt)
                do_prune = rnd.decide(np.float32(self.prune_chance)) and prune
                self._post_update(cfk, canon, queue, cur_status, new_info, nxt, changed, sink, prune_now=do_prune)
            if not canon.manages_execution(nxt.txn) and nxt.has_been(S_STABLE) and not nxt.has_been(S_TRUNCATED):
                # registerUnmanaged(safeStore, new TestSafeCommand(.., update.next)): the command as updated (the
                # WaitingOn executeAtLeast bump for awaitsOnlyDeps kinds, Updating.java:806-815, changes nothing the
                # harness or the release rule reads, and is not modelled); its pruned deps are queued loads
                cfk.update_unmanaged(nxt, sink, True)
                for t in cfk.last_load:
                    queue.append(('load', t))
            self.events += 1
            self.max_rows = max(self.max_rows, len(cfk.ids))
            if log:
                self.event_log.append(list(cfk.log))
                cfk.log.clear()
                self.note_log.append(list(cfk.notes))
                cfk.notes.clear()
            fresh = [t for t, _ in canon.notified[before:] if canon.manages_execution(t)]
            self.notified.update(fresh)
            if count_gating and gating_cases(cfk):
                self.gated_events += 1
            if check_full_scan:
                want = {t for t in self.notified if cfk.info.get(t) is not None and cfk.info[t].status == STABLE}
                got = set(full_scan_ready(cfk))
                if got != want:
                    self.full_scan_mismatches.append((self.events, sorted(got - want), sorted(want - got)))
            if keep_states_every and self.events % keep_states_every == 0:
                self.states[self.events] = cfk.copy()
            lagging = False
            if snapshot_lag:                          # also every state where the notifications lag the full scan
                want = {t for t in self.notified if cfk.info.get(t) is not None and cfk.info[t].status == STABLE}
                lagging = set(full_scan_ready(cfk)) != want
                self.lag_events += lagging
            if snapshot_every and (fresh or lagging or self.events % snapshot_every == 0):
                self.canon_views[self.events] = canon_view(canon)
                self.snapshots.append((self.events, self.rows(), frozenset(
                    t for t in self.notified if cfk.info.get(t) is not None and cfk.info[t].status == STABLE),
                    frozenset(full_scan_ready(cfk))))
        if log and (cfk.log or cfk.notes):             # the CFK updates of tasks run after the last logged event
            self.event_log.append(list(cfk.log))
            cfk.log.clear()
            self.note_log.append(list(cfk.notes))
            cfk.notes.clear()
        self.queue_left = len(queue)

    def _post_update(self, cfk, canon, queue, cur_status, new_info, cmd, changed, sink, prune_now):
        """CommandsForKeyUpdate.postProcess after CommandsForKey.update / updatePruned (+ maybePrune):
        notifyUnmanaged's lists (computed by the update), notifyManaged, LoadPruned, NotifyNotWaiting,
        NotifyUnmanagedOfCommit (PostProcess.java:60-244)."""
        load = cfk.last_load
        commit_n, apply_n = ([], []) if not changed else cfk.notify_unmanaged(cur_status, new_info)
        # the CFK's own notifyManaged (on the pre-prune CFK: see the module docstring)
        if changed:
            cfk.post_process(cur_status, cmd, sink)
        elif cmd.txn in cfk.info:                     # an unchanged CFK still post-processes the command
            cfk.post_process(cfk.info[cmd.txn].status, cmd, sink)
        if prune_now:
            cfk.maybe_prune(self.prune_interval, self.prune_hlc_delta)
        for t in load:                                # LoadPruned: every TxnId is below prunedBefore -> queued
            queue.append(('load', t))
        for u in apply_n:
            sink(u)
        if commit_n:
            adds = []
            for u in commit_n:
                if u < cfk.pruned_before:             # ifLoadedAndInitialised == null -> updateUnmanagedAsync
                    queue.append(('unmanaged', u))
                else:
                    cfk.update_unmanaged(canon.by_id.get(u), sink, False, adds)
            for rec in sorted(adds):
                k = bisect.bisect_left(cfk.unmanageds, rec)
                if k == len(cfk.unmanageds) or cfk.unmanageds[k] != rec:
                    cfk.unmanageds.insert(k, rec)

    def rows(self):
        """The CFK as the C-ABI takes it (CommandsForKey.SerializerSupport.create, :226-232): byId TxnInfos —
        TxnId, InternalStatus, executeAt, missing() as row indices."""
        cfk = self.cfk
        pos = {t: k for k, t in enumerate(cfk.ids)}
        out = []
        for t in cfk.ids:
            i = cfk.info[t]
            out.append((t, self.domains[t], i.status, i.execute_at, sorted(pos[m] for m in i.missing)))
        return out


# ---- packing for the C-ABI (ad_cfk_notify) ---------------------------------------------------------------------------
def ts_bits(t, domain=0):
    """(epoch, hlc, identity flags, node) -> Accord's raw (msb, lsb, node) (Timestamp.java:77-96)."""
    epoch, hlc, flags, node = t
    return (epoch << 15) | (hlc >> 48), ((hlc & ((1 << 48) - 1)) << 16) | flags | domain, node


def pack_states(states, scramble_undecided=True):
    """CFK states (lists of Run.rows() tuples) -> the ad_cfk_state arrays.  Rows below ACCEPTED carry no executeAt in
    the reference's release rule; with scramble_undecided their executeAt is all ones (proving it is never read)."""
    row_off, tm, tl, tn, em, el, en, st, moff, miss = [0], [], [], [], [], [], [], [], [0], []
    for rows in states:
        for t, dom, status, ex, missing in rows:
            m, l, n = ts_bits(t, dom)
            tm.append(m); tl.append(l); tn.append(n)
            if scramble_undecided and status < ACC:
                em.append((1 << 64) - 1); el.append((1 << 64) - 1); en.append(-1)
            else:
                m, l, n = ts_bits(ex)
                em.append(m); el.append(l); en.append(n)
            st.append(status)
            miss.extend(missing)
            moff.append(len(miss))
        row_off.append(len(st))
    return {"row_off": np.array(row_off, np.uint32), "txn_msb": np.array(tm, np.uint64), "txn_lsb": np.array(tl, np.uint64),
            "txn_node": np.array(tn, np.int32), "exec_msb": np.array(em, np.uint64), "exec_lsb": np.array(el, np.uint64),
            "exec_node": np.array(en, np.int32), "status": np.array(st, np.uint8), "miss_off": np.array(moff, np.uint32),
            "missing": np.array(miss if miss else [0], np.uint32)[:len(miss)] if miss else np.zeros(0, np.uint32)}


def gating_cases(cfk):
    """STABLE Read / Write txns that the scan reaches (after the last applied Write, not past the first unapplied
    Write) but that stay held because an undecided lower-TxnId txn they conflict with is not in their missing set:
    the Stable-waits-for-undecided case of :1237-1280."""
    committed = cfk.committed()
    maw = cfk.max_applied_write(committed)
    mu = cfk.min_undecided()
    min_undecided = cfk.ids[mu] if mu >= 0 else None
    out = []
    for i in range(maw + 1, len(committed)):
        t = committed[i]
        if t.status == APPLIED or not cfk.me(t.txn):
            continue
        if t.status == STABLE:
            und = [u for u in cfk.ids if u < t.execute_at and cfk.info[u].status < COMMITTED and cfk.me(u)
                   and witnesses(kind_of(t.txn), kind_of(u))]
            miss = missing_count(t, min_undecided, cfk.me)
            if [u for u in und if u not in t.missing] and len(und) != miss:
                out.append(t.txn)
        if kind_of(t.txn) == WRITE:
            break
    return out
