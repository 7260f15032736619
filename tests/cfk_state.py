"""Shared helpers for the CommandsForKey state-evolution tests.

The transition table is CommandsForKeyTest.Canon.TRANSITIONS exactly, over SaveStatus (accord-core/src/test/java/
accord/local/cfk/CommandsForKeyTest.java:235-246, restated in cfk_canon.TRANSITIONS): a row's SaveStatus moves, and
the CommandsForKey sees InternalStatus.from(SaveStatus) (CommandsForKey.java:504-528): PreAccepted and
AcceptedInvalidateWithDefinition are PREACCEPTED, Accepted(WithDefinition) ACCEPTED, then COMMITTED, STABLE, APPLIED,
INVALID; NotDefined and AcceptedInvalidate (no definition) have none, so the CFK does not change on them.  An
AcceptedInvalidate(WithDefinition) row can only become Invalidated (:240-241).  `brute_levels` is an independent
restatement of the release rule the Canon invariants check (:175-222): a txn is ready once every txn on its keys that
executes before it and that it witnesses has applied (Read/Write chains; applied / invalidated txns are done and wait
for nothing)."""
import numpy as np

import cfk_canon as K
from accord_amd import abi

TK, PA, AC, CM, SB, AP, IV = (abi.ST_TRANSITIVELY_KNOWN, abi.ST_PREACCEPTED, abi.ST_ACCEPTED, abi.ST_COMMITTED,
                              abi.ST_STABLE, abi.ST_APPLIED, abi.ST_INVALID)
TRANSITIONS = K.TRANSITIONS                 # SaveStatus -> its successors (:235-246)
INTERNAL = K._INTERNAL                      # SaveStatus -> InternalStatus (None: the CFK does not change)
SAVE_OF = {TK: K.NOT_DEFINED, PA: K.PRE_ACCEPTED, AC: K.ACCEPTED_SS, CM: K.COMMITTED_SS, SB: K.STABLE_SS,
           AP: K.APPLIED_SS, IV: K.INVALIDATED}


def save_statuses(status):
    """A SaveStatus for each InternalStatus (the unambiguous representative: PREACCEPTED -> PreAccepted)."""
    return np.array([SAVE_OF[int(s)] for s in status], np.int64)


DONE = (AP, IV)


def ts_key(msb, lsb, node):
    """Timestamp.compareTo order (Timestamp.java:208-217)."""
    return (int(msb), int(lsb) >> 16, int(lsb) & 0x1E, int(node))


def brute_levels(b):
    """Levels of a key-only Read/Write batch with current statuses, from the full (unreduced) rule:
    level(T) = 1 + max level over the not-done txns sharing a key with T, executing before T, that T witnesses
    (a Write witnesses Reads and Writes, a Read witnesses Writes); done txns (APPLIED / INVALID) get None."""
    n = b["n"]
    kind = ((b["txn_lsb"] >> np.uint64(1)) & np.uint64(7)).astype(int)
    ex = [ts_key(b["exec_msb"][i], b["exec_lsb"][i], b["exec_node"][i]) for i in range(n)]
    ko, keys = b["key_off"], b["keys"]
    by_key = {}
    for i in range(n):
        for k in keys[ko[i]:ko[i + 1]]:
            by_key.setdefault(int(k), []).append(i)
    order = sorted(range(n), key=lambda i: ex[i])
    lvl = [None] * n
    for t in order:
        if b["status"][t] in DONE:
            continue
        best = -1
        for k in keys[ko[t]:ko[t + 1]]:
            for d in by_key[int(k)]:
                if d == t or b["status"][d] in DONE or not ex[d] < ex[t]:
                    continue
                if kind[t] == abi.KIND_WRITE or kind[d] == abi.KIND_WRITE:
                    best = max(best, lvl[d])
        lvl[t] = best + 1
    return lvl


def ready_invariant(b, lvl):
    """CommandsForKeyTest.Canon.readyToExecute (:175-180): a txn released now (level 0, not done) finds every txn
    that executes before it on one of its keys and that it witnesses already applied (done)."""
    n = b["n"]
    kind = ((b["txn_lsb"] >> np.uint64(1)) & np.uint64(7)).astype(int)
    ex = [ts_key(b["exec_msb"][i], b["exec_lsb"][i], b["exec_node"][i]) for i in range(n)]
    ko, keys = b["key_off"], b["keys"]
    by_key = {}
    for i in range(n):
        for k in keys[ko[i]:ko[i + 1]]:
            by_key.setdefault(int(k), []).append(i)
    for t in range(n):
        if lvl[t] != 0:
            continue
        for k in keys[ko[t]:ko[t + 1]]:
            for d in by_key[int(k)]:
                if d != t and ex[d] < ex[t] and (kind[t] == abi.KIND_WRITE or kind[d] == abi.KIND_WRITE):
                    assert b["status"][d] in DONE, "txn %d released before %d (executes earlier, witnessed) applied" % (t, d)


def transitions(rng, status, ready, save, p_move=0.35, p_apply=0.6, p_invalid=0.02):
    """One round of Canon-style updates: every row moves with probability p_move along TRANSITIONS from its SaveStatus
    save[r] (Invalidated only with probability p_invalid); STABLE rows apply only when `ready` (released at level 0),
    with probability p_apply.  save is updated in place; returns (rows, new InternalStatus) of the rows whose
    InternalStatus changes (the CommandsForKey updates: a move to NotDefined / AcceptedInvalidate, or between the
    two PREACCEPTED SaveStatuses, changes nothing there)."""
    rows, new = [], []
    for r in range(len(status)):
        ss = int(save[r])
        if ss == K.STABLE_SS:
            if ready[r] and rng.random() < p_apply:
                save[r] = K.APPLIED_SS
                rows.append(r)
                new.append(AP)
            continue
        if ss not in TRANSITIONS or ss == K.STABLE_SS or rng.random() >= p_move:
            continue
        # Invalidated is rare unless it is the only successor (AcceptedInvalidate(WithDefinition), :240-241)
        choices = [x for x in TRANSITIONS[ss] if x != K.INVALIDATED or len(TRANSITIONS[ss]) == 1 or rng.random() < p_invalid]
        if not choices:
            continue
        nss = int(choices[rng.integers(len(choices))])
        save[r] = nss
        ni = INTERNAL.get(nss)
        if ni is not None and ni != int(status[r]):
            rows.append(r)
            new.append(ni)
    return np.array(rows, np.int64), np.array(new, np.uint8)
