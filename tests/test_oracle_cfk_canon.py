"""The restated CommandsForKeyTest harness (tests/cfk_canon.py) on the CPU: the Canon transition table is the
reference's (:235-246), every seed run satisfies the reference's own invariants (readyToExecute :175-180, notWaiting
:208-218, asserted inside the restatement), and the event-driven release of notifyManaged (postProcess with its kinds and
bounds, CommandsForKey.java:1121-1289) equals, after every event, the full-scan release rule ad_cfk_notify computes on the
device (cfk_canon.full_scan_ready): the set of STABLE Read / Write txns the CFK has notified so far.  Known answers for
the undecided-dependency gate (:1237-1280).  The GPU side: tests/test_gpu_cfk_release.py."""
import pytest

import cfk_canon as K
from cfk_state import TRANSITIONS


def test_transition_table_is_the_references():
    # CommandsForKeyTest.java:237-245, SaveStatus by SaveStatus
    want = {
        "NotDefined": ["PreAccepted", "AcceptedInvalidate", "AcceptedInvalidateWithDefinition", "Accepted",
                       "AcceptedWithDefinition", "Committed", "Stable", "Invalidated"],
        "PreAccepted": ["AcceptedInvalidateWithDefinition", "AcceptedWithDefinition", "Committed", "Stable", "Invalidated"],
        "AcceptedInvalidate": ["Invalidated"],
        "AcceptedInvalidateWithDefinition": ["Invalidated"],
        "Accepted": ["Committed", "Stable", "Invalidated"],
        "AcceptedWithDefinition": ["Committed", "Stable", "Invalidated"],
        "Committed": ["Stable"],
        "Stable": ["Applied"],
    }
    names = {K.NOT_DEFINED: "NotDefined", K.PRE_ACCEPTED: "PreAccepted", K.ACCEPTED_INVALIDATE: "AcceptedInvalidate",
             K.ACCEPTED_INVALIDATE_WD: "AcceptedInvalidateWithDefinition", K.ACCEPTED_SS: "Accepted",
             K.ACCEPTED_WD: "AcceptedWithDefinition", K.COMMITTED_SS: "Committed", K.STABLE_SS: "Stable",
             K.APPLIED_SS: "Applied", K.INVALIDATED: "Invalidated"}
    got = {names[k]: [names[x] for x in v] for k, v in TRANSITIONS.items()}
    assert got == want


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_event_driven_release_equals_full_scan(seed):
    r = K.Run(seed, 300, check_full_scan=True)
    assert r.canon.is_done() and r.events > 300
    assert r.full_scan_mismatches == [], r.full_scan_mismatches[:3]
    assert len(r.notified) > 10
    assert r.canon.ready_events                       # readyToExecute fired (and its invariant held)


def _cfk(domains, rows):
    """A hand-built CFK: rows of (TxnId, InternalStatus, executeAt, missing TxnIds)."""
    c = K.CFK(domains)
    for t, s, ex, miss in rows:
        c._insert(K.Info(t, s, ex, set(miss)))
    return c


def test_undecided_dependency_holds_a_stable_txn():
    d = {}
    w = K.txn_id(1, 10, K.WRITE, K.KEY, 1, d)           # undecided Write, lower TxnId
    r = K.txn_id(1, 20, K.READ, K.KEY, 1, d)
    ex_r = K.ts_from_values(1, 30, 1)
    # R's deps include W (W not missing): W undecided below R's executeAt holds R (expect 1 != 0 missing)
    assert K.full_scan_ready(_cfk(d, [(w, K.PREACC, w, ()), (r, K.STABLE, ex_r, ())])) == []
    assert K.gating_cases(_cfk(d, [(w, K.PREACC, w, ()), (r, K.STABLE, ex_r, ())])) == [r]
    # R did not witness W (W in missing): released
    assert K.full_scan_ready(_cfk(d, [(w, K.PREACC, w, ()), (r, K.STABLE, ex_r, (w,))])) == [r]
    # W committed before R's executeAt but not applied: R waits for it (the scan stops after W, R is beyond)
    assert K.full_scan_ready(_cfk(d, [(w, K.COMMITTED, K.ts_from_values(1, 25, 1), ()), (r, K.STABLE, ex_r, ())])) == []
    # W committed after R: decided, not before R -> released
    assert K.full_scan_ready(_cfk(d, [(w, K.COMMITTED, K.ts_from_values(1, 40, 1), ()), (r, K.STABLE, ex_r, ())])) == [r]
    # a Read does not wait for an undecided Read
    r0 = K.txn_id(1, 11, K.READ, K.KEY, 2, d)
    assert K.full_scan_ready(_cfk(d, [(r0, K.PREACC, r0, ()), (r, K.STABLE, ex_r, ())])) == [r]
    # a Write waits for an unapplied committed Read before it, and for an undecided Read
    w2 = K.txn_id(1, 21, K.WRITE, K.KEY, 1, d)
    ex_w2 = K.ts_from_values(1, 35, 1)
    assert K.full_scan_ready(_cfk(d, [(r, K.STABLE, ex_r, ()), (w2, K.STABLE, ex_w2, ())])) == [r]
    assert K.full_scan_ready(_cfk(d, [(r, K.APPLIED, ex_r, ()), (w2, K.STABLE, ex_w2, ())])) == [w2]
    assert K.full_scan_ready(_cfk(d, [(r0, K.PREACC, r0, ()), (r, K.APPLIED, ex_r, ()), (w2, K.STABLE, ex_w2, ())])) == []
    assert K.full_scan_ready(_cfk(d, [(r0, K.PREACC, r0, ()), (r, K.APPLIED, ex_r, ()), (w2, K.STABLE, ex_w2, (r0,))])) == [w2]


def test_gating_occurs_in_the_canon_stream():
    # the undecided-dependency gate is exercised by the reference's own stream, not only by the known answers
    held = sum(K.Run(seed, 200, count_gating=True).gated_events for seed in (0, 1, 2))
    assert held > 0
