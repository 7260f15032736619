"""Execution order over evolving CommandsForKey state on the oracle: levels with APPLIED /
INVALID txns done (oracle FLAG_DONE, oracle.cpp exec_levels) against an independent brute-force restatement of the
release rule, and a stream of Canon-style status transitions (CommandsForKeyTest.java:235-246) driven by the
oracle's own release order, checked against Canon's readyToExecute invariant (:175-180) at every step."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload
from cfk_state import DONE, PA, SB, brute_levels, ready_invariant, save_statuses, transitions


def _levels(b, flags=O.FLAG_MERGE | O.FLAG_LEVELS | O.FLAG_DONE):
    return O.OracleResult(b, abi.make_config(0, 1, 0.0, 1), flags).levels()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_done_levels_equal_brute_force(seed):
    # any statuses (also inconsistent ones: the full rule and the oracle's recurrence agree on every input)
    rng = np.random.default_rng(seed)
    n = 400
    st = rng.choice(list(range(8)), size=n).astype(np.uint8)
    b = workload.generate(n, keys_per_txn=2, keyspace=40, status=st, slow_frac=0.3, bump_max=40, seed=seed)
    lv, order = _levels(b)
    want = brute_levels(b)
    for t in range(n):
        if want[t] is None:
            assert lv[t] == abi.AD_LEVEL_DONE
        else:
            assert lv[t] == want[t], "txn %d" % t
    # the order: done txns first (executeAt order), then by (level, executeAt)
    key = [(0 if lv[t] == abi.AD_LEVEL_DONE else int(lv[t]) + 1) for t in order]
    assert key == sorted(key)


def test_without_done_flag_levels_ignore_status():
    b = workload.generate(300, keys_per_txn=2, keyspace=30, status=np.full(300, abi.ST_APPLIED, np.uint8), seed=5)
    lv, _ = _levels(b, O.FLAG_MERGE | O.FLAG_LEVELS)
    assert (lv != abi.AD_LEVEL_DONE).all() and lv.max() > 0


def test_canon_stream_ready_invariant():
    # a single store's state driven by the transition table; Stable txns apply only when the oracle releases
    # them (level 0), and every release satisfies readyToExecute
    rng = np.random.default_rng(7)
    n = 600
    b = workload.generate(n, keys_per_txn=2, keyspace=25, status=np.full(n, PA, np.uint8), slow_frac=0.3, bump_max=30, seed=7)
    applied = 0
    save = save_statuses(b["status"])
    for step in range(60):
        lv, _ = _levels(b)
        lvl = [None if x == abi.AD_LEVEL_DONE else int(x) for x in lv]
        assert lvl == brute_levels(b)
        ready_invariant(b, lvl)
        rows, new = transitions(rng, b["status"], [x == 0 for x in lvl], save)
        applied += int((new == abi.ST_APPLIED).sum())
        b["status"][rows] = new
    assert applied > 150 and (np.isin(b["status"], DONE)).mean() > 0.2
