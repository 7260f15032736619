"""The four PreAcceptTest known answers (test/messages/PreAcceptTest.java:85-290), restated exactly: the expected
PreAcceptOk(txnId, witnessedAt, deps) of each, from

* the PreAccept deps (oracle: CommandsForKey.mapReduceActive + Deps.Builder),
* maxConflicts.get(keys) over the store's MaxConflicts map carried from its earlier batches plus the batch
  (oracle_max_conflicts_ts / _export, the same contract as ad_max_conflicts_ts / _export), and
* the host's CommandStore.preaccept decision + Node.uniqueNow (accord_amd/witness.py).

The test node is ID1 on a MockCluster Clock(100) (MockCluster.java:385-423): Node.now starts at
Timestamp.fromValues(1, 100, ID1) (Node.java:188); clock.increment(10) runs before each PreAccept is processed.
Every message is one batch (a CommandStore sees them in arrival order), so a txn that arrives after a larger
TxnId sees it through the carried MaxConflicts map, as the reference's store does.  tests/test_gpu_max_conflicts.py
runs the same cases through the engine."""
import numpy as np

import oracle as O
from accord_amd import abi, witness as Wt
from batchkit import T, deps_of, make_batch

ID1, ID2, ID3 = 1, 2, 3
WRITE_KEY_FLAGS = abi.KIND_WRITE << 1          # TxnId flags of a key-domain Write (TxnId.java:132-165)


def store_process(batches, window=0):
    """Run batches in arrival order through one store (oracle), carrying MaxConflicts: per batch,
    (deps CSRs, maxConflict timestamps, fast flags)."""
    carry = None
    out = []
    cfg = abi.make_config(window, 1, 0.0, 1)
    for b in batches:
        res = O.OracleResult(b, cfg, O.FLAG_MERGE)
        om, ol, on, fast = O.max_conflicts_ts(b, cfg, carry)
        out.append(({c: res.deps(0, c) for c in range(abi.NUM_CLASSES)}, (om[0], ol[0], on[0]), fast[0]))
        carry = O.max_conflicts_export(b, carry)
    return out


def max_conflict(mc, i):
    t = (int(mc[0][i]), int(mc[1][i]), int(mc[2][i]))
    return None if t == Wt.NONE else t


def no_deps(deps, i):
    return all(deps_of(deps[c], i) == {} for c in range(abi.NUM_CLASSES))


def test_initial_command():
    # initialCommandTest (:85-122): txnId = clock.idForNode(1, ID2) = (1, 100, Write, Key, ID2); PreAcceptOk(txnId,
    # txnId, NONE deps)
    clock = Wt.NodeClock(ID1, 1, 100)
    txn = Wt.from_values(1, 100, WRITE_KEY_FLAGS, ID2)
    [(deps, mc, fast)] = store_process([make_batch([T(100, abi.KIND_WRITE, [10], node=ID2)])])
    assert no_deps(deps, 0) and max_conflict(mc, 0) is None and fast[0] == 1
    clock.clock += 10
    assert Wt.preaccept_witnessed_at(txn, max_conflict(mc, 0), clock) == txn


def test_multi_key_timestamp_update():
    # multiKeyTimestampUpdate (:187-222): (1, 100, ID2) on key 10 arrives first; then txnId2 = (1, 50, ID3) on keys
    # {10, 11}: no deps (the earlier arrival has the larger TxnId), maxConflict = (1, 100, ID2) > txnId2 -> slow path,
    # witnessedAt = uniqueNow(maxConflict) = (epoch 1, hlc 110, ID1).  Node.now was built at epoch 0 (Node.java:188,
    # before the test topology was reported), so nowAtLeast (:368-375) takes the max conflict's bits, flags included
    clock = Wt.NodeClock(ID1, 1, 100, now_epoch=0)
    first = make_batch([T(100, abi.KIND_WRITE, [10], node=ID2)])
    second = make_batch([T(50, abi.KIND_WRITE, [10, 11], node=ID3)])
    (_, mc1, f1), (deps2, mc2, f2) = store_process([first, second])
    assert f1[0] == 1
    assert no_deps(deps2, 0)
    assert max_conflict(mc2, 0) == Wt.from_values(1, 100, WRITE_KEY_FLAGS, ID2) and f2[0] == 0
    clock.clock += 10
    w = Wt.preaccept_witnessed_at(Wt.from_values(1, 50, WRITE_KEY_FLAGS, ID3), max_conflict(mc2, 0), clock)
    # expectedTs = Timestamp.fromValues(1, 110, ID1).withExtraFlags(txnId2.flags()), compared by PreAcceptOk.equals
    # -> Timestamp.equals (Timestamp.java:244-249: IDENTITY_LSB includes the kind flags): Node.nowAtLeast takes the
    # max conflict's bits (its flags: Write, Key — txnId2's too) with Node.now's hlc and node, and uniqueNow keeps
    # them (withNextHlc / withEpochAtLeast carry flags())
    assert Wt.equals(w, Wt.from_values(1, 110, WRITE_KEY_FLAGS, ID1))
    assert not Wt.equals(w, Wt.from_values(1, 110, 0, ID1))            # the flags are part of the identity


def test_single_key_newer_timestamp():
    # singleKeyNewerTimestamp (:224-249): txnId = (1, 110, ID2) with nothing recorded: PreAcceptOk(txnId, txnId, NONE)
    clock = Wt.NodeClock(ID1, 1, 100)
    txn = Wt.from_values(1, 110, WRITE_KEY_FLAGS, ID2)
    [(deps, mc, fast)] = store_process([make_batch([T(110, abi.KIND_WRITE, [10], node=ID2)])])
    assert no_deps(deps, 0) and fast[0] == 1
    assert Wt.preaccept_witnessed_at(txn, max_conflict(mc, 0), clock) == txn


def test_superseding_epoch_precludes_fast_path():
    # supersedingEpochPrecludesFastPath (:251-290): topology at epoch 2, txnId (1, 100, ID2) with no conflict: the
    # fast path needs txnId.epoch() >= time.epoch() (CommandStore.java:343) -> uniqueNow() = (2, 110, ID1)
    clock = Wt.NodeClock(ID1, 1, 100)
    clock.topology_epoch = 2
    txn = Wt.from_values(1, 100, WRITE_KEY_FLAGS, ID2)
    [(deps, mc, fast)] = store_process([make_batch([T(100, abi.KIND_WRITE, [10], node=ID2)])])
    assert no_deps(deps, 0) and max_conflict(mc, 0) is None and fast[0] == 1     # the device part: fast
    clock.clock += 10
    w = Wt.preaccept_witnessed_at(txn, max_conflict(mc, 0), clock)
    assert w == Wt.from_values(2, 110, 0, ID1)


def test_carry_is_max_over_batches():
    # the carried map is the per-key running max over every batch (MaxConflicts.update: Timestamp::max per key)
    b1 = make_batch([T(10, abi.KIND_WRITE, [1], exec_hlc=40), T(11, abi.KIND_READ, [2])])
    b2 = make_batch([T(20, abi.KIND_WRITE, [1], exec_hlc=30), T(21, abi.KIND_WRITE, [3], status=abi.ST_INVALID)])
    c1 = O.max_conflicts_export(b1)
    c2 = O.max_conflicts_export(b2, c1)
    assert list(c2[0]) == [1, 2]                           # key 3: the only txn is INVALID (never recorded)
    assert Wt.hlc((int(c2[1][0]), int(c2[2][0]), int(c2[3][0]))) == 40
    b3 = make_batch([T(30, abi.KIND_READ, [1, 2])])
    om, ol, on, fast = O.max_conflicts_ts(b3, abi.make_config(0, 1, 0.0, 1), c2)
    assert Wt.hlc((int(om[0, 0]), int(ol[0, 0]), int(on[0, 0]))) == 40 and fast[0, 0] == 0
