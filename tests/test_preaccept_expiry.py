"""The rest of CommandStore.preaccept (local/CommandStore.java:322-347) around the maxConflicts test:

    isExpired = now - txnId.hlc >= preAcceptTimeout && !kind.isSyncPoint()                              :326
             || rejectBefore.foldl(keys, rejectIfBefore > txnId ? null : test, txnId, isNull)           :327-328
    isExpired -> time.uniqueNow(txnId).asRejected()                                                    :330-331
    ExclusiveSyncPoint -> markExclusiveSyncPoint(ranges) ; return txnId                               :333-337

Pinned three ways: known answers from those lines for the oracle (oracle.cpp preaccept_rules) and the host restatement
(witness.preaccept / RejectBefore); an independent per-txn Python model against the oracle over mixed batches; and
(-m gpu) the device's fast flags (ad_preaccept_expiry) against the oracle, with ExclusiveSyncPoints, a carried
rejectBefore and the timeout test.  The reference has no test of these branches: parity unpinned beyond the cited
lines."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, witness as Wt, workload


def ts(hlc, kind=abi.KIND_WRITE, domain=0, node=1, epoch=1):
    return Wt.from_values(epoch, hlc, (kind << 1) | domain, node)


def test_host_preaccept_branches():
    clock = Wt.NodeClock(1, 1, 1_000_000)
    t = ts(500)
    # timeout: now - hlc >= timeout -> uniqueNow(txnId).asRejected()
    w = Wt.preaccept(t, None, clock, keys=(7,), pre_accept_timeout=1000)
    assert w[1] & Wt.REJECTED_FLAG and Wt.compare(w, t) > 0
    # sync points are exempt from the timeout; an ExclusiveSyncPoint answers its TxnId even above maxConflict
    esp = ts(501, abi.KIND_EXCLUSIVE_SYNC_POINT, domain=1)
    rb = Wt.RejectBefore()
    assert Wt.preaccept(esp, ts(900), clock, ranges=((0, 100),), reject_before=rb, pre_accept_timeout=1000) == esp
    assert rb.iv == [(0, 100, esp)]                                  # markExclusiveSyncPoint
    # a later-arriving lower TxnId on those keys is rejected; outside them it is not
    low = ts(400)
    assert Wt.preaccept(low, None, clock, keys=(50,), reject_before=rb)[1] & Wt.REJECTED_FLAG
    assert Wt.preaccept(low, None, clock, keys=(150,), reject_before=rb) == low
    # a higher TxnId passes the fold and takes the fast-path test
    hi_ = ts(600)
    assert Wt.preaccept(hi_, None, clock, keys=(50,), reject_before=rb) == hi_
    assert Wt.preaccept(hi_, ts(700), clock, keys=(50,), reject_before=rb)[1] & Wt.REJECTED_FLAG == 0
    # Timestamp::max merge of overlapping marks, normal form
    rb.add([(50, 200)], ts(450, abi.KIND_EXCLUSIVE_SYNC_POINT, 1))
    assert [(s, e) for s, e, _ in rb.iv] == [(0, 100), (100, 200)]
    rb.add([(50, 200)], ts(800, abi.KIND_EXCLUSIVE_SYNC_POINT, 1))
    assert [(s, e) for s, e, _ in rb.iv] == [(0, 50), (50, 200)]


def _batch(n, seed, hlc_start=1_000_000):
    rng = np.random.default_rng(seed)
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT],
                       p=[0.4, 0.4, 0.1, 0.1], size=n)
    return workload.generate(n, keys_per_txn=3, keyspace=3000, range_frac=0.25, range_width_max=200, seed=seed,
                             slow_frac=0.3, bump_max=300, kinds=kinds, hlc_start=hlc_start)


def _reject_table(seed):
    rng = np.random.default_rng(seed)
    rb = Wt.RejectBefore()
    for _ in range(12):
        s = int(rng.integers(0, 2900))
        rb.add([(s, s + int(rng.integers(1, 150)))], ts(1_000_000 + int(rng.integers(0, 9000)),
                                                        abi.KIND_EXCLUSIVE_SYNC_POINT, 1, int(rng.integers(1, 9))))
    return rb


def _model(b, fast_plain, now, timeout, rb):
    """Independent restatement over a batch: per txn the rules above applied to the plain maxConflicts flags."""
    want = fast_plain.copy()
    for i in range(b["n"]):
        t = (int(b["txn_msb"][i]), int(b["txn_lsb"][i]), int(b["txn_node"][i]))
        keys = [int(k) for k in b["keys"][b["key_off"][i]:b["key_off"][i + 1]]]
        ranges = []
        if b.get("range_off") is not None:
            ranges = [(int(b["range_start"][q]), int(b["range_end"][q]))
                      for q in range(int(b["range_off"][i]), int(b["range_off"][i + 1]))]
        k = Wt.kind(t)
        expired = timeout is not None and now - Wt.hlc(t) >= timeout and k not in (abi.KIND_SYNC_POINT,
                                                                                    abi.KIND_EXCLUSIVE_SYNC_POINT)
        if not expired and rb is not None:
            expired = rb.rejects(t, keys, ranges)
        if expired:
            want[:, i] = abi.FAST_REJECTED
        elif k == abi.KIND_EXCLUSIVE_SYNC_POINT:
            want[:, i] = 1
    return want


@pytest.mark.parametrize("timeout", [None, 4000])
def test_oracle_rules_match_model(timeout):
    b = _batch(3000, 5)
    rb = _reject_table(6)
    cfg = abi.make_config(16, 2, 0.2, 0xE5)
    now = 1_000_000 + 9000
    try:
        O.set_preaccept_expiry()
        plain = O.max_conflicts_ts(b, cfg)[3]
        # the plain flags with ExclusiveSyncPoints forced to TxnId are the no-expiry answer
        O.set_preaccept_expiry(now, O.NO_TIMEOUT if timeout is None else timeout, rb.table())
        got = O.max_conflicts_ts(b, cfg)[3]
        _, got_rank_path = O.max_conflicts(b, cfg)
    finally:
        O.set_preaccept_expiry()
    esp = (b["txn_lsb"] >> np.uint64(1)) & np.uint64(7) == abi.KIND_EXCLUSIVE_SYNC_POINT
    assert (plain[:, esp] == 1).all()
    want = _model(b, plain, now, timeout, rb)
    assert np.array_equal(got, want)
    assert (got == abi.FAST_REJECTED).any() and (got == 1).any() and (got == 0).any()
    assert np.array_equal(got_rank_path == abi.FAST_REJECTED, got == abi.FAST_REJECTED)


@pytest.mark.gpu
@pytest.mark.parametrize("timeout", [None, 4000])
def test_gpu_preaccept_rules_equal_oracle(engine_factory, timeout):
    b = _batch(6000, 7)
    rb = _reject_table(8)
    now = 1_000_000 + 9000
    cfg_args = (16, 3, 0.2, 0xE7)
    cfg = abi.make_config(*cfg_args)
    eng = engine_factory(window=16, replicas=3, drop_p=0.2, seed=0xE7)
    eng.load(b)
    eng.preaccept_deps()
    eng.preaccept_expiry(now, eng.NO_TIMEOUT if timeout is None else timeout, rb.table())
    d_rank, d_fast = eng.max_conflicts()
    d_ts = eng.max_conflicts_ts()
    try:
        O.set_preaccept_expiry(now, O.NO_TIMEOUT if timeout is None else timeout, rb.table())
        w_rank, w_fast = O.max_conflicts(b, cfg)
        w_ts = O.max_conflicts_ts(b, cfg)
    finally:
        O.set_preaccept_expiry()
    assert np.array_equal(d_rank, w_rank) and np.array_equal(d_fast, w_fast)
    for x, y in zip(d_ts, w_ts):
        assert np.array_equal(x, y)
    assert (d_fast == abi.FAST_REJECTED).any()
    # the fast-path merge leaves rejected replies out (only witnessedAt == TxnId replies are merged)
    eng.merge_fast()
    eng.preaccept_expiry()                                  # back to the handle's default: no expiry state
    _, plain = eng.max_conflicts()
    esp = (b["txn_lsb"] >> np.uint64(1)) & np.uint64(7) == abi.KIND_EXCLUSIVE_SYNC_POINT
    assert (plain != abi.FAST_REJECTED).all() and (plain[:, esp] == 1).all()


def _tie_case(seed=11):
    """rejectBefore entries equal to a txn's own TxnId (not rejected: `rejectIfBefore > txnId` is false on a tie,
    CommandStore.java:328) and the same msb / hlc / flags from a lower and a higher node (only the higher one
    rejects: node is compareTo's last tiebreak, Timestamp.java:208-217).  One key per txn over a wide keyspace,
    so each mark stabs only the txn it was made for."""
    b = workload.generate(400, keys_per_txn=1, keyspace=1 << 40, seed=seed)
    rb = Wt.RejectBefore()
    want = {}
    for j, i in enumerate(range(5, 400, 7)):
        k = int(b["keys"][b["key_off"][i]])
        t = (int(b["txn_msb"][i]), int(b["txn_lsb"][i]), int(b["txn_node"][i]))
        d = (0, -1, 1)[j % 3] if t[2] > 1 else (0, 1)[j % 2]
        rb.add([(k - 1, k)], (t[0], t[1], t[2] + d))
        want[i] = d > 0
    return b, rb, want


def test_reject_before_ties_on_the_real_txn_id():
    b, rb, want = _tie_case()
    cfg = abi.make_config(0, 1, 0.0, 0xE9)
    try:
        O.set_preaccept_expiry(0, O.NO_TIMEOUT, rb.table())
        _, fast = O.max_conflicts(b, cfg)
    finally:
        O.set_preaccept_expiry()
    for i, rej in want.items():
        t = (int(b["txn_msb"][i]), int(b["txn_lsb"][i]), int(b["txn_node"][i]))
        k = int(b["keys"][b["key_off"][i]])
        assert rb.rejects(t, [k], []) == rej
        assert (fast[0, i] == abi.FAST_REJECTED) == rej, i
    assert any(want.values()) and not all(want.values())


@pytest.mark.gpu
def test_gpu_reject_before_ties_on_the_real_txn_id(engine_factory):
    b, rb, want = _tie_case()
    cfg = abi.make_config(0, 1, 0.0, 0xE9)
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=0xE9)
    eng.load(b)
    eng.preaccept_deps()
    eng.preaccept_expiry(0, eng.NO_TIMEOUT, rb.table())
    _, d_fast = eng.max_conflicts()
    try:
        O.set_preaccept_expiry(0, O.NO_TIMEOUT, rb.table())
        _, w_fast = O.max_conflicts(b, cfg)
    finally:
        O.set_preaccept_expiry()
    assert np.array_equal(d_fast, w_fast)
    for i, rej in want.items():
        assert (d_fast[0, i] == abi.FAST_REJECTED) == rej, i
