"""ad_cfk_notify — CommandsForKey.notifyManaged's release rule on the device over evolving CFK state.

The CFK states are the ones the reference's own randomized harness produces: CommandsForKeyTest.test(seed, 1000)
(test/local/cfk/CommandsForKeyTest.java:590-646, restated in tests/cfk_canon.py with DefaultRandom) over 20 fixed
seeds.  After sampled events (every 25th, and every event that released something) the CFK — its byId TxnInfos with
InternalStatus, executeAt and missing() — goes to the device in its serialized layout, many states per launch (one
workgroup each); undecided rows carry an all-ones executeAt, which the rule must not read.  Checked per state:
* the device's release set == the STABLE Read / Write txns the restated CFK has notified (NotifySink.notWaiting) by then
  == the full-scan restatement (cfk_canon.full_scan_ready);
* Canon's notWaiting invariant (:208-211) on every device release: every committed key txn the released txn witnesses
  that executes before it has applied;
plus the known answers of the undecided-dependency gate and the input refusals."""
import numpy as np
import pytest

import cfk_canon as K
from accord_amd import abi, engine

pytestmark = pytest.mark.gpu
SEEDS = list(range(20))


def _check_states(eng, snapshots, domains):
    st = K.pack_states([rows for _, rows, _, _ in snapshots])
    got = eng.cfk_notify(st)
    off = st["row_off"]
    released = 0
    for k, (ev, rows, want, full) in enumerate(snapshots):
        g = got[off[k]:off[k + 1]]
        dev = {rows[i][0] for i in np.nonzero(g)[0]}
        assert dev == set(want), "event %d: device %s, reference %s" % (ev, sorted(dev - set(want))[:4], sorted(set(want) - dev)[:4])
        assert dev == set(full), "event %d: device vs the full-scan restatement" % ev
        released += len(dev)
        # Canon notWaiting invariant (:208-211) on the device's release
        for t in dev:
            tex = next(r[3] for r in rows if r[0] == t)
            for u, dom, s, ex, _ in rows:
                if dom == K.KEY and s in (K.COMMITTED, K.STABLE) and ex < tex and K.witnesses(K.kind_of(t), K.kind_of(u)):
                    raise AssertionError("event %d: %s released before %s applied" % (ev, t, u))
    return released


@pytest.mark.parametrize("chunk", range(5))
def test_canon_seeds_release_equals_reference(engine_factory, chunk):
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
    total = states = 0
    for seed in SEEDS[chunk * 4:(chunk + 1) * 4]:
        r = K.Run(seed, 1000, snapshot_every=25)
        assert r.canon.is_done()
        states += len(r.snapshots)
        total += _check_states(eng, r.snapshots, r.domains)
    assert states > 200 and total > 50


def test_gate_known_answers(engine_factory):
    d = {}
    w = K.txn_id(1, 10, K.WRITE, K.KEY, 1, d)
    r = K.txn_id(1, 20, K.READ, K.KEY, 1, d)
    r0 = K.txn_id(1, 11, K.READ, K.KEY, 2, d)
    w2 = K.txn_id(1, 21, K.WRITE, K.KEY, 1, d)
    ex_r, ex_w2 = K.ts_from_values(1, 30, 1), K.ts_from_values(1, 35, 1)
    cases = [
        ([(w, K.PREACC, w, ()), (r, K.STABLE, ex_r, ())], set()),                      # undecided dep holds R
        ([(w, K.PREACC, w, ()), (r, K.STABLE, ex_r, (w,))], {r}),                      # ... unless R did not witness it
        ([(w, K.COMMITTED, K.ts_from_values(1, 25, 1), ()), (r, K.STABLE, ex_r, ())], set()),
        ([(w, K.COMMITTED, K.ts_from_values(1, 40, 1), ()), (r, K.STABLE, ex_r, ())], {r}),
        ([(r0, K.PREACC, r0, ()), (r, K.STABLE, ex_r, ())], {r}),
        ([(r, K.STABLE, ex_r, ()), (w2, K.STABLE, ex_w2, ())], {r}),
        ([(r, K.APPLIED, ex_r, ()), (w2, K.STABLE, ex_w2, ())], {w2}),
        ([(r0, K.PREACC, r0, ()), (r, K.APPLIED, ex_r, ()), (w2, K.STABLE, ex_w2, ())], set()),
        ([(r0, K.PREACC, r0, ()), (r, K.APPLIED, ex_r, ()), (w2, K.STABLE, ex_w2, (r0,))], {w2}),
        ([], set()),                                                                     # an empty CFK
    ]
    states = []
    for rows, _ in cases:
        pos = {t: i for i, (t, *_rest) in enumerate(rows)}
        states.append([(t, d[t], s, ex, sorted(pos[m] for m in miss)) for t, s, ex, miss in rows])
    st = K.pack_states(states)
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
    got = eng.cfk_notify(st)
    for k, (rows, want) in enumerate(cases):
        g = got[st["row_off"][k]:st["row_off"][k + 1]]
        assert {rows[i][0] for i in np.nonzero(g)[0]} == want, "case %d" % k


def test_refusals(engine_factory):
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
    d = {}
    a = K.txn_id(1, 10, K.WRITE, K.KEY, 1, d)
    b = K.txn_id(1, 20, K.READ, K.KEY, 1, d)
    unsorted = K.pack_states([[(b, K.KEY, K.PREACC, b, []), (a, K.KEY, K.PREACC, a, [])]])
    with pytest.raises(engine.AccordDepsError) as e:
        eng.cfk_notify(unsorted)
    assert e.value.rc == abi.AD_ERR_UNSORTED
    bad = K.pack_states([[(a, K.KEY, K.PREACC, a, []), (b, K.KEY, K.STABLE, K.ts_from_values(1, 30, 1), [5])]])
    with pytest.raises(engine.IllegalArgumentException):
        eng.cfk_notify(bad)
