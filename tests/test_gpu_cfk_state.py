"""CommandsForKey state evolving across batches on the device: a store's stream of batches
through one handle, with status transitions of the kept rows between batches (ad_cfk_update, CommandsForKeyTest's
transition table), pruning at each ad_cfk_retain, and the execution order over [kept rows | new txns] with the
applied / invalidated rows done.  Per batch, against the oracle over EVERY txn so far (nothing pruned) with the
current statuses: the new txns' PreAccept deps and Deps.merge, every kept row's level and the order; the Canon
readyToExecute invariant (CommandsForKeyTest.java:175-180) on the device's release set; and Stable txns apply only
when the device releases them (level 0) — so the device's own order drives the state, as notifyManaged does."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, engine, workload
from cfk_state import AP, CM, IV, PA, SB, TRANSITIONS, brute_levels, ready_invariant, save_statuses, transitions
from test_oracle_history import _mapped, _take, keep_rows

pytestmark = pytest.mark.gpu


def _state_stream(n_b, nb, keyspace, seed, kinds=None):
    n = n_b * nb
    return workload.generate(n, keys_per_txn=3, keyspace=keyspace, status=np.full(n, PA, np.uint8), kinds=kinds,
                             slow_frac=0.3, bump_max=60, seed=seed)


@pytest.mark.parametrize("n_b,nb,keyspace,replicas", [(6, 1500, 200, 1), (4, 6000, 3000, 2), (8, 800, 60, 1)])
def test_cfk_state_stream(engine_factory, n_b, nb, keyspace, replicas):
    rng = np.random.default_rng(keyspace + nb)
    stream = _state_stream(n_b, nb, keyspace, seed=keyspace * 7 + nb)
    cfg = abi.make_config(0, replicas, 0.0, 0x5EED)       # snapshot queries: the statuses are current
    eng = engine_factory(window=0, replicas=replicas, drop_p=0.0, seed=0x5EED)
    pruned_total = 0
    save = save_statuses(stream["status"])
    for k in range(n_b):
        seen = (k + 1) * nb
        rows = np.arange(k * nb, seen)
        eng.load(_take(stream, rows))
        H, gid = eng.cfk_rows()
        assert np.array_equal(gid[H:], rows)
        pruned_total = k * nb - H
        eng.preaccept_deps()
        eng.merge()
        lv, order, depth = eng.exec_levels()
        # the oracle over every txn so far, current statuses, nothing pruned
        upto = _take(stream, np.arange(seen))
        full = O.OracleResult(upto, cfg, O.FLAG_MERGE | O.FLAG_LEVELS | O.FLAG_DONE)
        ident = np.arange(seen)
        for v in range(replicas):
            got, want = eng.fetch_deps(v, abi.CLASS_KEY), full.deps(v, abi.CLASS_KEY)
            for x in range(nb):
                assert _mapped(got, H + x, gid) == _mapped(want, k * nb + x, ident), "batch %d view %d txn %d" % (k, v, k * nb + x)
        got, want = eng.fetch_merged(abi.CLASS_KEY), full.merged(abi.CLASS_KEY)
        for x in range(0, nb, 5):
            assert _mapped(got, H + x, gid) == _mapped(want, k * nb + x, ident)
        wl, wo = full.levels()
        assert np.array_equal(lv, wl[gid]), "batch %d: levels of the kept rows and new txns" % k
        pos = np.empty(seen, np.int64)
        pos[wo] = np.arange(seen)
        assert np.all(np.diff(pos[gid[order]]) > 0), "batch %d: the order is the oracle's restricted to the rows held" % k
        if seen <= 3000:                                   # the independent restatement on the whole state
            bl = brute_levels(upto)
            assert [None if x == abi.AD_LEVEL_DONE else int(x) for x in wl] == bl
        lvl = [None if x == abi.AD_LEVEL_DONE else int(x) for x in wl]
        ready_invariant(upto, lvl)                         # every released txn found its witnessed predecessors applied
        # retain (the restated rule over the same rows), then this batch's transitions of the kept rows; Stable
        # rows apply only once released.  Pruned rows are applied / invalidated: they never move again.
        keep = keep_rows(_take(upto, gid.astype(np.int64)), gid, 0)
        assert eng.cfk_retain() == len(keep)
        keep_gids = gid[keep]
        rows_upd, new = transitions(rng, upto["status"], [x == 0 for x in lvl], save[:seen])
        held = np.zeros(seen, bool)
        held[keep_gids] = True
        assert not np.isin(upto["status"][~held], [PA, abi.ST_ACCEPTED, CM, SB]).any(), "a pruned row still had to execute"
        sel = held[rows_upd]
        rows_upd, new = rows_upd[sel], new[sel]
        if len(rows_upd):
            eng.cfk_update(rows_upd.astype(np.uint32), new, stream["exec_msb"][rows_upd], stream["exec_lsb"][rows_upd],
                           stream["exec_node"][rows_upd])
        stream["status"][rows_upd] = new
        if k == 1 and len(keep_gids):
            _refusals(eng, keep_gids, stream)
    assert pruned_total > 0


def _refusals(eng, keep_gids, stream):
    # an illegal move (TRANSITIVELY_KNOWN is no successor of anything) is refused and applies nothing; so is a
    # row the store does not hold, and descending gids
    g = int(keep_gids[0])
    with pytest.raises(engine.AccordDepsError):
        eng.cfk_update(np.array([g], np.uint32), np.array([abi.ST_TRANSITIVELY_KNOWN], np.uint8))
    with pytest.raises(engine.AccordDepsError):
        eng.cfk_update(np.array([stream["n"] + 5], np.uint32), np.array([PA], np.uint8))
    if len(keep_gids) > 1:
        with pytest.raises(engine.AccordDepsError):
            eng.cfk_update(np.array([keep_gids[1], keep_gids[0]], np.uint32), np.array([PA, PA], np.uint8))


def test_cfk_update_executeat_rules(engine_factory):
    n = 2000
    b = _state_stream(1, n, 100, seed=3)
    eng = engine_factory(window=0, replicas=1, drop_p=0.0)
    eng.load(b)
    eng.preaccept_deps()
    eng.cfk_retain()
    g = np.array([10], np.uint32)
    one = lambda f: np.array([b[f][10]])
    # commit with executeAt below the TxnId: refused
    with pytest.raises(engine.AccordDepsError):
        eng.cfk_update(g, np.array([CM], np.uint8), one("txn_msb"), one("txn_lsb") - np.uint64(1 << 16), one("txn_node"))
    # commit at a later executeAt, then stable at another one: the second is refused (fixed once committed)
    eng.cfk_update(g, np.array([CM], np.uint8), one("txn_msb"), one("txn_lsb") + np.uint64(5 << 16), one("txn_node"))
    with pytest.raises(engine.AccordDepsError):
        eng.cfk_update(g, np.array([SB], np.uint8), one("txn_msb"), one("txn_lsb") + np.uint64(6 << 16), one("txn_node"))
    eng.cfk_update(g, np.array([SB], np.uint8))
    eng.cfk_update(g, np.array([AP], np.uint8))
    with pytest.raises(engine.AccordDepsError):
        eng.cfk_update(g, np.array([IV], np.uint8))       # applied is terminal
    # updates need the kept rows: after the next load they are part of a batch, refused until the next retain
    eng.load(_state_stream(1, 10, 100, seed=4))
    with pytest.raises(engine.AccordDepsError):
        eng.cfk_update(g, np.array([SB], np.uint8))
