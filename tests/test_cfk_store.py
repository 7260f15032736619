"""Device-resident CommandsForKey state: ad_cfk_store_apply keeps byId TxnInfos and their missing() sets
in HBM from the stream of CommandsForKey.update calls, and ad_cfk_store_notify runs notifyManaged's release rule over
those rows -- the host uploads only the update events, never a CFK snapshot or a missing array.

The stream is the reference's own randomized harness, CommandsForKeyTest.test(seed, 1000)
(test/local/cfk/CommandsForKeyTest.java:590-646, restated in tests/cfk_canon.py): every CommandsForKey.update call it makes
(CFK.log) becomes one event; 20 seeds run as 20 keys of one store, in lockstep (one ad_cfk_store_apply per harness step).
Checked at every sampled step (every 25th and every step that notified):
* the resident rows == the restated CFK's byId rows: TxnId, InternalStatus, executeAt and missing() exactly
  (Updating.insertOrUpdate, local/cfk/Updating.java:99-358, kept to CommandsForKey's missing invariant :101-113);
* the device's release set == the txns the restated harness notified (NotWaiting) that are still STABLE == the
  full-scan restatement of notifyManaged (CommandsForKey.java:1208-1289).
CPU: the host model of the kernel's algorithm (tests/cfk_store_model.py) replayed over the same logs gives the same rows.
With pruning (Run(prune=True): the reference's test(seed) draws rnd.decide(pruneChance) and runs maybePrune, LoadPruned
and updateUnmanagedAsync tasks off its queue), the event log carries LOAD / PRUNE / LOADING ops and the same checks run
plus prunedBefore and the loadingPruned table (TxnIds and the witnesses that are rows); the device release set is
compared with the full-scan restatement (with isWaitingOnPruned), and the harness's own event-driven notifications,
which can lag it while a pruned TxnId loads, must be a subset of it."""
import numpy as np
import pytest

import cfk_canon as K
import cfk_store_model as M

SEEDS = list(range(20))


def _rows_of_snapshot(rows):
    return [(t, s, ex, list(m)) for t, _dom, s, ex, m in rows]


@pytest.mark.parametrize("seed", [0, 7, 13])
def test_store_model_replays_the_harness(seed):
    r = K.Run(seed, 1000, snapshot_every=25, log=True)
    model = M.StoreModel()
    snaps = {ev: rows for ev, rows, _, _ in r.snapshots}
    checked = 0
    for e, evs in enumerate(r.event_log, start=1):
        for ev in evs:
            model.apply(ev)
        if e in snaps:
            assert model.rows() == _rows_of_snapshot(snaps[e]), "seed %d step %d" % (seed, e)
            checked += 1
    assert checked > 50
    assert sum(len(m) for *_x, m in model.rows()) > 100          # missing() sets are exercised


PRUNE_SEEDS = list(range(20))


def _lp_state(cfk):
    pos = {t: k for k, t in enumerate(cfk.ids)}
    return (cfk.pruned_before, {lid: sorted(pos[w] for w in wit if w in pos) for lid, wit in cfk.loading.items()})


@pytest.mark.parametrize("seed", [1, 4, 7, 19])
def test_store_model_replays_the_pruned_harness(seed):
    r = K.Run(seed, 1000, snapshot_every=25, log=True, prune=True)
    assert r.cfk.prunes > 0
    model = M.StoreModel()
    snaps = {ev: rows for ev, rows, _, _ in r.snapshots}
    checked = 0
    for e, evs in enumerate(r.event_log, start=1):
        for ev in evs:
            model.apply(ev)
        if e in snaps:
            assert model.rows() == _rows_of_snapshot(snaps[e]), "seed %d step %d" % (seed, e)
            checked += 1
    assert checked > 50
    pb, lp = _lp_state(r.cfk)
    assert model.pruned_before == pb
    pos = {t: k for k, t in enumerate(model.ids)}
    got = {}
    for lid, b in zip(model.lp_id, model.lp_bits):
        got[lid] = sorted(pos[model.slot_txn[s]] for s in range(b.bit_length()) if (b >> s) & 1)
    assert got == lp


def test_pruned_harness_notifications_follow_the_full_scan():
    """Under pruning the event-driven notifications may lag the full scan while a pruned TxnId loads (a load that
    completes re-notifies nothing, CommandsForKey.java:1121-1128), never lead it."""
    lag = 0
    for seed in (2, 6, 8):
        r = K.Run(seed, 1000, prune=True, check_full_scan=True)
        assert r.cfk.prunes > 0 and r.loads > 0
        for _ev, extra, missing in r.full_scan_mismatches:
            assert not missing
            lag += len(extra)
    assert lag > 0


def _device_rows(d, domains_rev):
    out = []
    for i in range(len(d["status"])):
        out.append(((int(d["txn_msb"][i]), int(d["txn_lsb"][i]), int(d["txn_node"][i])), int(d["status"][i]),
                    (int(d["exec_msb"][i]), int(d["exec_lsb"][i]), int(d["exec_node"][i])),
                    [int(x) for x in d["missing"][d["miss_off"][i]:d["miss_off"][i + 1]]]))
    return out


def _bits_rows(rows, domains):
    out = []
    for t, dom, s, ex, m in rows:
        exb = K.ts_bits(ex, dom) if ex == t else K.ts_bits(ex)
        out.append((K.ts_bits(t, dom), s, exb, list(m)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("chunk,prune", [(0, False), (1, False), (0, True), (1, True)])
def test_gpu_store_follows_the_harness(engine_factory, chunk, prune):
    seeds = (PRUNE_SEEDS if prune else SEEDS)[chunk * 10:(chunk + 1) * 10]
    runs = [K.Run(seed, 1000, snapshot_every=25, log=True, prune=prune) for seed in seeds]
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
    cap = max(r.max_rows for r in runs) + 64
    eng.cfk_store_open(len(runs), cap)
    snaps = [{ev: (rows, want, full) for ev, rows, want, full in r.snapshots} for r in runs]
    steps = max(len(r.event_log) for r in runs)
    checked = released = 0
    for e in range(1, steps + 1):
        per_key = [r.event_log[e - 1] if e <= len(r.event_log) else [] for r in runs]
        # one domain map for the packing: each run's own (TxnIds are per key)
        ev = [M.pack_events([evs], r.domains) for evs, r in zip(per_key, runs)]
        merged = {f: np.concatenate([x[f] for x in ev]) if f not in ("ev_off", "deps_off") else None for f in ev[0]}
        off = [0]
        doff = [0]
        for x in ev:
            off.append(off[-1] + len(x["status"]))
            doff.extend((x["deps_off"][1:] + doff[-1]).tolist())
        merged["ev_off"] = np.array(off, np.uint32)
        merged["deps_off"] = np.array(doff, np.uint32)
        eng.cfk_store_apply(merged)
        due = [k for k in range(len(runs)) if e in snaps[k]]
        if not due:
            continue
        nrows, out = eng.cfk_store_notify()
        for k in due:
            rows, want, full = snaps[k][e]
            d = eng.cfk_store_fetch(k)
            assert _device_rows(d, None) == _bits_rows(rows, runs[k].domains), "seed %d step %d: rows" % (seeds[k], e)
            assert int(nrows[k]) == len(rows)
            dev = {rows[i][0] for i in np.nonzero(out[k, :len(rows)])[0]}
            if prune:
                assert dev == set(full), "seed %d step %d: device %s, full scan %s" % (
                    seeds[k], e, sorted(dev - set(full))[:3], sorted(set(full) - dev)[:3])
                assert set(want) <= dev
            else:
                assert dev == set(want), "seed %d step %d: device %s, harness %s" % (
                    seeds[k], e, sorted(dev - set(want))[:3], sorted(set(want) - dev)[:3])
                assert dev == set(full)
            released += len(dev)
            checked += 1
    assert checked > 500 and released > 100
    if prune:
        assert sum(r.cfk.prunes for r in runs) > 0
        for k, r in enumerate(runs):
            d = eng.cfk_store_pruning(k)
            pb, lp = _lp_state(r.cfk)
            assert d["pruned_before"] == K.ts_bits(pb, r.domains[pb]) if pb != K.NONE else d["pruned_before"] == (0, 0, 0)
            got = {}
            for j in range(len(d["lp_msb"])):
                got[(int(d["lp_msb"][j]), int(d["lp_lsb"][j]), int(d["lp_node"][j]))] = \
                    [int(x) for x in d["lp_rows"][d["lp_off"][j]:d["lp_off"][j + 1]]]
            assert got == {K.ts_bits(lid, r.domains[lid]): w for lid, w in lp.items()}
