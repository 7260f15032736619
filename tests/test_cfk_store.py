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


def _record(name, doc):
    """Counts a GPU test reports (gpurun_out/test_records/NAME.json when the directory can be made)."""
    import json
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "test_records")
    try:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".json"), "w") as f:
            json.dump(doc, f)
    except OSError:
        pass


def test_pruned_release_sets_keep_the_execution_invariants():
    """CPU: at every sampled step of 6 pruned seeds (including the steps where the event-driven notifications lag it),
    the full-scan release set — what ad_cfk_store_notify computes, checked equal on the GPU — satisfies the reference's
    execution-order invariants (CommandsForKeyTest.java:175-180, 206-218); some steps release txns not yet notified."""
    extras = 0
    for seed in (2, 4, 6, 8, 11, 17):
        r = K.Run(seed, 1000, snapshot_every=25, prune=True, snapshot_lag=True)
        for ev, _rows, want, full in r.snapshots:
            assert not K.release_invariant_violations(r.canon_views[ev], full), "seed %d step %d" % (seed, ev)
            extras += len(set(full) - set(want))
    assert extras > 0


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
# (1000 events: ~850 rows per key, the HBM-resident apply kernel; 240 events: <= 256 rows, the LDS-resident one;
# tiered: every key starts in a small regular tier and moves to the large tier mid-stream, within an apply call —
# 1000 events: 128-row LDS tier -> HBM large tier; 240 events: 64 -> 256 rows, LDS both)
@pytest.mark.parametrize("chunk,prune,events,tiered", [(0, False, 1000, False), (1, False, 1000, False),
                                                       (0, True, 1000, False), (1, True, 1000, False),
                                                       (0, False, 240, False), (0, True, 240, False),
                                                       (1, False, 1000, True), (1, True, 1000, True),
                                                       (0, True, 240, True)])
def test_gpu_store_follows_the_harness(engine_factory, chunk, prune, events, tiered):
    seeds = (PRUNE_SEEDS if prune else SEEDS)[chunk * 10:(chunk + 1) * 10]
    runs = [K.Run(seed, events, snapshot_every=25 if events >= 1000 else 8, log=True, prune=prune, snapshot_lag=prune)
            for seed in seeds]
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
    cap = max(r.max_rows for r in runs) + 64
    if events < 1000:
        assert max(r.max_rows for r in runs) <= 256
        cap = 256
    extras = 0
    if tiered:
        small = 128 if events >= 1000 else 64
        eng.cfk_store_open(len(runs), small, big_capacity=cap, big_keys=len(runs))
    else:
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
            flags = eng.cfk_store_notify_key(k) if tiered else out[k, :len(rows)]
            assert len(flags) == len(rows)
            dev = {rows[i][0] for i in np.nonzero(flags)[0]}
            if prune:
                assert dev == set(full), "seed %d step %d: device %s, full scan %s" % (
                    seeds[k], e, sorted(dev - set(full))[:3], sorted(set(full) - dev)[:3])
                assert set(want) <= dev
                # the device's release set — including the txns the event-driven harness has not notified yet (a
                # pruned TxnId loading) — keeps the reference's own execution-order invariants
                # (CommandsForKeyTest.java:175-180, 206-218) against Canon's committed commands at this step
                bad = K.release_invariant_violations(runs[k].canon_views[e], [rows[i][0] for i in np.nonzero(flags)[0]])
                assert not bad, "seed %d step %d: %s" % (seeds[k], e, bad[:3])
                extras += len(dev - set(want))
            else:
                assert dev == set(want), "seed %d step %d: device %s, harness %s" % (
                    seeds[k], e, sorted(dev - set(want))[:3], sorted(set(want) - dev)[:3])
                assert dev == set(full)
            released += len(dev)
            checked += 1
    assert checked > 500 and released > 100
    if prune:
        assert sum(r.cfk.prunes for r in runs) > 0
        _record("store_release_extras_chunk%d" % chunk, {"seeds": seeds, "sampled_steps": checked,
                                                          "released": released, "not_yet_notified_released": extras,
                                                          "lag_events": sum(r.lag_events for r in runs)})
        for k, r in enumerate(runs):
            d = eng.cfk_store_pruning(k)
            pb, lp = _lp_state(r.cfk)
            assert d["pruned_before"] == K.ts_bits(pb, r.domains[pb]) if pb != K.NONE else d["pruned_before"] == (0, 0, 0)
            got = {}
            for j in range(len(d["lp_msb"])):
                got[(int(d["lp_msb"][j]), int(d["lp_lsb"][j]), int(d["lp_node"][j]))] = \
                    [int(x) for x in d["lp_rows"][d["lp_off"][j]:d["lp_off"][j + 1]]]
            assert got == {K.ts_bits(lid, r.domains[lid]): w for lid, w in lp.items()}


# ---- mapReduceActive over the resident rows (ad_cfk_store_query) ------------------------------------------------------
QKINDS = (K.READ, K.WRITE, K.EPH, K.SYNC, K.ESP)


def store_queries(states, rng):
    """Queries against the CFK states of one lockstep step (states[k]: key k's CFK, None when its run has ended):
    per key, PreAccept queries of existing rows (bound = TxnId), fresh TxnIds of every kind beside rows (bound = TxnId),
    ExclusiveSyncPoints at and below prunedBefore (the future-dependency branch, CommandsForKey.java:967-980), Accept
    queries of committed rows (bound = executeAt, the txn itself left out: PreAccept.calculatePartialDeps :256-261);
    plus fresh TxnIds over 2-3 keys at once (the Deps.Builder union across keys).  -> [(keys, txn, bound)]"""
    out = []
    live = [k for k, c in enumerate(states) if c is not None and c.ids]
    for k in live:
        c = states[k]
        ids = c.ids
        for t in rng.choice(len(ids), size=min(3, len(ids)), replace=False):
            out.append(([k], ids[t], ids[t]))
        for _ in range(3):
            e, h, _f, n = ids[int(rng.integers(len(ids)))]
            kind = QKINDS[int(rng.integers(len(QKINDS)))]
            t = (e, h + int(rng.integers(0, 3)), kind << 1, n + int(rng.integers(-1, 2)))
            out.append(([k], t, t))
        if c.pruned_before != K.NONE:
            e, h, _f, n = c.pruned_before
            for d in (0, 1, 7):
                t = (e, max(0, h - d), K.ESP << 1, n)
                out.append(([k], t, t))
        com = [t for t in ids if c.info[t].status in (K.COMMITTED, K.STABLE, K.APPLIED) and c.info[t].execute_at != t]
        for t in (rng.choice(len(com), size=min(2, len(com)), replace=False) if com else []):
            out.append(([k], com[t], c.info[com[t]].execute_at))
    for _ in range(4):
        if len(live) < 2:
            break
        ks = sorted(rng.choice(live, size=min(len(live), int(rng.integers(2, 4))), replace=False).tolist())
        ids = states[ks[0]].ids
        e, h, _f, n = ids[int(rng.integers(len(ids)))]
        kind = QKINDS[int(rng.integers(len(QKINDS)))]
        t = (e, h, kind << 1, n)
        out.append((ks, t, t))
    return out


def expected_query(states, keys, txn, bound):
    """Deps.Builder over mapReduceActive per key: [keyDeps, directKeyDeps] as (keys, TxnIds, keysToTxnIds)."""
    kinds = K._WITNESSES[K.kind_of(txn)]
    per = [(k, states[k].map_reduce_active(bound, kinds, None if bound == txn else txn)) for k in keys]
    res = []
    for cls in (0, 1):
        lists = [(k, [t for t in lst if (K.kind_of(t) in (K.READ, K.WRITE)) == (cls == 0)]) for k, lst in per]
        lists = [(k, lst) for k, lst in lists if lst]
        u = sorted({t for _, lst in lists for t in lst})
        pos = {t: i for i, t in enumerate(u)}
        head, body, run = [], [], len(lists)
        for _, lst in lists:
            body.extend(pos[t] for t in lst)
            run += len(lst)
            head.append(run)
        res.append(([k for k, _ in lists], u, head + body))
    return res


def future_dep_fires(cfk, bound):
    return bound <= cfk.pruned_before and cfk.max_applied_write(cfk.committed()) >= 0


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [0, 1])
def test_gpu_store_queries_follow_map_reduce_active(engine_factory, chunk):
    """The 20 pruned Canon seeds (10 per chunk) as keys of one store; every 25 harness steps, PreAccept / Accept /
    ExclusiveSyncPoint queries against the resident rows (ad_cfk_store_query) == the restated CFK's mapReduceActive
    through Deps.Builder, keyDeps and directKeyDeps, including the prunedBefore future dependency."""
    seeds = PRUNE_SEEDS[chunk * 10:(chunk + 1) * 10]
    runs = [K.Run(seed, 1000, log=True, prune=True, keep_states_every=25) for seed in seeds]
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
    eng.cfk_store_open(len(runs), max(r.max_rows for r in runs) + 64)
    rng = np.random.default_rng(chunk)
    steps = max(len(r.event_log) for r in runs)
    nq = fut = multi = entries = 0
    for e in range(1, steps + 1):
        per_key = [r.event_log[e - 1] if e <= len(r.event_log) else [] for r in runs]
        ev = [M.pack_events([evs], r.domains) for evs, r in zip(per_key, runs)]
        merged = {f: np.concatenate([x[f] for x in ev]) if f not in ("ev_off", "deps_off") else None for f in ev[0]}
        off, doff = [0], [0]
        for x in ev:
            off.append(off[-1] + len(x["status"]))
            doff.extend((x["deps_off"][1:] + doff[-1]).tolist())
        merged["ev_off"] = np.array(off, np.uint32)
        merged["deps_off"] = np.array(doff, np.uint32)
        eng.cfk_store_apply(merged)
        states = [r.states.get(e) for r in runs]
        if not any(s is not None for s in states):
            continue
        qs = store_queries(states, rng)
        key_off = np.cumsum([0] + [len(ks) for ks, _, _ in qs]).astype(np.uint32)
        keys = np.array([k for ks, _, _ in qs for k in ks], np.uint32)
        tb = [K.ts_bits(t) for _, t, _ in qs]
        bb = [K.ts_bits(b) for _, _, b in qs]
        txn = tuple(np.array([x[i] for x in tb], dt) for i, dt in enumerate((np.uint64, np.uint64, np.int32)))
        bound = tuple(np.array([x[i] for x in bb], dt) for i, dt in enumerate((np.uint64, np.uint64, np.int32)))
        got = eng.cfk_store_query(key_off, keys, txn, bound)
        for q, (ks, t, b) in enumerate(qs):
            want = expected_query(states, ks, t, b)
            for cls in (0, 1):
                g = got[cls]
                wk, wu, wm = want[cls]
                gk = [int(x) for x in g["keys"][g["key_off"][q]:g["key_off"][q + 1]]]
                gm = [int(x) for x in g["k2t"][g["k2t_off"][q]:g["k2t_off"][q + 1]]]
                lo, hi = g["txn_off"][q], g["txn_off"][q + 1]
                gu = [(int(g["txn_msb"][i]), int(g["txn_lsb"][i]), int(g["txn_node"][i])) for i in range(lo, hi)]
                assert (gk, gu, gm) == (wk, [K.ts_bits(x) for x in wu], wm), \
                    "seeds %s step %d query %d (keys %s, txn %s, bound %s) class %d" % (seeds, e, q, ks, t, b, cls)
                entries += len(wu)
            nq += 1
            multi += len(ks) > 1
            fut += any(future_dep_fires(states[k], b) for k in ks)
    assert nq > 1000 and multi > 50 and entries > 1000
    assert fut > 20                                       # the prunedBefore branch was taken


# ---- unmanaged txns on the device (AD_CFK_OP_UNMANAGED*, notifyUnmanaged) -------------------------------------------------
def _pack_step(runs, e):
    per_key = [r.event_log[e - 1] if e <= len(r.event_log) else [] for r in runs]
    ev = [M.pack_events([evs], r.domains) for evs, r in zip(per_key, runs)]
    merged = {f: np.concatenate([x[f] for x in ev]) if f not in ("ev_off", "deps_off") else None for f in ev[0]}
    off, doff = [0], [0]
    for x in ev:
        off.append(off[-1] + len(x["status"]))
        doff.extend((x["deps_off"][1:] + doff[-1]).tolist())
    merged["ev_off"] = np.array(off, np.uint32)
    merged["deps_off"] = np.array(doff, np.uint32)
    return merged


def test_harness_logs_unmanaged_registrations():
    """CPU: the harness's event log carries every registerUnmanaged / updateUnmanaged call (AD_CFK_OP_UNMANAGED*), and its
    notifications (commit, applied, ready) occur, with and without pruning."""
    for prune in (False, True):
        reg = notes = 0
        tags = set()
        for seed in (1, 4, 7):
            r = K.Run(seed, 1000, log=True, prune=prune)
            reg += sum(1 for evs in r.event_log for ev in evs if len(ev) > 4 and ev[4] in (K.OP_UNMANAGED, K.OP_UNMANAGED_RECHECK))
            notes += sum(len(x) for x in r.note_log)
            tags |= {t for x in r.note_log for t, _ in x}
        assert reg > 100 and notes > 100 and tags == {0, 1, 2}, (prune, reg, notes, tags)


@pytest.mark.gpu
@pytest.mark.parametrize("prune", [False, True])
def test_gpu_store_unmanaged_follow_the_harness(engine_factory, prune):
    """20 Canon seeds as 20 keys, lockstep: after every harness step the device's unmanaged notifications (in order, per key)
    == the restated notifyUnmanaged / updateUnmanaged's (PostProcess.java:164-246, Updating.java:715-849), and every 25
    steps the device's unmanaged registry == the restated CFK's unmanageds."""
    seeds = PRUNE_SEEDS if prune else SEEDS
    runs = [K.Run(seed, 1000, log=True, prune=prune, keep_states_every=25) for seed in seeds]
    eng = engine_factory(window=0, replicas=1, drop_p=0.0, seed=1)
    eng.cfk_store_open(len(runs), max(r.max_rows for r in runs) + 64)
    steps = max(len(r.event_log) for r in runs)
    seen, regs, tags = 0, 0, {0: 0, 1: 0, 2: 0}
    for e in range(1, steps + 1):
        eng.cfk_store_apply(_pack_step(runs, e))
        got = eng.cfk_store_notified()
        for k, r in enumerate(runs):
            want = [(t, K.ts_bits(u, r.domains[u])) for t, u in (r.note_log[e - 1] if e <= len(r.note_log) else [])]
            assert [(t, u) for _ev, t, u in got[k]] == want, "seed %d step %d" % (seeds[k], e)
            seen += len(want)
            for t, _ in want:
                tags[t] += 1
            st = r.states.get(e)
            if st is not None:
                reg = eng.cfk_store_unmanaged(k)
                assert reg == [(p, K.ts_bits(w), K.ts_bits(u, r.domains[u])) for p, w, u in st.unmanageds], \
                    "seed %d step %d: registry" % (seeds[k], e)
                regs += len(reg)
    assert seen > 500 and regs > 100 and min(tags.values()) > 20, (seen, regs, tags)
    _record("store_unmanaged_%s" % ("prune" if prune else "plain"), {"notifications": seen, "by_tag": tags,
                                                                      "registry_entries_checked": regs})
