#!/usr/bin/env python3
"""Throughput of the device-resident CommandsForKey store (ad_cfk_store_apply) on a C3-distributed
event stream: events/s, with the hottest key's serial chain named.

Stream (seeded, synthetic): BASELINE configs[2]'s generator — 1,048,576 txns x 4 keys, Zipf(0.99) over 10^7 keys,
50 % Reads / Writes — replayed as the CommandsForKey.update calls a replica makes (CommandsForKey.java:987-1057): txn i
is PreAccepted at step i, Committed and Stable (executeAt = TxnId, deps = the earlier txns on the key within the
in-flight window W that it witnesses, Kind.witnesses — on the Commit update) at step i + W, Applied at step i + 2W;
after every Apply a maybePrune(4, 0) event on the key (Pruning.java:164-233) keeps each key's rows near its in-flight
set.  Every
(txn, key) pair is one event per transition on its key: ~21 M events over ~1.1 M keys.  Events go to the store in
calls of `--batch` txns' steps, grouped by key; keys are applied in parallel (one workgroup each) and each key's
events in order — the hottest key (~200 k pairs, ~1 M events) is a serial chain, as it is in the reference (one
CommandsForKey per key, updated copy-on-write per event).

Timing: wall time of the ad_cfk_store_apply calls (upload + kernel + the completion sync), the packing of the next
call excluded (done before the timed loop).  Prints one JSON object."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))

import numpy as np  # noqa: E402

from accord_amd import abi, engine, workload  # noqa: E402

ST_PREACC, ST_COMMITTED, ST_STABLE, ST_APPLIED = 2, 4, 5, 6
DEP_LAGS = 8


def build_stream(n, window):
    b = workload.config("C3", n=n)
    keys = np.asarray(b["keys"])
    key_off = np.asarray(b["key_off"], np.int64)
    P = len(keys)
    ptxn = np.repeat(np.arange(n, dtype=np.int64), np.diff(key_off))
    uk, kidx = np.unique(keys, return_inverse=True)
    K = len(uk)
    kind = ((np.asarray(b["txn_lsb"]) >> np.uint64(1)) & np.uint64(7)).astype(np.int64)
    order = np.lexsort((ptxn, kidx))                 # pairs by (key, txn)
    sk, st = kidx[order], ptxn[order]
    # deps of pair p (its txn i on key k): the earlier pairs on k with txn > i - W that i's kind witnesses
    # (a Read witnesses Writes, a Write Reads and Writes), ascending
    dep = np.full((P, DEP_LAGS), -1, np.int64)
    for d in range(1, DEP_LAGS + 1):
        prev_k = np.concatenate([np.full(d, -1), sk[:-d]])
        prev_t = np.concatenate([np.full(d, -1), st[:-d]])
        ok = (prev_k == sk) & (prev_t > st - window)
        ok &= (kind[st] == abi.KIND_WRITE) | (kind[np.maximum(prev_t, 0)] == abi.KIND_WRITE)
        dep[order, DEP_LAGS - d] = np.where(ok, prev_t, -1)   # lag d at column DEP_LAGS - d: ascending txn
    return b, K, kidx, ptxn, dep


def pack_call(b, kidx, ptxn, dep, key_off, s0, s1, window, K):
    """The events of steps [s0, s1): PreAccept of txns [s0, s1), Commit + Stable of [s0 - W, s1 - W), Apply (+ prune)
    of [s0 - 2W, s1 - 2W) — grouped by key, in (step, transition) order within a key."""
    tm, tl, tn = (np.asarray(b[f]) for f in ("txn_msb", "txn_lsb", "txn_node"))
    n = len(tm)
    parts = []
    for shift, trans in ((0, (0,)), (window, (1, 2)), (2 * window, (3, 4))):
        lo, hi = max(s0 - shift, 0), min(max(s1 - shift, 0), n)
        if hi <= lo:
            continue
        pr = np.arange(key_off[lo], key_off[hi], dtype=np.int64)
        for tr in trans:
            parts.append(np.stack([pr, np.full(len(pr), tr, np.int64)], 1))
    if not parts:
        return None
    ev = np.concatenate(parts)
    pair, tr = ev[:, 0], ev[:, 1]
    step = ptxn[pair] + np.array([0, window, window, 2 * window, 2 * window])[tr]
    o = np.lexsort((tr, ptxn[pair], step, kidx[pair]))
    pair, tr = pair[o], tr[o]
    key = kidx[pair]
    t = ptxn[pair]
    m = len(pair)
    status = np.array([ST_PREACC, ST_COMMITTED, ST_STABLE, ST_APPLIED, 0], np.uint8)[tr]
    op = np.where(tr == 4, abi.CFK_OP_PRUNE, abi.CFK_OP_UPDATE).astype(np.uint8)
    prune = tr == 4
    out = {"txn_msb": np.where(prune, 0, tm[t]).astype(np.uint64), "txn_lsb": np.where(prune, 0, tl[t]).astype(np.uint64),
           "txn_node": np.where(prune, 0, tn[t]).astype(np.int32), "status": status, "op": op,
           # executeAt = TxnId (fast path); a PRUNE event: interval 4 in exec_node, minHlcDelta 0 in exec_msb
           "exec_msb": np.where(prune, 0, tm[t]).astype(np.uint64), "exec_lsb": np.where(prune, 0, tl[t]).astype(np.uint64),
           "exec_node": np.where(prune, 4, tn[t]).astype(np.int32)}
    # deps on the Commit; the Stable / Apply updates carry none: by then every witnessed txn below the command is decided
    # (committed at its own step + W), so the rebuilt missing() is empty either way, and re-sending deps that pruning
    # already removed would only queue loads of them (LoadPruned) this stream does not model
    with_deps = tr == 1
    d = np.where(with_deps[:, None], dep[pair], -1)
    cnt = (d >= 0).sum(1)
    doff = np.zeros(m + 1, np.uint32)
    np.cumsum(cnt, out=doff[1:])
    dd = d[d >= 0]                                    # row-major: each event's deps ascending
    out["deps_off"] = doff
    out["deps_msb"], out["deps_lsb"], out["deps_node"] = tm[dd].astype(np.uint64), tl[dd].astype(np.uint64), tn[dd].astype(np.int32)
    ev_off = np.zeros(K + 1, np.uint32)
    np.cumsum(np.bincount(key, minlength=K), out=ev_off[1:])
    out["ev_off"] = ev_off
    return out, int(np.bincount(key, minlength=K).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--txns", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=16384, help="txns' steps per ad_cfk_store_apply call")
    ap.add_argument("--window", type=int, default=32)
    ap.add_argument("--cap", type=int, default=128, help="rows per key")
    ap.add_argument("--calls", type=int, default=0, help="stop after this many calls (0: the whole stream)")
    args = ap.parse_args()
    t0 = time.perf_counter()
    b, K, kidx, ptxn, dep = build_stream(args.txns, args.window)
    key_off = np.asarray(b["key_off"], np.int64)
    n = args.txns
    calls = []
    s = 0
    end = n + 2 * args.window
    while s < end and (not args.calls or len(calls) < args.calls):
        c = pack_call(b, kidx, ptxn, dep, key_off, s, min(s + args.batch, end), args.window, K)
        if c is not None:
            calls.append(c)
        s += args.batch
    t_pack = time.perf_counter() - t0
    eng = engine.DepsEngine(device=0, window=0, replicas=1, drop_p=0.0, seed=1)
    eng.cfk_store_open(K, args.cap)
    ev_total = sum(len(c[0]["status"]) for c in calls)
    hot = sum(c[1] for c in calls)
    per_call = []
    t1 = time.perf_counter()
    for ev, _ in calls:
        a = time.perf_counter()
        eng.cfk_store_apply(ev)
        per_call.append(time.perf_counter() - a)
    dt = time.perf_counter() - t1
    rows, _ = eng.cfk_store_notify()
    eng.close()
    print(json.dumps({
        "what": "ad_cfk_store_apply on a C3-distributed CommandsForKey.update stream (profiles/store_bench.py docstring)",
        "txns": n, "keys": K, "window": args.window, "cap_rows_per_key": args.cap, "calls": len(calls),
        "events": ev_total, "seconds": dt, "events_per_s": ev_total / dt,
        "hottest_key_events": hot, "hottest_key_serial_us_per_event": dt / hot * 1e6,
        "call_ms": {"min": min(per_call) * 1e3, "median": float(np.median(per_call)) * 1e3, "max": max(per_call) * 1e3},
        "max_rows_at_end": int(rows.max()), "pack_s": t_pack}))


if __name__ == "__main__":
    main()
