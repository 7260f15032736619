"""Debug: replay pruned Canon seeds on the device store step by step; report the first divergence from the host model."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "cassandra-accord_amd"))
import numpy as np
import cfk_canon as K, cfk_store_model as M
from accord_amd import engine, abi

seeds = [int(x) for x in sys.argv[1:]] or list(range(10))
runs = [K.Run(s, 1000, log=True, prune=True) for s in seeds]
models = [M.StoreModel() for _ in runs]
eng = engine.DepsEngine(window=0, replicas=1, drop_p=0.0, seed=1)
cap = max(r.max_rows for r in runs) + 64
eng.cfk_store_open(len(runs), cap)
steps = max(len(r.event_log) for r in runs)
for e in range(1, steps + 1):
    per_key = [r.event_log[e - 1] if e <= len(r.event_log) else [] for r in runs]
    ev = [M.pack_events([evs], r.domains) for evs, r in zip(per_key, runs)]
    merged = {f: np.concatenate([x[f] for x in ev]) for f in ev[0] if f not in ("ev_off", "deps_off")}
    off, doff = [0], [0]
    for x in ev:
        off.append(off[-1] + len(x["status"]))
        doff.extend((x["deps_off"][1:] + doff[-1]).tolist())
    merged["ev_off"] = np.array(off, np.uint32)
    merged["deps_off"] = np.array(doff, np.uint32)
    for m, evs in zip(models, per_key):
        for x in evs:
            m.apply(x)
    try:
        eng.cfk_store_apply(merged)
    except Exception as exc:
        print("step", e, "apply error", exc)
    nrows, _ = eng.cfk_store_notify()
    bad = [k for k in range(len(runs)) if int(nrows[k]) != len(models[k].ids)]
    if bad:
        k = bad[0]
        print("step", e, "seed", seeds[k], "device rows", int(nrows[k]), "model rows", len(models[k].ids))
        print("events:", [(x[0], x[1], x[4:] if len(x) > 4 else "") for x in per_key[k]])
        d = eng.cfk_store_pruning(k)
        print("device pb", d["pruned_before"], "model pb", K.ts_bits(models[k].pruned_before, runs[k].domains.get(models[k].pruned_before, 0)) if models[k].pruned_before != K.NONE else 0)
        print("device loading", len(d["lp_msb"]), "model loading", len(models[k].lp_id))
        dr = eng.cfk_store_fetch(k)
        dev = [(int(dr["txn_msb"][i]), int(dr["txn_lsb"][i]), int(dr["txn_node"][i]), int(dr["status"][i])) for i in range(len(dr["status"]))]
        mod = [K.ts_bits(t, runs[k].domains[t]) + (row[0],) for t, row in zip(models[k].ids, models[k].row)]
        for i, (a, b) in enumerate(zip(dev, mod)):
            if a != b:
                print("first row diff at", i, "device", a, "model", b)
                break
        break
else:
    print("no divergence over", steps, "steps")
