"""profiles/shard_levels.py S PER_STORE [levels...] — the cross-store protocol of S key-range stores in one process
(LocalTransport, one GPU): C5's generator (4 uniform keys over 10^7) at S x PER_STORE txns, per level protocol the
phase seconds summed over the stores (divide by S for one GPU's share), the level-edge count (gather) or the delta
pairs sent (rounds), and the rounds.  A measurement recipe (GPU box), not a test."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import sharding, workload  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4
per = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
protos = sys.argv[3:] or ["gather", "rounds", "auto"]
w, r, p, seed = 32, 3, 0.1, workload.SEEDS["C5"]
b = workload.generate(S * per, 4, 10_000_000, "uniform", seed=seed)
bounds = sharding.even_bounds(0, 10_000_000, S)
hs = sharding.home_stores(b, bounds)
masks = sharding.holder_masks(b, bounds)
for proto in protos:
    stores = []
    for k in range(S):
        local, gid, _ = sharding.slice_for_shard(b, bounds[k], bounds[k + 1])
        st = sharding.ShardStore(0, window=w, replicas=r, drop_p=p, seed=seed)
        st.load(local, gid, hs[gid], b["n"], k, S, holders=masks[gid] if proto in ("rounds", "kahn", "auto") else None)
        stores.append(st)
    for rep in range(2):                                   # the first is a warm-up
        tm = {}
        t0 = time.perf_counter()
        rounds = sharding.LocalTransport.run(stores, levels=proto, timings=tm)
        dt = time.perf_counter() - t0
    rec = {"proto": proto, "stores": S, "txns": int(b["n"]), "rounds": rounds, "wall_s": dt,
           "phases_s_summed": {k: round(v, 4) for k, v in tm.items()},
           "local_txns": [int(st.gid.size) for st in stores],
           "pairs_sent": [int(getattr(st, "pairs_sent", 0)) for st in stores], "kahn_bytes": [int(getattr(st, "kahn_bytes", 0)) for st in stores], "depth": int(getattr(stores[0], "depth", 0) or 0)}
    print(json.dumps(rec), flush=True)
    for st in stores:
        st.close()
