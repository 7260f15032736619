"""profiles/level_modes.py CFG [n] — the level stage of one config under each level algorithm (ad_set_level_mode):
per mode the pipeline ms/step, the level stage ms and its iteration / block / round counts.  A measurement recipe
(GPU box), not a test."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import engine, workload  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else None
b = workload.config(cfg, n=n)
out = {}
for name, mode in (("auto", 0), ("fixpoint", 1), ("blocks", 2), ("kahn", 3)):
    eng = engine.DepsEngine(device=0, window=32, replicas=3, drop_p=0.1, seed=workload.SEEDS[cfg])
    eng.load(b)
    eng.set_level_mode(mode)
    eng.run_pipeline()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        eng.run_pipeline()
        ts.append(time.perf_counter() - t0)
    st = eng.last_times()
    lv, _ = eng.fetch_levels()
    out[name] = {"ms": 1e3 * min(ts), "levels_ms": st["levels"], "iterations": st["level_iterations"],
                 "blocks": st["level_blocks"], "rounds": st["level_rounds"], "path": st["level_path"],
                 "depth": int(lv.max()) + 1}
    print(name, json.dumps(out[name]), flush=True)
    eng.close()
