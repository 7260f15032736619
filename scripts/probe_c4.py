"""Probe: BASELINE configs[3] (C4, mixed key + range txns) at a given size through the staged engine calls;
prints CSR sizes and stage times.  Usage: python scripts/probe_c4.py N"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
from accord_amd import abi, engine, workload

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
t0 = time.time()
b = workload.config("C4", n=n)
print("gen %.1fs n=%d P=%d Q=%d" % (time.time() - t0, n, len(b["keys"]), len(b["range_start"])), flush=True)
with engine.DepsEngine(0, 32, 3, 0.1, workload.SEEDS["C4"]) as eng:
    eng.load(b)
    for it in range(2):
        t = time.time(); s = eng.preaccept_deps(); td = time.time() - t
        print("deps %.3fs" % td, [(x.keys, x.k2t, x.txns) for x in s], flush=True)
        t = time.time(); m = eng.merge(); tm = time.time() - t
        print("merge %.3fs" % tm, [(x.keys, x.k2t, x.txns) for x in m], flush=True)
        t = time.time(); lv, order, iters = eng.exec_levels(); tl = time.time() - t
        print("levels %.3fs iters=%d maxlevel=%d" % (tl, iters, lv.max()), flush=True)
