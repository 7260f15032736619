"""Scratch bisection of a deps parity miss (EphemeralRead + range txns, window 16)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cassandra-accord_amd")]
import numpy as np
import oracle as O
from accord_amd import abi, workload, engine


def run(b, window, name):
    cfg = abi.make_config(window, 3, 0.1, 0xACC0D1)
    ref = O.OracleResult(b, cfg, O.FLAG_MERGE)
    e = engine.DepsEngine(window=window, replicas=3, drop_p=0.1, seed=0xACC0D1)
    e.load(b)
    e.preaccept_deps()
    bad = []
    for v in range(3):
        for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY, abi.CLASS_RANGE):
            g, w = e.fetch_deps(v, c), ref.deps(v, c)
            if not g.equal(w):
                i = g.first_difference(w)
                bad.append((v, c, i))
    print(name, "window", window, "bad", bad[:4], e.last_times().get("key_classes"), flush=True)
    e.close()


n = 6000
rng = np.random.default_rng(77)
kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ], size=n, p=[0.45, 0.45, 0.1])
base = dict(range_frac=0.1, range_width_max=100, seed=77)
run(workload.generate(n, 3, 5000, "uniform", kinds=kinds, **base), 16, "eph+ranges")
run(workload.generate(n, 3, 5000, "uniform", kinds=kinds, **base), 32, "eph+ranges")
k2 = np.where(kinds == abi.KIND_EPHEMERAL_READ, abi.KIND_READ, kinds)
run(workload.generate(n, 3, 5000, "uniform", kinds=k2, **base), 16, "no-eph+ranges")
run(workload.generate(n, 3, 5000, "uniform", kinds=kinds, seed=77), 16, "eph-no-ranges")
b = workload.generate(n, 3, 5000, "uniform", kinds=kinds, **base)
dom = (b["txn_lsb"] & np.uint64(1)).astype(bool)
k3 = kinds.copy(); k3[dom] = abi.KIND_READ
run(workload.generate(n, 3, 5000, "uniform", kinds=k3, **base), 16, "eph-keys-only+range-reads")
k4 = kinds.copy(); k4[~dom & (kinds == abi.KIND_EPHEMERAL_READ)] = abi.KIND_READ
run(workload.generate(n, 3, 5000, "uniform", kinds=k4, **base), 16, "eph-ranges-only")
