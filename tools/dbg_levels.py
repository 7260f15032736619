"""Debug: where GPU exec levels differ from the oracle on mixed-kind batches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cassandra-accord_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
from accord_amd import abi, engine, workload  # noqa: E402


def run(b, window, fix=False):
    cfg = abi.make_config(window, 3, 0.1, 0xACC0D1)
    ref = O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS)
    eng = engine.DepsEngine(window=window, replicas=3, drop_p=0.1, seed=0xACC0D1)
    if fix:
        eng.set_level_mode(True)
    eng.load(b)
    eng.preaccept_deps()
    eng.merge()
    lv, order, _ = eng.exec_levels()
    rlv, _ = ref.levels()
    bad = np.nonzero(lv != rlv)[0]
    eng.close()
    return bad, lv, rlv


rng = np.random.default_rng(9)
n = 6000
K = [abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT]
kinds = rng.choice(K, size=n, p=[0.35, 0.35, 0.1, 0.1, 0.1])
status = rng.choice([abi.ST_APPLIED, abi.ST_STABLE, abi.ST_COMMITTED, abi.ST_PREACCEPTED, abi.ST_ACCEPTED,
                     abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN, abi.ST_HISTORICAL], size=n,
                    p=[0.5, 0.1, 0.1, 0.05, 0.05, 0.1, 0.05, 0.05]).astype(np.uint8)
rw = np.where(kinds > 1, abi.KIND_WRITE, kinds)
for name, kk, st in (("rw+status", rw, status), ("kinds+applied", kinds, None), ("both", kinds, status)):
    for fix in (False, True):
        b = workload.generate(n, keys_per_txn=3, keyspace=200, kinds=kk, status=st, seed=12)
        bad, lv, rlv = run(b, 8, fix)
        print(name, "fixpoint" if fix else "kahn", "bad", len(bad), bad[:8], "kinds", [int(kk[i]) for i in bad[:8]],
              "gpu", lv[bad[:8]].tolist(), "ora", rlv[bad[:8]].tolist())
