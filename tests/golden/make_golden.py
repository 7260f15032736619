#!/usr/bin/env python3
"""Generates tests/golden/*.npz: seeded input batches + the oracle's outputs for them.

The reference is Java (no JVM in this image), so these vectors come from the oracle (the
CPU restatement in oracle/), itself pinned to the reference's own tests (tests/test_oracle_*.py).  They
freeze the expected bytes so a GPU run can be checked without re-running the oracle, and so any later
change to the oracle shows up as a fixture diff.

Run: python tests/golden/make_golden.py   (rewrites the fixtures)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from accord_amd import abi, workload  # noqa: E402

CSR_FIELDS = ("key_off", "keys", "k2t_off", "k2t", "txn_off", "txns")


def mixed_kinds(n, seed):
    rng = np.random.default_rng(seed)
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT,
                        abi.KIND_EXCLUSIVE_SYNC_POINT], size=n, p=[0.35, 0.35, 0.1, 0.1, 0.1])
    status = rng.choice([abi.ST_APPLIED, abi.ST_STABLE, abi.ST_COMMITTED, abi.ST_PREACCEPTED, abi.ST_ACCEPTED,
                         abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN, abi.ST_HISTORICAL], size=n,
                        p=[0.5, 0.1, 0.1, 0.05, 0.05, 0.1, 0.05, 0.05]).astype(np.uint8)
    return workload.generate(n, keys_per_txn=3, keyspace=300, kinds=kinds, status=status, seed=seed)


# name -> (batch, config(window, replicas, drop_p, seed), compute levels)
CASES = {
    "c2_small": (lambda: workload.config("C2", n=3000), (32, 3, 0.1, 0xACC0D1), True),
    "c3_small": (lambda: workload.config("C3", n=3000), (32, 3, 0.1, 0xACC0D2), True),
    "c4_small": (lambda: workload.generate(2000, 4, 20000, "uniform", range_frac=0.1, range_width_max=400,
                                           seed=0xACC0D3), (32, 3, 0.1, 0xACC0D3), True),
    "hot_keys": (lambda: workload.generate(2000, keys_per_txn=2, keyspace=5, slow_frac=0.5, bump_max=300, seed=11),
                 (4, 2, 0.3, 11), True),
    "mixed_kinds": (lambda: mixed_kinds(1500, 12), (8, 3, 0.2, 12), False),
}


def save(name):
    mk, (w, r, p, s), levels = CASES[name]
    b = mk()
    cfg = abi.make_config(w, r, p, s)
    res = O.OracleResult(b, cfg, O.FLAG_MERGE | (O.FLAG_LEVELS if levels else 0))
    out = {"cfg": np.array([w, r, s], np.uint64), "drop_p": np.array([p], np.float32)}
    for f in abi.BATCH_FIELDS:
        if b.get(f) is not None:
            out["in_" + f] = np.asarray(b[f], abi.BATCH_FIELDS[f])
    for v in range(r):
        for c in range(abi.NUM_CLASSES):
            csr = res.deps(v, c)
            for f in CSR_FIELDS:
                out["deps_%d_%d_%s" % (v, c, f)] = getattr(csr, f)
    for c in range(abi.NUM_CLASSES):
        csr = res.merged(c)
        for f in CSR_FIELDS:
            out["merged_%d_%s" % (c, f)] = getattr(csr, f)
    if levels:
        lv, order = res.levels()
        out["level"], out["order"] = lv, order
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)


def load(name):
    """-> (batch dict, (window, replicas, drop_p, seed), {key: array})."""
    z = dict(np.load(os.path.join(HERE, name + ".npz")))
    b = {"n": int(len(z["in_txn_msb"]))}
    for f in abi.BATCH_FIELDS:
        b[f] = z.get("in_" + f)
    w, r, s = (int(x) for x in z["cfg"])
    return b, (w, r, float(z["drop_p"][0]), s), z


def csr_from(z, prefix, is_range):
    return abi.Csr(*(z[prefix + f] for f in CSR_FIELDS), is_range=is_range)


if __name__ == "__main__":
    for name in CASES:
        save(name)
        print("wrote", name, os.path.getsize(os.path.join(HERE, name + ".npz")), "bytes")
