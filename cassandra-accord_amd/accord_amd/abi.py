"""ctypes mirror of include/accord_deps.h (structs + constants).

Shared by the product binding (engine.py) and the test-only oracle binding (oracle/oracle.py); it
holds no logic, only the C layout, so both sides of a parity test marshal the same bytes.
"""
import ctypes as C

import numpy as np

AD_OK = 0
AD_ERR_ARGUMENT = -1
AD_ERR_STATE = -2
AD_ERR_UNSORTED = -3
AD_ERR_UNSUPPORTED = -4
AD_ERR_DEVICE = -5
AD_ERR_NOMEM = -6
FAST_REJECTED = 2                 # ad_max_conflicts fast flag: the replica rejects (AD_FAST_REJECTED)
AD_RANK_NONE = 0xFFFFFFFF   # ad_max_conflicts: Timestamp.NONE
AD_LEVEL_DONE = 0xFFFFFFFF  # ad_exec_levels over a CFK history batch: an APPLIED / INVALID row

# Txn.Kind ordinals (primitives/Txn.java:53-113)
KIND_READ, KIND_WRITE, KIND_EPHEMERAL_READ, KIND_SYNC_POINT, KIND_EXCLUSIVE_SYNC_POINT, KIND_LOCAL_ONLY = range(6)
DOMAIN_KEY, DOMAIN_RANGE = 0, 1
# CommandsForKey.InternalStatus ordinals (local/cfk/CommandsForKey.java:493-502)
(ST_TRANSITIVELY_KNOWN, ST_HISTORICAL, ST_PREACCEPTED, ST_ACCEPTED, ST_COMMITTED, ST_STABLE, ST_APPLIED,
 ST_INVALID) = range(8)
CLASS_KEY, CLASS_DIRECT_KEY, CLASS_RANGE = 0, 1, 2
NUM_CLASSES = 3
CLASS_NAMES = ("keyDeps", "directKeyDeps", "rangeDeps")

_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)


class AdBatch(C.Structure):
    _fields_ = [("n", C.c_size_t),
                ("txn_msb", _u64p), ("txn_lsb", _u64p), ("txn_node", _i32p),
                ("exec_msb", _u64p), ("exec_lsb", _u64p), ("exec_node", _i32p),
                ("status", _u8p),
                ("key_off", _u32p), ("keys", _u64p),
                ("range_off", _u32p), ("range_start", _u64p), ("range_end", _u64p)]


class AdCfkState(C.Structure):
    """ad_cfk_state: CFK states (byId TxnInfos per key) for ad_cfk_notify."""
    _fields_ = [("keys", C.c_size_t), ("rows", C.c_size_t), ("row_off", _u32p),
                ("txn_msb", _u64p), ("txn_lsb", _u64p), ("txn_node", _i32p),
                ("exec_msb", _u64p), ("exec_lsb", _u64p), ("exec_node", _i32p),
                ("status", _u8p), ("miss_off", _u32p), ("missing", _u32p)]


class AdCfkEvents(C.Structure):
    """ad_cfk_events: CommandsForKey.update events for the resident store (ad_cfk_store_apply), grouped by key."""
    _fields_ = [("m", C.c_size_t), ("ev_off", _u32p), ("txn_msb", _u64p), ("txn_lsb", _u64p), ("txn_node", _i32p),
                ("status", _u8p), ("exec_msb", _u64p), ("exec_lsb", _u64p), ("exec_node", _i32p),
                ("deps_off", _u32p), ("deps_msb", _u64p), ("deps_lsb", _u64p), ("deps_node", _i32p), ("op", _u8p)]


class AdCfkQueries(C.Structure):
    """ad_cfk_queries: mapReduceActive queries against the resident store (ad_cfk_store_query)."""
    _fields_ = [("nq", C.c_size_t), ("key_off", _u32p), ("keys", _u32p), ("txn_msb", _u64p), ("txn_lsb", _u64p),
                ("txn_node", _i32p), ("bound_msb", _u64p), ("bound_lsb", _u64p), ("bound_node", _i32p)]


CFK_OP_UPDATE, CFK_OP_LOAD, CFK_OP_PRUNE, CFK_OP_LOADING, CFK_OP_UNMANAGED, CFK_OP_UNMANAGED_RECHECK = 0, 1, 2, 3, 4, 5  # AD_CFK_OP_*

CFK_EVENT_FIELDS = (("ev_off", np.uint32), ("txn_msb", np.uint64), ("txn_lsb", np.uint64), ("txn_node", np.int32),
                    ("status", np.uint8), ("exec_msb", np.uint64), ("exec_lsb", np.uint64), ("exec_node", np.int32),
                    ("deps_off", np.uint32), ("deps_msb", np.uint64), ("deps_lsb", np.uint64), ("deps_node", np.int32))


def make_cfk_events(ev):
    """Dict of arrays (CFK_EVENT_FIELDS) -> (AdCfkEvents, keep-alive dict)."""
    keep = {f: np.ascontiguousarray(ev[f], dt) for f, dt in CFK_EVENT_FIELDS}
    s = AdCfkEvents()
    s.m = len(keep["status"])
    for f, dt in CFK_EVENT_FIELDS:
        a = keep[f]
        ct = {np.uint32: _u32p, np.uint64: _u64p, np.int32: _i32p, np.uint8: _u8p}[dt]
        setattr(s, f, a.ctypes.data_as(ct) if a.size else None)
    if ev.get("op") is not None:                     # optional: AD_CFK_OP_* per event (NULL: every event an UPDATE)
        keep["op"] = np.ascontiguousarray(ev["op"], np.uint8)
        s.op = keep["op"].ctypes.data_as(_u8p) if keep["op"].size else None
    return s, keep


CFK_STATE_FIELDS = (("row_off", np.uint32), ("txn_msb", np.uint64), ("txn_lsb", np.uint64), ("txn_node", np.int32),
                    ("exec_msb", np.uint64), ("exec_lsb", np.uint64), ("exec_node", np.int32), ("status", np.uint8),
                    ("miss_off", np.uint32), ("missing", np.uint32))


def make_cfk_state(st):
    """Dict of arrays (CFK_STATE_FIELDS) -> (AdCfkState, keep-alive list)."""
    keep = {}
    for f, dt in CFK_STATE_FIELDS:
        keep[f] = np.ascontiguousarray(st[f], dt)
    s = AdCfkState()
    s.keys = len(keep["row_off"]) - 1
    s.rows = len(keep["status"])
    for f, dt in CFK_STATE_FIELDS:
        a = keep[f]
        ct = {np.uint32: _u32p, np.uint64: _u64p, np.int32: _i32p, np.uint8: _u8p}[dt]
        setattr(s, f, a.ctypes.data_as(ct))
    return s, keep


class AdConfig(C.Structure):
    """ad_config: the store's replica views."""
    _fields_ = [("replicas", C.c_uint32), ("reserved_", C.c_uint32)]


class AdReplicaModel(C.Structure):
    """ad_replica_model: the benchmark's in-flight window / replica drop model (generator setting)."""
    _fields_ = [("window", C.c_uint32), ("drop_p", C.c_float), ("seed", C.c_uint64)]


class ModelConfig(C.Structure):
    """One query model (replicas + window / drop_p / seed): the oracle's oracle_config; the engine splits it
    into ad_config + ad_replica_model."""
    _fields_ = [("window", C.c_uint32), ("replicas", C.c_uint32), ("drop_p", C.c_float),
                ("pad_", C.c_uint32), ("seed", C.c_uint64)]


class AdCsrSizes(C.Structure):
    _fields_ = [("n", C.c_size_t), ("keys", C.c_size_t), ("k2t", C.c_size_t),
                ("txn_cap", C.c_size_t), ("txns", C.c_size_t)]


class AdCsrOut(C.Structure):
    _fields_ = [("key_off", _u32p), ("keys", _u64p), ("k2t_off", _u32p), ("k2t", _i32p),
                ("txn_off", _u32p), ("txns", _u32p)]


class AdCsrIn(C.Structure):
    _fields_ = [("key_off", _u32p), ("keys", _u64p), ("k2t_off", _u32p), ("k2t", _i32p),
                ("txn_off", _u32p), ("txns", _u32p)]


class AdStageTimes(C.Structure):
    _fields_ = [("prepare", C.c_float), ("sort", C.c_float), ("deps", C.c_float), ("merge", C.c_float),
                ("levels", C.c_float), ("total", C.c_float),
                ("deps_entries", C.c_uint64), ("merged_entries", C.c_uint64), ("level_edges", C.c_uint64),
                ("level_iterations", C.c_uint32), ("walk_items", C.c_uint32),
                ("level_blocks", C.c_uint32), ("level_rounds", C.c_uint32),
                ("key_classes", C.c_uint32), ("level_path", C.c_uint32),
                ("deferred_txns", C.c_uint32), ("fill_items", C.c_uint32),
                ("deps_speculative", C.c_uint32),
                ("vitems", C.c_uint64), ("range_entries", C.c_uint64),
                ("gather_items", C.c_uint32), ("chains_fused", C.c_uint32)]


def ptr(a, ctype):
    """Pointer to a contiguous numpy array (None for None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed across the C-ABI must be contiguous"
    return a.ctypes.data_as(C.POINTER(ctype))


BATCH_FIELDS = {
    "txn_msb": np.uint64, "txn_lsb": np.uint64, "txn_node": np.int32,
    "exec_msb": np.uint64, "exec_lsb": np.uint64, "exec_node": np.int32,
    "status": np.uint8, "key_off": np.uint32, "keys": np.uint64,
    "range_off": np.uint32, "range_start": np.uint64, "range_end": np.uint64,
}


def make_batch(b):
    """Build an AdBatch view over a dict of numpy arrays (see workload.generate). The returned
    struct keeps references to the (dtype-normalised) arrays in ``_keep``."""
    arrs = {}
    for name, dt in BATCH_FIELDS.items():
        a = b.get(name)
        if a is None:
            arrs[name] = None
            continue
        arrs[name] = np.ascontiguousarray(a, dtype=dt)
    n = len(arrs["txn_msb"])
    st = AdBatch(n,
                 ptr(arrs["txn_msb"], C.c_uint64), ptr(arrs["txn_lsb"], C.c_uint64), ptr(arrs["txn_node"], C.c_int32),
                 ptr(arrs["exec_msb"], C.c_uint64), ptr(arrs["exec_lsb"], C.c_uint64), ptr(arrs["exec_node"], C.c_int32),
                 ptr(arrs["status"], C.c_uint8), ptr(arrs["key_off"], C.c_uint32), ptr(arrs["keys"], C.c_uint64),
                 ptr(arrs["range_off"], C.c_uint32), ptr(arrs["range_start"], C.c_uint64), ptr(arrs["range_end"], C.c_uint64))
    st._keep = arrs
    return st


def make_config(window=32, replicas=3, drop_p=0.1, seed=0xACC0D1):
    return ModelConfig(window, replicas, drop_p, 0, seed)


class Csr:
    """A batched per-txn CSR (one Deps class of one view), compacted host copy."""

    __slots__ = ("key_off", "keys", "k2t_off", "k2t", "txn_off", "txns", "is_range")

    def __init__(self, key_off, keys, k2t_off, k2t, txn_off, txns, is_range=False):
        self.key_off, self.keys, self.k2t_off, self.k2t = key_off, keys, k2t_off, k2t
        self.txn_off, self.txns, self.is_range = txn_off, txns, is_range

    @staticmethod
    def alloc(sizes, is_range=False):
        n = sizes.n
        return Csr(np.zeros(n + 1, np.uint32), np.zeros(sizes.keys * (2 if is_range else 1), np.uint64),
                   np.zeros(n + 1, np.uint32), np.zeros(sizes.k2t, np.int32),
                   np.zeros(n + 1, np.uint32), np.zeros(sizes.txns, np.uint32), is_range)

    def as_out(self):
        return AdCsrOut(ptr(self.key_off, C.c_uint32), ptr(self.keys, C.c_uint64), ptr(self.k2t_off, C.c_uint32),
                        ptr(self.k2t, C.c_int32), ptr(self.txn_off, C.c_uint32), ptr(self.txns, C.c_uint32))

    def as_in(self):
        return AdCsrIn(ptr(self.key_off, C.c_uint32), ptr(self.keys, C.c_uint64), ptr(self.k2t_off, C.c_uint32),
                       ptr(self.k2t, C.c_int32), ptr(self.txn_off, C.c_uint32), ptr(self.txns, C.c_uint32))

    @property
    def n(self):
        return len(self.key_off) - 1

    def entries(self):
        return int(len(self.k2t) - (self.key_off[-1]))

    def txn(self, i):
        """(keys, txn_ranks, keysToTxnIds) of txn i — the exact SerializerSupport.create arguments
        (KeyDeps.java:69-72 / RangeDeps.java:100-103), with TxnIds as batch ranks."""
        w = 2 if self.is_range else 1
        ks = self.keys[w * self.key_off[i]:w * self.key_off[i + 1]]
        if self.is_range:
            ks = ks.reshape(-1, 2)
        return ks, self.txns[self.txn_off[i]:self.txn_off[i + 1]], self.k2t[self.k2t_off[i]:self.k2t_off[i + 1]]

    def equal(self, other):
        return all(np.array_equal(getattr(self, f), getattr(other, f))
                   for f in ("key_off", "keys", "k2t_off", "k2t", "txn_off", "txns"))

    def first_difference(self, other):
        """Index of the first txn whose CSR differs (or None) — for readable parity failures."""
        for i in range(min(self.n, other.n)):
            a, b = self.txn(i), other.txn(i)
            if not all(np.array_equal(x, y) for x, y in zip(a, b)):
                return i
        return None if self.n == other.n else min(self.n, other.n)
