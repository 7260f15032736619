"""Python binding of libaccord_deps.so (the gfx950 deps engine) over its C-ABI.

This is a thin ctypes layer mirroring the reference operations a host drives on this path:

* ``preaccept_deps()``  — PreAccept.calculatePartialDeps for every txn of the batch, per replica view
  (messages/PreAccept.java:245-267)
* ``merge()``           — Deps.merge of the replica replies (primitives/Deps.java:281-286)
* ``exec_levels()``     — execution order (local/Commands.java:617-821, CommandsForKey.notifyManaged)
* ``max_conflicts()``   — CommandStore.preaccept's witnessedAt proposal per view (local/CommandStore.java:322-347)

There is no CPU fallback: if the HIP library is missing or no GPU is visible the constructor raises.
"""
import ctypes as C
import os

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "libaccord_deps.so")
_LIB = None


class AccordDepsError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__("%s (rc=%d)" % (msg, rc))
        self.rc = rc


class IllegalArgumentException(AccordDepsError):
    pass


class IllegalStateException(AccordDepsError):
    pass


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libaccord_deps.so not built (run `make -C cassandra-accord_amd` / __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.ad_open.argtypes = [C.c_int, C.POINTER(abi.AdConfig), C.POINTER(vp)]
        L.ad_set_replica_model.argtypes = [vp, C.POINTER(abi.AdReplicaModel)]
        L.ad_close.argtypes = [vp]
        L.ad_close.restype = None
        L.ad_last_error.argtypes = [vp]
        L.ad_last_error.restype = C.c_char_p
        L.ad_device_count.restype = C.c_int
        L.ad_load_batch.argtypes = [vp, C.POINTER(abi.AdBatch)]
        L.ad_preaccept_deps.argtypes = [vp, C.POINTER(abi.AdCsrSizes)]
        L.ad_accept_deps.argtypes = [vp, C.POINTER(abi.AdCsrSizes)]
        L.ad_cfk_retain.argtypes = [vp, C.POINTER(C.c_size_t)]
        L.ad_cfk_reset.argtypes = [vp]
        L.ad_cfk_rows.argtypes = [vp, C.POINTER(C.c_size_t), C.POINTER(C.c_uint32)]
        L.ad_cfk_update.argtypes = [vp, C.c_size_t, C.POINTER(C.c_uint32), C.POINTER(C.c_uint8), C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_int32)]
        L.ad_fetch_deps.argtypes = [vp, C.c_uint32, C.c_uint32, C.POINTER(abi.AdCsrOut)]
        L.ad_merge_deps.argtypes = [vp, C.POINTER(abi.AdCsrSizes)]
        L.ad_fetch_merged.argtypes = [vp, C.c_uint32, C.POINTER(abi.AdCsrOut)]
        L.ad_fetch_rows.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_size_t, C.c_size_t, C.POINTER(abi.AdCsrSizes),
                                    C.POINTER(abi.AdCsrOut)]
        L.ad_fetch_inverse.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_size_t, C.c_size_t, C.POINTER(C.c_size_t),
                                       C.POINTER(C.c_uint32), C.POINTER(C.c_int32)]
        L.ad_cfk_notify.argtypes = [vp, C.POINTER(abi.AdCfkState), C.POINTER(C.c_uint8)]
        L.ad_cfk_store_open.argtypes = [vp, C.c_uint32, C.c_uint32]
        L.ad_cfk_store_open_tiered.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
        L.ad_cfk_store_notify_key.argtypes = [vp, C.c_uint32, vp, C.c_size_t, C.POINTER(C.c_size_t)]
        L.ad_cfk_store_apply.argtypes = [vp, C.POINTER(abi.AdCfkEvents)]
        L.ad_cfk_store_notify.argtypes = [vp, vp, vp]
        L.ad_cfk_store_fetch.argtypes = [vp, C.c_uint32, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)] + [vp] * 9
        L.ad_cfk_store_pruning.argtypes = [vp, C.c_uint32, vp, vp, vp, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)] + [vp] * 5
        L.ad_cfk_store_query.argtypes = [vp, C.POINTER(abi.AdCfkQueries), C.POINTER(abi.AdCsrSizes)]
        L.ad_cfk_store_unmanaged.argtypes = [vp, C.c_uint32, C.POINTER(C.c_size_t)] + [vp] * 7
        L.ad_cfk_store_notified.argtypes = [vp, vp, C.POINTER(C.c_size_t)] + [vp] * 5
        L.ad_cfk_store_query_fetch.argtypes = [vp, C.c_uint32, C.POINTER(abi.AdCsrOut), vp, vp, vp]
        L.ad_preaccept_expiry.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_size_t, vp, vp, vp, vp, vp]
        L.ad_merge_host.argtypes = [vp, C.POINTER(abi.AdCsrIn), C.c_uint32, C.POINTER(abi.AdCsrSizes)]
        L.ad_exec_levels.argtypes = [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.ad_run_pipeline.argtypes = [vp]
        L.ad_max_conflicts.argtypes = [vp, vp, vp]
        L.ad_fetch_levels.argtypes = [vp, vp, vp]
        L.ad_last_times.argtypes = [vp, C.POINTER(abi.AdStageTimes)]
        L.ad_set_trace.argtypes = [vp, C.c_uint64]
        L.ad_set_level_mode.argtypes = [vp, C.c_int]
        L.ad_set_pipeline_union.argtypes = [vp, C.c_int]
        L.ad_kernel_count.restype = C.c_int
        L.ad_kernel_name.argtypes = [C.c_int]
        L.ad_kernel_name.restype = C.c_char_p
        L.ad_kernel_stats.argtypes = [vp, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_uint64), C.POINTER(C.c_double)]
        L.ad_reset_kernel_stats.argtypes = [vp]
        L.ad_kernel_units.argtypes = [vp, C.c_int, C.POINTER(C.c_uint64)]
        L.ad_shard_bounds.argtypes = [C.POINTER(C.c_uint64), C.c_size_t, C.c_uint32, C.POINTER(C.c_uint64)]
        L.ad_max_conflicts_carry.argtypes = [vp, C.c_size_t, vp, vp, vp, vp]
        L.ad_merge_deps_fast.argtypes = [vp, C.POINTER(abi.AdCsrSizes)]
        L.ad_max_conflicts_ts.argtypes = [vp, vp, vp, vp, vp]
        L.ad_max_conflicts_export.argtypes = [vp, C.POINTER(C.c_size_t), vp, vp, vp, vp]
        L.ad_max_conflicts_carry_ranges.argtypes = [vp, C.c_size_t, vp, vp, vp, vp, vp]
        L.ad_max_conflicts_export_ranges.argtypes = [vp, C.POINTER(C.c_size_t), vp, vp, vp, vp, vp]
        L.ad_recover.argtypes = [vp, vp, C.c_size_t, C.POINTER(C.c_size_t)]
        L.ad_fetch_recovery.argtypes = [vp, C.c_uint32, C.c_uint32, vp, vp, vp]
        L.ad_fetch_recovery_flags.argtypes = [vp, vp]
        L.ad_load_batch_async.argtypes = [vp, C.POINTER(abi.AdBatch)]
        L.ad_load_batch_commit.argtypes = [vp]
        L.ad_host_alloc.argtypes = [C.c_size_t]
        L.ad_host_alloc.restype = vp
        L.ad_host_free.argtypes = [vp]
        L.ad_host_free.restype = None
        L.ad_merged_sizes.argtypes = [vp, C.POINTER(abi.AdCsrSizes)]
        L.ad_fetch_merged_all.argtypes = [vp, C.POINTER(abi.AdCsrOut)]
        L.ad_fetch_results_async.argtypes = [vp, C.POINTER(abi.AdCsrOut), vp, vp]
        L.ad_fetch_wait.argtypes = [vp]
        _LIB = L
    return _LIB


EXPORTED = ("ad_open", "ad_set_replica_model", "ad_close", "ad_last_error", "ad_device_count", "ad_load_batch", "ad_preaccept_deps", "ad_accept_deps",
            "ad_max_conflicts_carry", "ad_max_conflicts_ts", "ad_max_conflicts_export", "ad_max_conflicts_carry_ranges",
            "ad_max_conflicts_export_ranges", "ad_merge_deps_fast",
            "ad_fetch_deps", "ad_fetch_rows", "ad_fetch_inverse", "ad_preaccept_expiry", "ad_cfk_notify", "ad_cfk_store_open", "ad_cfk_store_open_tiered", "ad_cfk_store_notify_key", "ad_cfk_store_apply", "ad_cfk_store_notify", "ad_cfk_store_fetch", "ad_cfk_store_pruning", "ad_cfk_store_query", "ad_cfk_store_query_fetch", "ad_cfk_store_unmanaged", "ad_cfk_store_notified", "ad_merge_deps", "ad_fetch_merged", "ad_merge_host", "ad_exec_levels", "ad_max_conflicts",
            "ad_run_pipeline", "ad_fetch_levels", "ad_last_times", "ad_set_level_mode", "ad_set_pipeline_union", "ad_set_trace", "ad_kernel_count", "ad_kernel_name", "ad_kernel_stats", "ad_kernel_units",
            "ad_reset_kernel_stats", "ad_shard_bounds", "ad_shard_setup", "ad_shard_export", "ad_shard_send_to_host",
            "ad_shard_import_host", "ad_comm_unique_id", "ad_comm_init", "ad_comm_destroy", "ad_shard_query_positions", "ad_shard_alltoall", "ad_shard_merge",
            "ad_shard_fetch", "ad_shard_levels_round", "ad_shard_levels_get", "ad_shard_levels_set",
            "ad_shard_levels_allreduce", "ad_shard_order", "ad_shard_set_holders", "ad_shard_levels_deltas",
            "ad_shard_levels_apply", "ad_shard_levels_exchange", "ad_cfk_retain", "ad_cfk_reset", "ad_cfk_rows", "ad_cfk_update",
            "ad_recover", "ad_fetch_recovery", "ad_fetch_recovery_flags", "ad_shard_level_edges", "ad_shard_levels_solve",
            "ad_shard_levels_gather", "ad_ephemeral_read_deps", "ad_load_batch_async", "ad_load_batch_commit",
            "ad_host_alloc", "ad_host_free", "ad_merged_sizes", "ad_fetch_merged_all", "ad_fetch_results_async", "ad_fetch_wait", "ad_shard_kahn_begin",
            "ad_shard_kahn_outbox", "ad_shard_kahn_inbox", "ad_shard_kahn_exchange", "ad_shard_kahn_step",
            "ad_shard_kahn_finish", "ad_shard_kahn_sent", "ad_shard_kahn_run", "ad_shard_kahn_depth")


class PinnedArena:
    """Page-locked host arrays (ad_host_alloc): batches and fetched Deps whose H2D / D2H copies are DMA
    transfers.  Arrays are numpy views; they live until close()."""

    def __init__(self):
        self._blocks = []

    def empty(self, count, dtype):
        dt = np.dtype(dtype)
        nbytes = max(int(count) * dt.itemsize, 64)
        p = lib().ad_host_alloc(nbytes)
        if not p:
            raise MemoryError("ad_host_alloc(%d) failed" % nbytes)
        self._blocks.append(p)
        buf = (C.c_uint8 * nbytes).from_address(p)
        return np.frombuffer(buf, dtype=dt, count=int(count))

    def copy(self, a):
        out = self.empty(a.size, a.dtype)
        out[:] = a.reshape(-1)
        return out

    def batch(self, b):
        """A pinned copy of a workload batch dict (numpy arrays copied, scalars kept)."""
        return {k: (self.copy(v) if isinstance(v, np.ndarray) else v) for k, v in b.items()}

    def csr(self, s, is_range=False):
        """An abi.Csr sized by ad_csr_sizes `s`, in pinned memory."""
        n = s.n
        return abi.Csr(self.empty(n + 1, np.uint32), self.empty(s.keys * (2 if is_range else 1), np.uint64),
                       self.empty(n + 1, np.uint32), self.empty(s.k2t, np.int32),
                       self.empty(n + 1, np.uint32), self.empty(s.txns, np.uint32), is_range=is_range)

    def close(self):
        for p in self._blocks:
            lib().ad_host_free(p)
        self._blocks = []


class DepsEngine:
    """One CommandStore shard on one GPU (an ad_handle)."""

    def __init__(self, device=0, window=32, replicas=3, drop_p=0.1, seed=0xACC0D1):
        """replicas -> ad_config; window / drop_p / seed -> ad_set_replica_model (the benchmark's replica model:
        window=0, drop_p=0 is the plain snapshot a live store queries).  self.cfg holds all four for the oracle."""
        self.cfg = abi.make_config(window, replicas, drop_p, seed)
        self.replicas = replicas
        self.device = device
        h = C.c_void_p()
        rc = lib().ad_open(device, C.byref(abi.AdConfig(replicas, 0)), C.byref(h))
        if rc != abi.AD_OK:
            raise AccordDepsError(rc, "ad_open(device=%d) failed" % device)
        self.h = h
        self.n = 0
        self._check(lib().ad_set_replica_model(h, C.byref(abi.AdReplicaModel(window, drop_p, seed))),
                    "ad_set_replica_model")

    def close(self):
        if getattr(self, "h", None):
            lib().ad_close(self.h)
            self.h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc == abi.AD_OK:
            return
        msg = "%s: %s" % (what, lib().ad_last_error(self.h).decode())
        if rc == abi.AD_ERR_ARGUMENT:
            raise IllegalArgumentException(rc, msg)
        if rc == abi.AD_ERR_STATE:
            raise IllegalStateException(rc, msg)
        raise AccordDepsError(rc, msg)

    def load(self, batch):
        self._batch = abi.make_batch(batch)
        self._check(lib().ad_load_batch(self.h, C.byref(self._batch)), "ad_load_batch")
        # rows on the device: the batch, after any CFK history rows kept from the previous batch (ad_cfk_retain)
        hr = C.c_size_t()
        self._check(lib().ad_cfk_rows(self.h, C.byref(hr), None), "ad_cfk_rows")
        self.hist_rows = hr.value
        self.n = self.n_rows = batch["n"] + hr.value

    def load_async(self, batch):
        """Stage the next batch on the copy stream (ad_load_batch_async); the loaded batch keeps running.
        `batch` must stay alive until load_commit()."""
        staged = abi.make_batch(batch)
        self._check(lib().ad_load_batch_async(self.h, C.byref(staged)), "ad_load_batch_async")
        self._staged, self._staged_n = staged, batch["n"]      # a refused call leaves the staged batch as it was

    def load_commit(self):
        self._check(lib().ad_load_batch_commit(self.h), "ad_load_batch_commit")
        self._batch = self._staged
        self._staged = None
        self.hist_rows = 0
        self.n = self.n_rows = self._staged_n

    def merged_sizes(self):
        sizes = (abi.AdCsrSizes * abi.NUM_CLASSES)()
        self._check(lib().ad_merged_sizes(self.h, sizes), "ad_merged_sizes")
        return sizes

    def fetch_merged_all(self, outs=None):
        """The merged Deps of all three classes in one call (ad_fetch_merged_all); `outs` optional
        preallocated abi.Csr per class (e.g. PinnedArena.csr of merged_sizes())."""
        if outs is None:
            s = self.merged_sizes()
            outs = [abi.Csr.alloc(s[c], is_range=(c == abi.CLASS_RANGE)) for c in range(abi.NUM_CLASSES)]
        arr = (abi.AdCsrOut * abi.NUM_CLASSES)(*[o.as_out() for o in outs])
        self._check(lib().ad_fetch_merged_all(self.h, arr), "ad_fetch_merged_all")
        return outs

    def fetch_results_async(self, outs, levels=None):
        """Page out the merged Deps (outs: pinned abi.Csr per class, sized by merged_sizes()) and, with levels = a pinned
        (levels, order) pair, the levels and order, while the device goes on (ad_fetch_results_async); the buffers
        hold the results once fetch_wait() returns and must not be touched before."""
        self._async_outs = (outs, levels, (abi.AdCsrOut * abi.NUM_CLASSES)(*[o.as_out() for o in outs]))
        lv = levels[0].ctypes.data if levels is not None else None
        od = levels[1].ctypes.data if levels is not None else None
        self._check(lib().ad_fetch_results_async(self.h, self._async_outs[2], lv, od), "ad_fetch_results_async")

    def fetch_wait(self):
        self._check(lib().ad_fetch_wait(self.h), "ad_fetch_wait")
        self._async_outs = None

    def preaccept_deps(self):
        sizes = (abi.AdCsrSizes * (self.replicas * abi.NUM_CLASSES))()
        self._check(lib().ad_preaccept_deps(self.h, sizes), "ad_preaccept_deps")
        self._dep_sizes = sizes
        return sizes

    def ephemeral_read_deps(self):
        """Deps with bound = Timestamp.MAX (GetEphemeralReadDeps.java:76): fetch with fetch_deps."""
        sizes = (abi.AdCsrSizes * (self.replicas * abi.NUM_CLASSES))()
        self._check(lib().ad_ephemeral_read_deps(self.h, sizes), "ad_ephemeral_read_deps")
        self._dep_sizes = sizes
        return sizes

    def accept_deps(self):
        """Deps with bound = executeAt (Accept.calculatePartialDeps / GetDeps): fetch with fetch_deps."""
        sizes = (abi.AdCsrSizes * (self.replicas * abi.NUM_CLASSES))()
        self._check(lib().ad_accept_deps(self.h, sizes), "ad_accept_deps")
        self._dep_sizes = sizes
        return sizes

    def cfk_retain(self):
        """Keep this batch's still-visible CFK rows on the device for the next load (returns the kept row count)."""
        k = C.c_size_t()
        self._check(lib().ad_cfk_retain(self.h, C.byref(k)), "ad_cfk_retain")
        return k.value

    def cfk_reset(self):
        self._check(lib().ad_cfk_reset(self.h), "ad_cfk_reset")

    def recover(self, rows):
        """BeginRecovery's store queries for the recovering rows (ad_recover, after a merge on this batch) ->
        (out, reject): out[which][cls] = (off [nq+1], keys [E] or [E, 2], txns [E]) — which 0 =
        earlierCommittedWitness, 1 = earlierAcceptedNoWitness, each Deps as its entries in Deps order (the
        Deps.Builder stream; wire.relations_to_csr / KeyDeps.Builder build the SerializerSupport arrays);
        reject [nq] uint8 = rejectsFastPath."""
        rows = np.ascontiguousarray(rows, np.uint32)
        nq = len(rows)
        ent = (C.c_size_t * 6)()
        self._check(lib().ad_recover(self.h, rows.ctypes.data, nq, ent), "ad_recover")
        out = []
        for w in range(2):
            cl = []
            for c in range(abi.NUM_CLASSES):
                e = ent[w * 3 + c]
                kw = 2 if c == abi.CLASS_RANGE else 1
                off = np.zeros(nq + 1, np.uint32)
                keys = np.zeros(max(e * kw, 1), np.uint64)
                txns = np.zeros(max(e, 1), np.uint32)
                self._check(lib().ad_fetch_recovery(self.h, w, c, off.ctypes.data, keys.ctypes.data, txns.ctypes.data),
                            "ad_fetch_recovery")
                keys = keys[:e * kw].reshape(-1, 2) if kw == 2 else keys[:e]
                cl.append((off, keys, txns[:e]))
            out.append(cl)
        rej = np.zeros(max(nq, 1), np.uint8)
        self._check(lib().ad_fetch_recovery_flags(self.h, rej.ctypes.data), "ad_fetch_recovery_flags")
        return out, rej[:nq]

    def cfk_notify(self, state):
        """CommandsForKey.notifyManaged's release rule (ad_cfk_notify) over CFK states: `state` is a dict of the
        abi.CFK_STATE_FIELDS arrays (per key its byId TxnInfos: TxnId, InternalStatus, executeAt, missing as row
        indices).  Returns not_waiting [rows] uint8."""
        s, keep = abi.make_cfk_state(state)
        out = np.zeros(max(s.rows, 1), np.uint8)
        self._check(lib().ad_cfk_notify(self.h, C.byref(s), out.ctypes.data_as(C.POINTER(C.c_uint8))), "ad_cfk_notify")
        return out[:s.rows]

    # ---- device-resident CommandsForKey states (ad_cfk_store_*) -------------------------------------------------
    def cfk_store_open(self, keys, capacity, big_capacity=0, big_keys=0):
        """K resident CFKs of up to `capacity` rows each (rounded up to a multiple of 64, at most 8192); with big_keys,
        a key outgrowing them moves to one of big_keys large-tier slots of big_capacity rows (<= 16384) in the call."""
        if big_keys:
            self._check(lib().ad_cfk_store_open_tiered(self.h, keys, capacity, big_capacity, big_keys),
                        "ad_cfk_store_open_tiered")
        else:
            self._check(lib().ad_cfk_store_open(self.h, keys, capacity), "ad_cfk_store_open")
        self._cs_keys, self._cs_cap = keys, capacity          # not_waiting rows at the caller's capacity

    def cfk_store_notify_key(self, key):
        """After cfk_store_notify: one key's not_waiting flags over all of its rows (a large-tier key's beyond the
        bulk output's capacity too)."""
        n = C.c_size_t()
        self._check(lib().ad_cfk_store_notify_key(self.h, key, None, 0, C.byref(n)), "ad_cfk_store_notify_key")
        out = np.zeros(max(n.value, 1), np.uint8)
        self._check(lib().ad_cfk_store_notify_key(self.h, key, out.ctypes.data, out.size, C.byref(n)),
                    "ad_cfk_store_notify_key")
        return out[:n.value]

    def cfk_store_apply(self, events):
        """CommandsForKey.update events (a dict of abi.CFK_EVENT_FIELDS arrays, grouped by key through ev_off)."""
        s, keep = abi.make_cfk_events(events)
        self._check(lib().ad_cfk_store_apply(self.h, C.byref(s)), "ad_cfk_store_apply")

    def cfk_store_notify(self):
        """notifyManaged's release rule over the resident rows: (rows [K], not_waiting [K, capacity] uint8)."""
        rows = np.zeros(self._cs_keys, np.uint32)
        out = np.zeros((self._cs_keys, self._cs_cap), np.uint8)
        self._check(lib().ad_cfk_store_notify(self.h, rows.ctypes.data, out.ctypes.data), "ad_cfk_store_notify")
        return rows, out

    def cfk_store_fetch(self, key):
        """One key's resident rows: dict of txn_msb/lsb/node, exec_msb/lsb/node, status, miss_off, missing (byId row
        indices)."""
        n, tot = C.c_size_t(), C.c_size_t()
        nulls = [None] * 9
        self._check(lib().ad_cfk_store_fetch(self.h, key, C.byref(n), C.byref(tot), *nulls), "ad_cfk_store_fetch")
        r = n.value
        out = {"txn_msb": np.zeros(max(r, 1), np.uint64), "txn_lsb": np.zeros(max(r, 1), np.uint64),
               "txn_node": np.zeros(max(r, 1), np.int32), "exec_msb": np.zeros(max(r, 1), np.uint64),
               "exec_lsb": np.zeros(max(r, 1), np.uint64), "exec_node": np.zeros(max(r, 1), np.int32),
               "status": np.zeros(max(r, 1), np.uint8), "miss_off": np.zeros(r + 1, np.uint32),
               "missing": np.zeros(max(tot.value, 1), np.uint32)}
        order = ("txn_msb", "txn_lsb", "txn_node", "exec_msb", "exec_lsb", "exec_node", "status", "miss_off", "missing")
        self._check(lib().ad_cfk_store_fetch(self.h, key, C.byref(n), C.byref(tot), *(out[f].ctypes.data for f in order)),
                    "ad_cfk_store_fetch")
        for f in order:
            if f != "miss_off":
                out[f] = out[f][:r if f != "missing" else tot.value]
        return out

    def cfk_store_pruning(self, key):
        """One key's prunedBefore (msb, lsb, node) and loadingPruned table: dict of pruned_before, lp_msb/lsb/node,
        lp_off, lp_rows (the witnesses that are rows, byId row indices)."""
        n, tot = C.c_size_t(), C.c_size_t()
        self._check(lib().ad_cfk_store_pruning(self.h, key, None, None, None, C.byref(n), C.byref(tot), *([None] * 5)),
                    "ad_cfk_store_pruning")
        L = n.value
        pm, pl, pn = C.c_uint64(), C.c_uint64(), C.c_int32()
        out = {"lp_msb": np.zeros(max(L, 1), np.uint64), "lp_lsb": np.zeros(max(L, 1), np.uint64),
               "lp_node": np.zeros(max(L, 1), np.int32), "lp_off": np.zeros(L + 1, np.uint32),
               "lp_rows": np.zeros(max(tot.value, 1), np.uint32)}
        self._check(lib().ad_cfk_store_pruning(self.h, key, C.byref(pm), C.byref(pl), C.byref(pn), C.byref(n), C.byref(tot),
                                               *(out[f].ctypes.data for f in ("lp_msb", "lp_lsb", "lp_node", "lp_off",
                                                                             "lp_rows"))), "ad_cfk_store_pruning")
        for f in ("lp_msb", "lp_lsb", "lp_node"):
            out[f] = out[f][:L]
        out["lp_rows"] = out["lp_rows"][:tot.value]
        out["pruned_before"] = (pm.value, pl.value, pn.value)
        return out

    def cfk_store_unmanaged(self, key):
        """One key's unmanaged registry (Unmanaged.compareTo order): list of (pending, waitingUntil (msb, lsb, node),
        TxnId (msb, lsb, node))."""
        n = C.c_size_t()
        self._check(lib().ad_cfk_store_unmanaged(self.h, key, C.byref(n), *([None] * 7)), "ad_cfk_store_unmanaged")
        m = n.value
        arr = [np.zeros(max(m, 1), dt) for dt in (np.uint8, np.uint64, np.uint64, np.int32, np.uint64, np.uint64, np.int32)]
        self._check(lib().ad_cfk_store_unmanaged(self.h, key, C.byref(n), *(x.ctypes.data for x in arr)), "ad_cfk_store_unmanaged")
        return [(int(arr[0][i]), (int(arr[1][i]), int(arr[2][i]), int(arr[3][i])), (int(arr[4][i]), int(arr[5][i]), int(arr[6][i])))
                for i in range(m)]

    def cfk_store_notified(self):
        """The last cfk_store_apply's unmanaged notifications: per key a list of (event index within the key's events
        of the call, tag, TxnId (msb, lsb, node)); tag 0 commit, 1 applied, 2 ready at (re)registration."""
        cnt = np.zeros(self._cs_keys, np.uint32)
        tot = C.c_size_t()
        self._check(lib().ad_cfk_store_notified(self.h, cnt.ctypes.data, C.byref(tot), *([None] * 5)), "ad_cfk_store_notified")
        m = tot.value
        arr = [np.zeros(max(m, 1), dt) for dt in (np.uint32, np.uint8, np.uint64, np.uint64, np.int32)]
        self._check(lib().ad_cfk_store_notified(self.h, cnt.ctypes.data, C.byref(tot), *(x.ctypes.data for x in arr)),
                    "ad_cfk_store_notified")
        out, o = [], 0
        for k in range(self._cs_keys):
            out.append([(int(arr[0][i]), int(arr[1][i]), (int(arr[2][i]), int(arr[3][i]), int(arr[4][i])))
                        for i in range(o, o + int(cnt[k]))])
            o += int(cnt[k])
        return out

    def cfk_store_query(self, key_off, keys, txn, bound):
        """CommandsForKey.mapReduceActive over the resident rows for queries (ad_cfk_store_query): key_off [nq + 1] /
        keys (store key indices, ascending per query); txn and bound: (msb, lsb, node) arrays [nq] (the querying TxnId and
        startedBefore).  Returns [keyDeps, directKeyDeps], each a dict of key_off, keys, k2t_off, k2t, txn_off and the
        TxnIds as txn_msb / txn_lsb / txn_node."""
        ko = np.ascontiguousarray(key_off, np.uint32)
        ks = np.ascontiguousarray(keys, np.uint32)
        arr = [np.ascontiguousarray(x, dt) for x, dt in zip((*txn, *bound), (np.uint64, np.uint64, np.int32) * 2)]
        q = abi.AdCfkQueries()
        q.nq = len(ko) - 1
        q.key_off = ko.ctypes.data_as(abi._u32p); q.keys = ks.ctypes.data_as(abi._u32p)
        for f, x in zip(("txn_msb", "txn_lsb", "txn_node", "bound_msb", "bound_lsb", "bound_node"), arr):
            setattr(q, f, x.ctypes.data_as(abi._i32p if x.dtype == np.int32 else abi._u64p))
        sizes = (abi.AdCsrSizes * 2)()
        self._check(lib().ad_cfk_store_query(self.h, C.byref(q), sizes), "ad_cfk_store_query")
        out = []
        for cls in range(2):
            sz = sizes[cls]
            d = {"key_off": np.zeros(q.nq + 1, np.uint32), "keys": np.zeros(max(sz.keys, 1), np.uint64),
                 "k2t_off": np.zeros(q.nq + 1, np.uint32), "k2t": np.zeros(max(sz.k2t, 1), np.int32),
                 "txn_off": np.zeros(q.nq + 1, np.uint32), "txn_msb": np.zeros(max(sz.txns, 1), np.uint64),
                 "txn_lsb": np.zeros(max(sz.txns, 1), np.uint64), "txn_node": np.zeros(max(sz.txns, 1), np.int32)}
            o = abi.AdCsrOut()
            o.key_off = d["key_off"].ctypes.data_as(abi._u32p); o.keys = d["keys"].ctypes.data_as(abi._u64p)
            o.k2t_off = d["k2t_off"].ctypes.data_as(abi._u32p); o.k2t = d["k2t"].ctypes.data_as(abi._i32p)
            o.txn_off = d["txn_off"].ctypes.data_as(abi._u32p); o.txns = None
            self._check(lib().ad_cfk_store_query_fetch(self.h, cls, C.byref(o), d["txn_msb"].ctypes.data,
                                                       d["txn_lsb"].ctypes.data, d["txn_node"].ctypes.data),
                        "ad_cfk_store_query_fetch")
            for f, nf in (("keys", sz.keys), ("k2t", sz.k2t), ("txn_msb", sz.txns), ("txn_lsb", sz.txns), ("txn_node", sz.txns)):
                d[f] = d[f][:nf]
            out.append(d)
        return out

    def cfk_update(self, gid, status, exec_msb=None, exec_lsb=None, exec_node=None):
        """Status transitions of kept rows between batches (after cfk_retain, before the next load): gid[m]
        ascending global ranks, status[m] InternalStatus, optional executeAt arrays (CommandsForKeyTest's
        transition table; a refused update applies none)."""
        g = np.ascontiguousarray(gid, np.uint32)
        s = np.ascontiguousarray(status, np.uint8)
        u64p, i32p = C.POINTER(C.c_uint64), C.POINTER(C.c_int32)
        ex = None
        if exec_msb is not None:
            ex = (np.ascontiguousarray(exec_msb, np.uint64), np.ascontiguousarray(exec_lsb, np.uint64),
                  np.ascontiguousarray(exec_node, np.int32))
        self._check(lib().ad_cfk_update(self.h, len(g), g.ctypes.data_as(C.POINTER(C.c_uint32)),
                                        s.ctypes.data_as(C.POINTER(C.c_uint8)),
                                        ex[0].ctypes.data_as(u64p) if ex else None, ex[1].ctypes.data_as(u64p) if ex else None,
                                        ex[2].ctypes.data_as(i32p) if ex else None), "ad_cfk_update")

    def cfk_rows(self):
        """(history rows H, gid[n]: global arrival rank of every row of the loaded batch)."""
        hr = C.c_size_t()
        g = np.zeros(max(self.n_rows, 1), np.uint32)
        self._check(lib().ad_cfk_rows(self.h, C.byref(hr), g.ctypes.data_as(C.POINTER(C.c_uint32))), "ad_cfk_rows")
        return hr.value, g[:self.n_rows]

    def fetch_deps(self, view, cls):
        s = self._dep_sizes[view * abi.NUM_CLASSES + cls]
        out = abi.Csr.alloc(s, is_range=(cls == abi.CLASS_RANGE))
        o = out.as_out()
        self._check(lib().ad_fetch_deps(self.h, view, cls, C.byref(o)), "ad_fetch_deps")
        return out

    def fetch_rows(self, view, cls, lo, hi):
        """Rows [lo, hi) of replica view `view` (view == replicas: the merged Deps) for class `cls`, as an
        abi.Csr over hi - lo txns (paged fetch: full-size batches hold ~10^9 entries per view)."""
        s = abi.AdCsrSizes()
        self._check(lib().ad_fetch_rows(self.h, view, cls, lo, hi, C.byref(s), None), "ad_fetch_rows")
        out = abi.Csr.alloc(s, is_range=(cls == abi.CLASS_RANGE))
        o = out.as_out()
        self._check(lib().ad_fetch_rows(self.h, view, cls, lo, hi, C.byref(s), C.byref(o)), "ad_fetch_rows")
        return out

    def fetch_inverse(self, view, cls, lo=0, hi=None):
        """KeyDeps.txnIdsToKeys / RangeDeps.txnIdsToRanges (RelationMultiMap.invert) of rows [lo, hi) of view
        `view`'s class `cls` (view == replicas: the merged Deps), computed on the device: (off [m + 1], inv) with
        row i's inverse at inv[off[i]:off[i + 1]] = nTxnIds end offsets (based at nTxnIds), then per TxnId index
        its ascending key (range) indices."""
        hi = self.n if hi is None else hi
        tot = C.c_size_t()
        off = np.zeros(hi - lo + 1, np.uint32)
        self._check(lib().ad_fetch_inverse(self.h, view, cls, lo, hi, C.byref(tot),
                                           off.ctypes.data_as(C.POINTER(C.c_uint32)), None), "ad_fetch_inverse")
        inv = np.zeros(max(tot.value, 1), np.int32)
        self._check(lib().ad_fetch_inverse(self.h, view, cls, lo, hi, C.byref(tot), None,
                                           inv.ctypes.data_as(C.POINTER(C.c_int32))), "ad_fetch_inverse")
        return off, inv[:tot.value]

    def merge(self):
        sizes = (abi.AdCsrSizes * abi.NUM_CLASSES)()
        self._check(lib().ad_merge_deps(self.h, sizes), "ad_merge_deps")
        self._merge_sizes = sizes
        return sizes

    def merge_fast(self):
        """The coordinator's fast-path Deps.merge: per txn only the views whose proposal is witnessedAt == TxnId
        (the fast flags of the last max_conflicts / max_conflicts_ts).  Fetch with fetch_merged()."""
        sizes = (abi.AdCsrSizes * abi.NUM_CLASSES)()
        self._check(lib().ad_merge_deps_fast(self.h, sizes), "ad_merge_deps_fast")
        self._merge_sizes = sizes
        return sizes

    def merge_host(self, replies):
        """Deps.merge of caller-supplied replies over the loaded batch: replies[r][cls] is an abi.Csr (the
        same per-txn canonical layout ad_fetch_deps returns).  Fetch the result with fetch_merged()."""
        r = len(replies)
        arr = (abi.AdCsrIn * (r * abi.NUM_CLASSES))()
        keep = []
        for v, rep in enumerate(replies):
            for c in range(abi.NUM_CLASSES):
                csr = rep[c]
                keep.append(csr)
                arr[v * abi.NUM_CLASSES + c] = csr.as_in()
        sizes = (abi.AdCsrSizes * abi.NUM_CLASSES)()
        self._check(lib().ad_merge_host(self.h, arr, r, sizes), "ad_merge_host")
        self._merge_sizes = sizes
        return sizes

    def fetch_merged(self, cls):
        s = self._merge_sizes[cls]
        out = abi.Csr.alloc(s, is_range=(cls == abi.CLASS_RANGE))
        o = out.as_out()
        self._check(lib().ad_fetch_merged(self.h, cls, C.byref(o)), "ad_fetch_merged")
        return out

    def exec_levels(self, want_order=True):
        lv = np.zeros(max(self.n, 1), np.uint32)
        order = np.zeros(max(self.n, 1), np.uint32) if want_order else None
        it = C.c_uint32()
        self._check(lib().ad_exec_levels(self.h, lv.ctypes.data_as(C.POINTER(C.c_uint32)),
                                         order.ctypes.data_as(C.POINTER(C.c_uint32)) if want_order else None,
                                         C.byref(it)), "ad_exec_levels")
        return lv[:self.n], (order[:self.n] if want_order else None), it.value

    def max_conflicts(self):
        """CommandStore.preaccept per replica view (local/CommandStore.java:322-347), after preaccept_deps():
        (max_rank [R, n] uint32 — rank of the txn whose executeAt is maxConflicts.get(keys), AD_RANK_NONE for
        Timestamp.NONE; fast [R, n] uint8 — 1 when the replica answers witnessedAt = TxnId).  A slow-path
        replica answers time.uniqueNow(that executeAt), which the host clock supplies."""
        R, n = self.replicas, self.n
        rank = np.zeros((R, max(n, 1)), np.uint32)
        fast = np.zeros((R, max(n, 1)), np.uint8)
        self._check(lib().ad_max_conflicts(self.h, rank.ctypes.data, fast.ctypes.data), "ad_max_conflicts")
        return rank[:, :n], fast[:, :n]

    def max_conflicts_carry(self, table):
        """The store's MaxConflicts map from earlier batches: (keys u64 ascending, msb, lsb, node) arrays."""
        k, m, l, nd = (np.ascontiguousarray(table[0], np.uint64), np.ascontiguousarray(table[1], np.uint64),
                       np.ascontiguousarray(table[2], np.uint64), np.ascontiguousarray(table[3], np.int32))
        self._carry = (k, m, l, nd)
        self._check(lib().ad_max_conflicts_carry(self.h, len(k), k.ctypes.data, m.ctypes.data, l.ctypes.data,
                                                 nd.ctypes.data), "ad_max_conflicts_carry")

    NO_TIMEOUT = 0xFFFFFFFFFFFFFFFF

    def preaccept_expiry(self, now=0, timeout=NO_TIMEOUT, reject_before=None):
        """CommandStore.preaccept's expiry state for the following max_conflicts(_ts) calls (ad_preaccept_expiry): the
        clock's now (hlc), preAcceptTimeout (NO_TIMEOUT: none) and rejectBefore (witness.RejectBefore.table() arrays,
        or None).  Fast flags then read 1 fast path, 0 slow path, abi.FAST_REJECTED rejected (uniqueNow(TxnId)
        .asRejected()); ExclusiveSyncPoints answer their TxnId."""
        t = reject_before if reject_before is not None else (np.zeros(0, np.uint64),) * 4 + (np.zeros(0, np.int32),)
        s, e, m, l, nd = (np.ascontiguousarray(a, dt) for a, dt in zip(t, (np.uint64,) * 4 + (np.int32,)))
        self._check(lib().ad_preaccept_expiry(self.h, now, timeout, len(s), s.ctypes.data, e.ctypes.data, m.ctypes.data,
                                              l.ctypes.data, nd.ctypes.data), "ad_preaccept_expiry")

    def max_conflicts_ts(self):
        """maxConflicts.get(keys) per view and txn over the carry and the batch as raw timestamps:
        (msb [R, n], lsb [R, n], node [R, n], fast [R, n]); Timestamp.NONE = (0, 0, 0)."""
        R, n = self.replicas, self.n
        msb = np.zeros((R, max(n, 1)), np.uint64)
        lsb = np.zeros((R, max(n, 1)), np.uint64)
        node = np.zeros((R, max(n, 1)), np.int32)
        fast = np.zeros((R, max(n, 1)), np.uint8)
        self._check(lib().ad_max_conflicts_ts(self.h, msb.ctypes.data, lsb.ctypes.data, node.ctypes.data, fast.ctypes.data),
                    "ad_max_conflicts_ts")
        return msb[:, :n], lsb[:, :n], node[:, :n], fast[:, :n]

    def max_conflicts_export(self):
        """The MaxConflicts table after this batch: (keys, msb, lsb, node)."""
        m = C.c_size_t()
        self._check(lib().ad_max_conflicts_export(self.h, C.byref(m), None, None, None, None), "ad_max_conflicts_export")
        k = np.zeros(max(m.value, 1), np.uint64)
        ms = np.zeros(max(m.value, 1), np.uint64)
        ls = np.zeros(max(m.value, 1), np.uint64)
        nd = np.zeros(max(m.value, 1), np.int32)
        self._check(lib().ad_max_conflicts_export(self.h, C.byref(m), k.ctypes.data, ms.ctypes.data, ls.ctypes.data,
                                                  nd.ctypes.data), "ad_max_conflicts_export")
        c = m.value
        return k[:c], ms[:c], ls[:c], nd[:c]

    def max_conflicts_carry_ranges(self, table):
        """The range part of the store's MaxConflicts map: (starts, ends, msb, lsb, node), sorted disjoint (s, e]."""
        a = tuple(np.ascontiguousarray(x, dt) for x, dt in zip(table, (np.uint64,) * 4 + (np.int32,)))
        self._carry_ranges = a
        self._check(lib().ad_max_conflicts_carry_ranges(self.h, len(a[0]), *(x.ctypes.data for x in a)),
                    "ad_max_conflicts_carry_ranges")

    def max_conflicts_export_ranges(self):
        """The intervals of the MaxConflicts map after this batch: (starts, ends, msb, lsb, node)."""
        m = C.c_size_t()
        self._check(lib().ad_max_conflicts_export_ranges(self.h, C.byref(m), None, None, None, None, None),
                    "ad_max_conflicts_export_ranges")
        k = max(m.value, 1)
        out = tuple(np.zeros(k, np.uint64) for _ in range(4)) + (np.zeros(k, np.int32),)
        self._check(lib().ad_max_conflicts_export_ranges(self.h, C.byref(m), *(x.ctypes.data for x in out)),
                    "ad_max_conflicts_export_ranges")
        return tuple(x[:m.value] for x in out)

    def run_pipeline(self):
        self._check(lib().ad_run_pipeline(self.h), "ad_run_pipeline")

    def fetch_levels(self, out=None):
        """(levels, order) left on the device by the last run_pipeline / exec_levels; `out` an optional
        preallocated (levels, order) pair of uint32 arrays with at least n entries (e.g. pinned)."""
        lv, order = out if out is not None else (np.zeros(max(self.n, 1), np.uint32), np.zeros(max(self.n, 1), np.uint32))
        if len(lv) < self.n or len(order) < self.n or lv.dtype != np.uint32 or order.dtype != np.uint32:
            raise ValueError("fetch_levels: out arrays too small or not uint32")
        self._check(lib().ad_fetch_levels(self.h, lv.ctypes.data, order.ctypes.data), "ad_fetch_levels")
        return lv[:self.n], order[:self.n]

    def last_times(self):
        t = abi.AdStageTimes()
        self._check(lib().ad_last_times(self.h, C.byref(t)), "ad_last_times")
        return {f: getattr(t, f) for f, _ in abi.AdStageTimes._fields_}

    LEVELS_AUTO, LEVELS_FIXPOINT, LEVELS_BLOCKS, LEVELS_KAHN, LEVELS_PULL_ABORT, LEVELS_BLOCKS_WIDE = 0, 1, 2, 3, 4, 5

    def set_level_mode(self, mode):
        """LEVELS_AUTO (default; False): one-pass pull levels for short key chains, executeAt blocks for deep
        key-only batches, Kahn with explicit edges for mixed batches; LEVELS_FIXPOINT (True): always the chain
        fixpoint; LEVELS_BLOCKS: executeAt blocks for every key-only batch; LEVELS_KAHN: the Kahn wavefront
        instead of the pull levels; LEVELS_PULL_ABORT (tests): the pull levels abort at once and the Kahn
        wavefronts recompute the batch (the abort path of AUTO); LEVELS_BLOCKS_WIDE (tests): LEVELS_BLOCKS with the
        64-bit scan words the block walk uses for batches of more than 2^20 txns."""
        mode = int(mode) if not isinstance(mode, bool) else (1 if mode else 0)
        self._check(lib().ad_set_level_mode(self.h, mode), "ad_set_level_mode")

    def set_pipeline_union(self, on):
        """True: run_pipeline builds the merged Deps as the deps stage's union view (a generator-only shortcut, a
        side figure); False (default): k_merge_ref merges the R replies' CSRs (Deps.merge)."""
        self._check(lib().ad_set_pipeline_union(self.h, 1 if on else 0), "ad_set_pipeline_union")

    def set_trace(self, mask):
        """Enable HIP-event timing of the kernels whose id bit is set (see kernel_ids())."""
        self._check(lib().ad_set_trace(self.h, mask), "ad_set_trace")

    def reset_kernel_stats(self):
        self._check(lib().ad_reset_kernel_stats(self.h), "ad_reset_kernel_stats")

    def kernel_stats(self):
        """{kernel name: (launches, total ms, elements processed)} for every traced kernel with a launch."""
        out = {}
        for k in range(lib().ad_kernel_count()):
            name, calls, ms, units = C.c_char_p(), C.c_uint64(), C.c_double(), C.c_uint64()
            self._check(lib().ad_kernel_stats(self.h, k, C.byref(name), C.byref(calls), C.byref(ms)), "ad_kernel_stats")
            self._check(lib().ad_kernel_units(self.h, k, C.byref(units)), "ad_kernel_units")
            if calls.value:
                out[name.value.decode()] = (calls.value, ms.value, units.value)
        return out


def kernel_ids():
    """{kernel name: id} of the traceable kernels."""
    out = {}
    for k in range(lib().ad_kernel_count()):
        out[lib().ad_kernel_name(k).decode()] = k
    return out


def device_count():
    return lib().ad_device_count()
