/*
 * accord_deps.h — C-ABI of the MI355X batched dependency-resolution engine.
 *
 * This is the drop-in boundary for Accord's PreAccept-deps -> Deps.merge -> execution-order
 * hot path.  Every entry point is plain C (pointers + sizes, integer status codes, no
 * exceptions, no torch/HIP types) so a Java host can bind it through Panama FFM
 * (java.lang.foreign) and rebuild Accord objects through the reference's raw-CSR constructors.
 * See INTEGRATION.md for the Java-side binding.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * accord-core/src/main/java/accord/):
 *
 *   ad_preaccept_deps / ad_fetch_deps
 *       SafeCommandStore.mapReduceActive            local/SafeCommandStore.java:292
 *       InMemorySafeStore.mapReduceActive           impl/InMemoryCommandStore.java:864-871
 *       CommandsForKey.mapReduceActive              local/cfk/CommandsForKey.java:925-983
 *       PreAccept.calculatePartialDeps              messages/PreAccept.java:245-267
 *       Deps.AbstractBuilder.add / build            primitives/Deps.java:80-135
 *       RelationMultiMap.AbstractBuilder.build      utils/RelationMultiMap.java:201-260
 *     output layout == KeyDeps.SerializerSupport.create(Keys, TxnId[], int[])  primitives/KeyDeps.java:69-72
 *                       RangeDeps.SerializerSupport.create(Range[], TxnId[], int[]) primitives/RangeDeps.java:100-103
 *   ad_merge_deps
 *       Deps.merge(List, Function)                  primitives/Deps.java:281-286
 *       KeyDeps.merge / RelationMultiMap.LinearMerger  primitives/KeyDeps.java:115-135, utils/RelationMultiMap.java:284-406
 *       RelationMultiMap.linearUnion                utils/RelationMultiMap.java:562-816
 *   ad_fetch_inverse
 *       KeyDeps.txnIdsToKeys / RangeDeps.txnIdsToRanges  primitives/KeyDeps.java:362-367, RangeDeps.java:576-582
 *       RelationMultiMap.invert                     utils/RelationMultiMap.java:907-938
 *   ad_exec_levels
 *       Commands.initialiseWaitingOn/updateWaitingOn/maybeExecute  local/Commands.java:617-775
 *       CommandsForKey.notifyManaged                local/cfk/CommandsForKey.java:1208-1289
 *
 * Threading: one handle per CommandStore-shard / GPU; a handle owns one HIP stream and its
 * device arena.  Calls on different handles may run concurrently; calls on one handle must
 * be serialised by the caller (InMemoryCommandStore.SingleThread, impl/InMemoryCommandStore.java:1144).
 *
 * Ownership: the caller owns every host buffer passed in; the library never retains a caller
 * pointer after a call returns.  Output sizes come from a two-call protocol (sizes, then a
 * fetch into caller-allocated buffers), mirroring ArrayBuffers' complete/discard discipline
 * (utils/ArrayBuffers.java:32-50).
 */
#ifndef ACCORD_DEPS_H
#define ACCORD_DEPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------ */
/* Status codes (Invariants.illegalArgument / illegalState map onto the negative values).      */
/* ------------------------------------------------------------------------------------------ */
typedef enum ad_status {
    AD_OK = 0,
    AD_ERR_ARGUMENT = -1,      /* IllegalArgumentException (e.g. duplicate key within a txn)  */
    AD_ERR_STATE = -2,         /* IllegalStateException (call order, missing batch)           */
    AD_ERR_UNSORTED = -3,      /* batch TxnIds not strictly ascending (CFK byId order)        */
    AD_ERR_UNSUPPORTED = -4,   /* timestamp/key widths beyond the packed encoding             */
    AD_ERR_DEVICE = -5,        /* HIP runtime error                                           */
    AD_ERR_NOMEM = -6
} ad_status;

/* Txn.Kind ordinals (primitives/Txn.java:53-113); TxnId flags = kind << 1 | domain (TxnId.java:132-165). */
enum { AD_KIND_READ = 0, AD_KIND_WRITE = 1, AD_KIND_EPHEMERAL_READ = 2, AD_KIND_SYNC_POINT = 3,
       AD_KIND_EXCLUSIVE_SYNC_POINT = 4, AD_KIND_LOCAL_ONLY = 5 };
enum { AD_DOMAIN_KEY = 0, AD_DOMAIN_RANGE = 1 };

/* CommandsForKey.InternalStatus ordinals (local/cfk/CommandsForKey.java:493-502). */
enum { AD_ST_TRANSITIVELY_KNOWN = 0, AD_ST_HISTORICAL = 1, AD_ST_PREACCEPTED = 2, AD_ST_ACCEPTED = 3,
       AD_ST_COMMITTED = 4, AD_ST_STABLE = 5, AD_ST_APPLIED = 6, AD_ST_INVALID = 7 };

/* Deps classes, in Deps' own index order (primitives/Deps.java:143-155; DepsTest index order). */
enum { AD_CLASS_KEY = 0, AD_CLASS_DIRECT_KEY = 1, AD_CLASS_RANGE = 2, AD_NUM_CLASSES = 3 };

/* ------------------------------------------------------------------------------------------ */
/* Batch input (host SoA).  One batch = the transactions one CommandStore shard resolves.      */
/*                                                                                             */
/* Timestamps are passed as Accord's raw bits: msb = epoch<<15 | hlc>>>48, lsb = hlc<<16|flags, */
/* node = Node.Id.id (Timestamp.java:77-96).  Ordering is Timestamp.compareTo                  */
/* (Timestamp.java:208-217): msb unsigned, lsb>>>16, lsb & 0x1E, node signed.                  */
/*                                                                                             */
/* TxnIds must be strictly ascending: the batch is CommandsForKey.byId order, which is also    */
/* the arrival order of the status model below.                                               */
/* ------------------------------------------------------------------------------------------ */
typedef struct ad_batch {
    size_t n;                       /* transactions                                           */
    const uint64_t* txn_msb;        /* [n] TxnId                                              */
    const uint64_t* txn_lsb;        /* [n]                                                    */
    const int32_t*  txn_node;       /* [n]                                                    */
    const uint64_t* exec_msb;       /* [n] final (committed) executeAt                        */
    const uint64_t* exec_lsb;       /* [n]                                                    */
    const int32_t*  exec_node;      /* [n]                                                    */
    const uint8_t*  status;         /* [n] the row's InternalStatus (under a replica model with    */
                                    /*     window W > 0: its status once outside the window)      */
    const uint32_t* key_off;        /* [n+1] key footprint CSR                                */
    const uint64_t* keys;           /* [key_off[n]] order-preserving key encoding (Key.compareTo) */
    const uint32_t* range_off;      /* [n+1] range footprint CSR (NULL when no range txns)    */
    const uint64_t* range_start;    /* [range_off[n]] Range.EndInclusive (start, end]         */
    const uint64_t* range_end;      /* [range_off[n]]                                         */
} ad_batch;

/* Store configuration: the number of replica views a handle answers for (the coordinator's R PreAccept
 * replies, CoordinatePreAccept / PreAccept.reduce).  A live GpuCommandStore opens with replicas = 1 and
 * reads every row's status as given (the W = 0 snapshot of SafeCommandStore.mapReduceActive,
 * local/SafeCommandStore.java:292). */
typedef struct ad_config {
    uint32_t replicas;              /* R replica views to build (1..8)                          */
    uint32_t reserved_;             /* 0                                                        */
} ad_config;

/* The benchmark's replica model — a workload generator setting, not store state: when txn i
 * (rank order) is PreAccepted, every txn j < i with j >= i - window is still in flight
 * (PREACCEPTED_OR_ACCEPTED_INVALIDATE); every j < i - window has its given status.  A replica view r in
 * [0, replicas) additionally has not yet witnessed each in-flight j with probability drop_p, decided by
 * ad_drop_hash(seed, r, i, j) (the same function the oracle uses).  A handle starts with window = 0 and
 * drop_p = 0 (the plain snapshot); ad_set_replica_model changes it for the following stage calls. */
typedef struct ad_replica_model {
    uint32_t window;                /* W (BASELINE: 32)                                        */
    float    drop_p;                /* per in-flight dependency drop probability per view       */
    uint64_t seed;                  /* drop hash seed                                          */
} ad_replica_model;

/* ------------------------------------------------------------------------------------------ */
/* Batched PartialDeps output.  For class c of view v, per txn i:                               */
/*   keys      [key_off[i]   .. key_off[i+1])    sorted unique keys (u64) that carry deps       */
/*   txn ranks [txn_off[i]   .. txn_off[i]+txn_cnt[i])  sorted unique dependency ranks (into   */
/*                                                the batch; rank -> TxnId is the batch row)   */
/*   k2t       [k2t_off[i]   .. k2t_off[i+1])    exactly KeyDeps.keysToTxnIds for this txn:    */
/*             nKeys end-offsets (first offset base = nKeys) followed by txn indices           */
/*             (KeyDeps.java:153-172).  For RangeDeps the "keys" are ranges (start,end pairs). */
/* ------------------------------------------------------------------------------------------ */
typedef struct ad_csr_sizes {
    size_t n;                       /* txns                                                     */
    size_t keys;                    /* total key (or range) entries over all txns              */
    size_t k2t;                     /* total keysToTxnIds ints                                  */
    size_t txn_cap;                 /* total txn-rank capacity (sum of per-txn entry counts)    */
    size_t txns;                    /* total unique dependency txns (sum of txn_cnt)            */
} ad_csr_sizes;

typedef struct ad_csr_out {         /* caller-allocated, sized by ad_csr_sizes                  */
    uint32_t* key_off;              /* [n+1]                                                    */
    uint64_t* keys;                 /* [keys]  (RangeDeps: [2*keys] start,end interleaved)      */
    uint32_t* k2t_off;              /* [n+1]                                                    */
    int32_t*  k2t;                  /* [k2t]                                                    */
    uint32_t* txn_off;              /* [n+1]  compacted: txn_off[i+1]-txn_off[i] == txn_cnt[i]  */
    uint32_t* txns;                 /* [txns] dependency ranks                                  */
} ad_csr_out;

typedef struct ad_handle ad_handle;

/* Drop decision shared by the device path and the oracle (splitmix64 finaliser). */
static inline uint64_t ad_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint32_t ad_drop_hash(uint64_t seed, uint32_t view, uint32_t i, uint32_t j) {
    return (uint32_t)(ad_mix64(seed ^ ad_mix64(((uint64_t)view << 56) ^ ((uint64_t)i << 28) ^ (uint64_t)j)) >> 32);
}
static inline uint32_t ad_drop_threshold(float p) {
    if (p <= 0.0f) return 0u;
    if (p >= 1.0f) return 0xFFFFFFFFu;
    return (uint32_t)((double)p * 4294967296.0);
}

/* ------------------------------------------------------------------------------------------ */
/* Lifecycle                                                                                   */
/* ------------------------------------------------------------------------------------------ */
int  ad_open(int device, const ad_config* cfg, ad_handle** out);
/* Benchmark / test generators only (see ad_replica_model): a live store never calls it. */
int  ad_set_replica_model(ad_handle* h, const ad_replica_model* model);
void ad_close(ad_handle* h);
const char* ad_last_error(const ad_handle* h);
int  ad_device_count(void);

/* Copy one batch host->device (the only PCIe transfer of the inputs).  Replaces the previous batch. */
int  ad_load_batch(ad_handle* h, const ad_batch* batch);

/* Double-buffered upload for a stream of batches (the CommandStore's next batch while this one runs):
 * ad_load_batch_async enqueues the H2D copies of `batch` on the handle's copy stream into a second set of
 * input buffers and returns at once; the loaded batch and its results stay untouched.  ad_load_batch_commit
 * waits for those copies (the host arrays may be reused after it returns) and makes the staged batch the
 * loaded one, as ad_load_batch would.  The host arrays must stay valid until the commit; from pinned memory
 * (ad_host_alloc) the copies are DMA transfers that overlap the device work of the loaded batch.  Not for
 * batches after ad_cfk_retain (AD_ERR_UNSUPPORTED: the kept rows are prepended by ad_load_batch). */
int  ad_load_batch_async(ad_handle* h, const ad_batch* batch);
int  ad_load_batch_commit(ad_handle* h);

/* Page-locked host memory for batches and fetched Deps (hipHostMalloc); NULL on failure. */
void* ad_host_alloc(size_t bytes);
void  ad_host_free(void* p);

/* ------------------------------------------------------------------------------------------ */
/* Stage 1 — PreAccept deps for every txn of the loaded batch under cfg->replicas views.       */
/* Runs on the device; sizes[v * AD_NUM_CLASSES + c] receives the CSR sizes of view v class c. */
/* ------------------------------------------------------------------------------------------ */
int  ad_preaccept_deps(ad_handle* h, ad_csr_sizes* sizes /* [replicas*AD_NUM_CLASSES] */);
/* The same deps with bound = executeAt instead of TxnId: Accept.calculatePartialDeps (messages/Accept.java
 * :113-116) and GetDeps.apply (messages/GetDeps.java:76) call PreAccept.calculatePartialDeps with the
 * proposed executeAt, so every txn with TxnId < executeAt (later arrivals included) is a candidate and the
 * txn itself is left out (PreAccept.java:256-261).  Each query is answered at the arrival position of its
 * executeAt (the window / status model applies from there).  Fetch with ad_fetch_deps; ad_merge_deps and the
 * later stages use the last deps computed.  Not in sharded mode (AD_ERR_UNSUPPORTED). */
int  ad_accept_deps(ad_handle* h, ad_csr_sizes* sizes /* [replicas*AD_NUM_CLASSES] */);
/* GetEphemeralReadDeps (messages/GetEphemeralReadDeps.java:76): PreAccept.calculatePartialDeps with bound
 * Timestamp.MAX — every txn of the batch's CFKs and range commands the query kind witnesses (the txn itself
 * left out), answered after every arrival (the in-flight window is the batch's last W txns).  Same outputs as
 * ad_preaccept_deps; not over CFK history batches or sharded stores. */
int  ad_ephemeral_read_deps(ad_handle* h, ad_csr_sizes* sizes /* [replicas*3] */);
int  ad_fetch_deps(ad_handle* h, uint32_t view, uint32_t cls, ad_csr_out* out);

/* Stage 2 — Deps.merge of the R replica replies produced by stage 1 (device-resident). */
int  ad_merge_deps(ad_handle* h, ad_csr_sizes* sizes /* [AD_NUM_CLASSES] */);
int  ad_fetch_merged(ad_handle* h, uint32_t cls, ad_csr_out* out);
/* All three merged classes in one call: sizes[3] (txns == txn_cap: the merged TxnId lists are exact) and the
 * arrays straight from HBM into out[3] with one stream sync (no host-side compaction) — with pinned buffers
 * the whole page-out is three DMA streams.  An empty range class gets zero offsets. */
int  ad_merged_sizes(ad_handle* h, ad_csr_sizes* sizes /* [AD_NUM_CLASSES] */);
int  ad_fetch_merged_all(ad_handle* h, ad_csr_out* out /* [AD_NUM_CLASSES] */);
/* The merged Deps (as ad_fetch_merged_all) and the levels / order (as ad_fetch_levels; either may be NULL) paged out
 * asynchronously: copied on the device into a staging buffer, then paged out on a copy stream while the caller goes
 * on (the next ad_load_batch_commit / ad_run_pipeline may follow at once).  `out` and the level arrays must be pinned
 * host memory (ad_host_alloc) and stay untouched until ad_fetch_wait returns. */
int  ad_fetch_results_async(ad_handle* h, ad_csr_out* out /* [3] */, uint32_t* level_out, uint32_t* order_out);
int  ad_fetch_wait(ad_handle* h);

/* Stage 2 on the fast path — CoordinateTransaction.onPreAccepted (coordinate/CoordinateTransaction.java:71-101):
 * when the coordinator takes the fast path it merges only the replies whose witnessedAt == TxnId (:75); the slow
 * path merges all (:81, ad_merge_deps).  Per txn, view v's reply is folded iff the fast flag of the last
 * ad_max_conflicts / ad_max_conflicts_ts on this batch is set for (v, txn).  Result as ad_merge_deps
 * (ad_fetch_merged / ad_fetch_rows with view == replicas). */
int  ad_merge_deps_fast(ad_handle* h, ad_csr_sizes* sizes /* [AD_NUM_CLASSES] */);

/* Paged fetch: rows [lo, hi) of replica view `view`'s CSR of class `cls` (view == replicas: the merged
 * Deps), offsets rebased to 0.  Two calls: out == NULL fills *sizes (n = hi - lo), then the caller
 * allocates and passes out.  Lets a host stream a full-size batch's Deps (C4: ~10^9 entries per view)
 * txn window by txn window, as the replies of KeyDeps/RangeDeps.SerializerSupport.create are consumed. */
int  ad_fetch_rows(ad_handle* h, uint32_t view, uint32_t cls, size_t lo, size_t hi, ad_csr_sizes* sizes, ad_csr_out* out);

/* The txn -> keys inverse of rows [lo, hi) of view `view`'s class `cls` (view == replicas: the merged Deps), built on
 * the device: KeyDeps.txnIdsToKeys (primitives/KeyDeps.java:362-367) / RangeDeps.txnIdsToRanges
 * (primitives/RangeDeps.java:576-582), i.e. RelationMultiMap.invert (utils/RelationMultiMap.java:907-938) of each row's
 * keysToTxnIds.  Row i's inverse is inv[off[i] .. off[i+1]): nTxnIds end offsets (the first based at nTxnIds), then
 * per TxnId index its key (range) indices ascending — the int[] the reference caches in txnIdsToKeys.  *total = the
 * window's ints; off / inv may be NULL (two calls: sizes, then the data).  AD_ERR_UNSUPPORTED when the window holds
 * 2^31 ints or more (page smaller windows, as with ad_fetch_rows). */
int  ad_fetch_inverse(ad_handle* h, uint32_t view, uint32_t cls, size_t lo, size_t hi, size_t* total,
                      uint32_t* off /* [hi-lo+1] */, int32_t* inv /* [*total] */);

/* Stage 2' — Deps.merge of caller-supplied replies (host CSR, same batch).  parts[r*AD_NUM_CLASSES+c]. */
typedef struct ad_csr_in {
    const uint32_t* key_off; const uint64_t* keys; const uint32_t* k2t_off; const int32_t* k2t;
    const uint32_t* txn_off; const uint32_t* txns;
} ad_csr_in;
int  ad_merge_host(ad_handle* h, const ad_csr_in* parts, uint32_t r, ad_csr_sizes* sizes);

/* Stage 3 — execution order over the merged deps: level_out[i] = Kahn wavefront index of txn i,
 * order_out = txn ranks sorted by (level, executeAt).  Either pointer may be NULL. */
int  ad_exec_levels(ad_handle* h, uint32_t* level_out, uint32_t* order_out, uint32_t* iterations_out);

/* Stage 1b — the replica's witnessedAt proposal per view, after ad_preaccept_deps on the same batch:
 *   CommandStore.preaccept            local/CommandStore.java:322-347   (maxConflicts.get(keys), fast-path test :342-344)
 *   MaxConflicts.get / update         local/MaxConflicts.java:46-59
 *   CommandStore.updateMaxConflicts   local/CommandStore.java:282-291, SafeCommandStore.java:210-222 (globally visible kinds)
 * max_rank[v*n + i] = the batch rank of the txn whose executeAt is maxConflicts.get(keysOrRanges of i) in view v — the
 * greatest executeAt (Timestamp.compareTo; ties to the larger rank) over the globally visible txns j < i whose footprint
 * meets i's that the view has stored (not TRANSITIVELY_KNOWN/INVALID; in-flight j unless the view dropped it) — or
 * AD_RANK_NONE (Timestamp.NONE).  MaxConflicts is a ReducingRangeMap (keys are points, ranges (start, end] intervals):
 * a key txn meets the txns on its keys and the range txns covering one; a range txn the key txns inside its ranges
 * and the range txns crossing them.  fast[v*n + i] = 1 when TxnId_i >= that timestamp (or NONE): the replica answers
 * witnessedAt = TxnId (fast path), else time.uniqueNow(maxConflict), which the host clock supplies.
 * Model assumption (stated, not pinned by the reference): an in-flight j the view holds contributes its batch
 * executeAt — the value MaxConflicts holds once j commits.  In the reference a PreAccepted j contributes the
 * view's own earlier witnessedAt proposal for j (<= its final executeAt for slow-path txns) until it commits,
 * so for views holding slow-path j in flight max_rank / fast may be higher / lower than a live replica's.
 * The oracle (oracle.cpp Oracle::max_conflict) makes the same assumption.
 * Either pointer may be NULL.  Sharded stores (ad_shard_setup): rows are local, max_rank holds global arrival ranks; PreAccept.reduce's
 * mergeMax across stores (messages/PreAccept.java:141-156) is then a per-txn max over the stores' answers. */
#define AD_RANK_NONE 0xFFFFFFFFu
/* ad_exec_levels over a batch carrying CFK history: the level of a row already APPLIED or INVALID (done) */
#define AD_LEVEL_DONE 0xFFFFFFFFu
int  ad_max_conflicts(ad_handle* h, uint32_t* max_rank /* [replicas*n] */, uint8_t* fast /* [replicas*n] */);

/* The rest of CommandStore.preaccept (local/CommandStore.java:322-347) around maxConflicts.get; it shapes the fast
 * flags of ad_max_conflicts and ad_max_conflicts_ts (the same store state answers every view):
 *   isExpired = now - TxnId.hlc >= preAcceptTimeout && !kind.isSyncPoint()                         (:326)
 *            || rejectBefore.foldl(keys, rejectIfBefore > TxnId -> reject)                            (:327-328)
 *     -> the replica answers time.uniqueNow(TxnId).asRejected(): fast = AD_FAST_REJECTED               (:330-331)
 *   an ExclusiveSyncPoint that is not expired answers its TxnId whatever maxConflict is: fast = 1      (:333-337)
 * ad_preaccept_expiry sets that state for the following calls: the node clock's now (hlc units) and
 * Agent.preAcceptTimeout (AD_NO_TIMEOUT: no timeout test; the handle's default), and rejectBefore — the
 * ReducingRangeMap<Timestamp> markExclusiveSyncPoint builds (:300-306: Timestamp::max of the ExclusiveSyncPoint TxnIds
 * marked over each range) — as sorted disjoint intervals (start, end] with a Timestamp each (a key k stabs
 * (k - 1, k]); m = 0 clears it.  The host merges each batch's ExclusiveSyncPoints into it (witness.RejectBefore). */
#define AD_FAST_REJECTED 2
#define AD_NO_TIMEOUT 0xFFFFFFFFFFFFFFFFull
int  ad_preaccept_expiry(ad_handle* h, uint64_t now_hlc, uint64_t pre_accept_timeout, size_t m, const uint64_t* starts,
                         const uint64_t* ends, const uint64_t* msb, const uint64_t* lsb, const int32_t* node);

/* Stage 1b across batches — the store's MaxConflicts map outlives a batch (local/MaxConflicts.java:32-96,
 * CommandStore.updateMaxConflicts :282-291).  The host carries it between batches as a table sorted by key:
 *   ad_max_conflicts_carry   the table from earlier batches (keys strictly ascending; m = 0 clears it); it applies
 *                            to every later ad_max_conflicts_ts on this handle and to the export
 *   ad_max_conflicts_ts      per view v and txn i: maxConflicts.get(keys of i) over the carried table AND the batch
 *                            (as ad_max_conflicts), as a raw Timestamp (msb, lsb, node; Timestamp.NONE = 0, 0, 0),
 *                            and fast = TxnId >= it (CommandStore.java:343).  Arrays [replicas*n]; NULL skips one
 *   ad_max_conflicts_export  the table after this batch: the carry merged with every key's greatest recorded
 *                            executeAt in the batch (final statuses; TRANSITIVELY_KNOWN / INVALID unrecorded).
 *                            Two calls: keys == NULL returns *m only.  Needs ad_max_conflicts(_ts) on the batch.
 *   ad_max_conflicts_carry_ranges   the range part of the carried map (MaxConflicts is a ReducingRangeMap,
 *                            local/MaxConflicts.java:32-59): sorted disjoint intervals (start, end] (start < end,
 *                            end <= next start) with a Timestamp each; m = 0 clears it.  A key k is the interval
 *                            (k - 1, k], so the key table and the intervals together are the whole map: _ts folds
 *                            every carried key and interval the txn's keys or ranges meet (range txns included)
 *   ad_max_conflicts_export_ranges  the intervals after this batch: the carried intervals merged with every range
 *                            the batch's recorded range txns cover (MaxConflicts.update = merge(this, create(ranges,
 *                            executeAt)), Timestamp::max), as the normal form — maximal pieces of one value.  Two calls
 *                            as _export (starts == NULL: *m only).  Key txns update the key table, range txns the
 *                            intervals; Timestamps that compare equal keep the larger raw lsb.
 * A txn that PreAccepts in a later batch than a larger-TxnId txn (arrival order != TxnId order,
 * PreAcceptTest.multiKeyTimestampUpdate) sees it through the carry. */
int  ad_max_conflicts_carry(ad_handle* h, size_t m, const uint64_t* keys, const uint64_t* msb, const uint64_t* lsb,
                            const int32_t* node);
int  ad_max_conflicts_carry_ranges(ad_handle* h, size_t m, const uint64_t* starts, const uint64_t* ends,
                                   const uint64_t* msb, const uint64_t* lsb, const int32_t* node);
int  ad_max_conflicts_ts(ad_handle* h, uint64_t* msb, uint64_t* lsb, int32_t* node, uint8_t* fast);
int  ad_max_conflicts_export(ad_handle* h, size_t* m, uint64_t* keys, uint64_t* msb, uint64_t* lsb, int32_t* node);
int  ad_max_conflicts_export_ranges(ad_handle* h, size_t* m, uint64_t* starts, uint64_t* ends, uint64_t* msb,
                                    uint64_t* lsb, int32_t* node);

/* ------------------------------------------------------------------------------------------ */
/* Device-resident pipeline (benchmark / service loop): stage 1 + 2 + 3 with no host copies of */
/* outputs.  Kernel timing: HIP events on the handle's stream.                                 */
/* ------------------------------------------------------------------------------------------ */
int  ad_run_pipeline(ad_handle* h);
/* on != 0: ad_run_pipeline builds the merged Deps as the deps stage's "union view" (an entry kept by any replica
 * view) instead of merging the R replies (k_merge_cap, the default).  A shortcut only a generator holding every
 * view's inputs can take — a coordinator receiving replies from other nodes cannot; kept as a side figure. */
int  ad_set_pipeline_union(ad_handle* h, int on);
/* Levels and execution order left on the device by the last ad_run_pipeline / ad_exec_levels (no
 * recomputation).  Either pointer may be NULL.  AD_ERR_STATE if none were computed for this batch. */
int  ad_fetch_levels(ad_handle* h, uint32_t* level_out, uint32_t* order_out);
typedef struct ad_stage_times {     /* milliseconds of the last ad_run_pipeline, event-timed */
    float prepare, sort, deps, merge, levels, total;
    uint64_t deps_entries;          /* emitted (key,txn) entries over all views/classes      */
    uint64_t merged_entries;        /* entries of the merged Deps                             */
    uint64_t level_edges;           /* key-chain entries visited per level sweep              */
    uint32_t level_iterations;
    uint32_t walk_items;            /* (txn,key) entries with an earlier entry of their key: the */
                                    /* ones the deps walks visit (P - distinct keys)             */
    uint32_t level_blocks;          /* executeAt blocks walked by the block level path (0: Kahn)  */
    uint32_t level_rounds;          /* block-scan rounds over those blocks                        */
    uint32_t key_classes;           /* key-footprint CSRs the deps stage computed per batch: 2R, or */
                                    /* R when the batch has no directKeyDeps (no key sync points)   */
    uint32_t level_path;            /* the pull levels' outcome: 0 not tried, 1 pulled, 2 a far    */
                                    /* predecessor (> 65536 rows ahead) -> Kahn, 3 aborted -> Kahn;  */
                                    /* mixed key + range batches 10 + (1 pulled in executeAt order,  */
                                    /* 2 long chain, 3 ExclusiveSyncPoint / EphemeralRead present, 4 */
                                    /* executeAt rank miss, 5 aborted) -> else the Kahn wavefronts   */
    uint32_t deferred_txns;         /* small txns the walk's inline ids could not finish: unioned by  */
                                    /* k_txn_union (the rest by k_txn_finish)                         */
    uint32_t fill_items;            /* (txn, key) entries the fill walk re-walks (pairs of txns with   */
                                    /* more than 4 keys)                                              */
    uint32_t deps_speculative;      /* k_txn_finish launched before the CSR sizes reached the host:    */
                                    /* 0 no, 1 yes and the buffers fit, 2 yes but re-run after sizing  */
    uint64_t vitems;                /* virtual query items of large txns (one per (txn, CFK key))      */
    uint64_t range_entries;         /* RangeDeps entries over all views (part of deps_entries)         */
    uint32_t gather_items;          /* entries in key segments of more than one entry: the records the */
                                    /* fused tile kernel (k_seg_fuse) gathers (walk_items + segments);  */
                                    /* 0 when the batch took the three-kernel path                      */
    uint32_t chains_fused;          /* 1: k_seg_fuse built the pull pass's key chains (no k_chain_build) */
} ad_stage_times;
int  ad_last_times(ad_handle* h, ad_stage_times* out);

/* Execution-level algorithm (all give identical levels; the choice only affects speed):
 * AD_LEVELS_AUTO (default): batches with only key Read/Write txns (no direct/range deps, no range txns) use
 * one-pass pull levels (each txn publishes 1 + its predecessors' maximum once they are final, one launch)
 * while every key chain is short, and executeAt blocks (block_levels.h: a Jacobi fixpoint of write-epoch max
 * scans per block, walked in executeAt order) when some chain is long (deep graphs: Zipf hot keys); mixed batches use
 * the Kahn wavefront (each txn visited once, when released) with explicit (b)/(c) edges.
 * AD_LEVELS_FIXPOINT always uses the chain fixpoint; AD_LEVELS_BLOCKS uses the executeAt blocks for every
 * key-only batch; AD_LEVELS_KAHN uses the Kahn wavefront instead of the pull levels (tests cross-check the
 * algorithms). */
#define AD_LEVELS_AUTO 0
#define AD_LEVELS_FIXPOINT 1
#define AD_LEVELS_BLOCKS 2
#define AD_LEVELS_KAHN 3
#define AD_LEVELS_PULL_ABORT 4      /* tests: the pull levels abort at once, the Kahn wavefronts recompute the batch */
#define AD_LEVELS_BLOCKS_WIDE 5     /* tests: AD_LEVELS_BLOCKS with the 64-bit scan words batches of > 2^20 txns use */
int  ad_set_level_mode(ad_handle* h, int mode);

/* Per-kernel HIP-event timing (trace mode).  mask bit k enables kernel id k (0 <= k < ad_kernel_count()); the
 * events are recorded on the handle's stream around each launch of that kernel.  ad_kernel_stats
 * synchronises the stream and returns the kernel's name, launches and summed milliseconds since the
 * last ad_reset_kernel_stats. */
int  ad_set_trace(ad_handle* h, uint64_t mask);
int  ad_kernel_count(void);
const char* ad_kernel_name(int kid);
int  ad_kernel_stats(ad_handle* h, int kid, const char** name, uint64_t* calls, double* total_ms);
int  ad_reset_kernel_stats(ad_handle* h);
/* elements the traced launches of kernel kid processed (its algorithmic unit: pairs, txns, sort items) */
int  ad_kernel_units(ad_handle* h, int kid, uint64_t* units);

/* ------------------------------------------------------------------------------------------ */
/* Recovery — BeginRecovery's store queries (messages/BeginRecovery.java:126-145) for the   */
/* recovering txns rows[nq] of the loaded batch, each a SafeCommandStore.mapReduceFull over its footprint     */
/* (CommandsForKey.mapReduceFull local/cfk/CommandsForKey.java:824-923 per key, mapReduceRangesInternal        */
/* impl/InMemoryCommandStore.java:884-1017 over the range commands):                                         */
/*   which 0  earlierCommittedWitness  = stableStartedBeforeAndWitnessed :344-352                              */
/*   which 1  earlierAcceptedNoWitness = acceptedOrCommittedStartedBeforeWithoutWitnessing :329-342            */
/*   flags    rejectsFastPath = hasAcceptedOrCommittedStartedAfterWithoutWitnessing :354-367                   */
/*                              || hasStableExecutesAfterWithoutWitnessing :369-380                            */
/* The store is the loaded batch with its statuses and executeAts (every txn known, nothing pruned); each      */
/* txn's Deps are the merged Deps on the handle (ad_merge_deps / _fast / ad_merge_host: what it was accepted   */
/* or committed with); a CFK entry's missing() follows the CommandsForKey invariant (Updating.java:194-287,    */
/* :340-352).  Rows already PreCommitted (status >= COMMITTED) answer Deps.NONE and false (:126-130).         */
/* entries[which * 3 + class] receives the entry counts.  ad_fetch_recovery returns one (Deps, class) as the   */
/* built Deps flattened to its (key or range, TxnId rank) entries in Deps order: off[nq + 1] per recovering    */
/* txn, keys[entries] (range class: [2 * entries] start, end), txns[entries]; any pointer may be NULL.        */
/* Not in sharded mode.                                                                                       */
/* ------------------------------------------------------------------------------------------ */
int  ad_recover(ad_handle* h, const uint32_t* rows, size_t nq, size_t* entries /* [6], or NULL */);
int  ad_fetch_recovery(ad_handle* h, uint32_t which, uint32_t cls, uint32_t* off, uint64_t* keys, uint32_t* txns);
int  ad_fetch_recovery_flags(ad_handle* h, uint8_t* reject_fast_path /* [nq] */);

/* ------------------------------------------------------------------------------------------ */
/* CommandsForKey state across batches.  A store's batches continue one TxnId order; instead  */
/* of a closed world per batch, ad_cfk_retain (after ad_preaccept_deps on a batch) keeps on the device every txn */
/* whose CFK entries a later query can still see — in flight for a later query (global rank >= next - W), or on  */
/* some key not prunable (Pruning.java:164-233: TRANSITIVELY_KNOWN / INVALID / unmanaged entries, and committed  */
/* Reads/Writes executing before the key's greatest committed Write below every later TxnId, are never emitted  */
/* again by mapReduceActive, CommandsForKey.java:925-983).  The next ad_load_batch puts those rows first: the    */
/* loaded batch is [kept rows | new txns], window / drop decisions and MaxConflicts use global arrival ranks,    */
/* and every output row / TxnId is a combined row (ad_cfk_rows maps rows to global ranks).  The new txns'      */
/* deps equal those of the whole stream resolved at once.  Statuses of kept rows are current (ad_cfk_update);  */
/* ad_exec_levels orders the combined rows with APPLIED / INVALID rows done.  Key batches only; ad_accept_deps   */
/* and sharded mode are refused over a batch with history rows (AD_ERR_UNSUPPORTED).                            */
/* ------------------------------------------------------------------------------------------ */
int  ad_cfk_retain(ad_handle* h, size_t* retained /* out: kept rows, or NULL */);
int  ad_cfk_reset(ad_handle* h);                        /* forget the kept rows: the next batch starts afresh */
/* State transitions between batches (after ad_cfk_retain, before the next ad_load_batch): the kept rows with
 * global ranks gid[m] (strictly ascending) move to status[m] (InternalStatus), with executeAt (three arrays, or
 * all NULL to keep it).  Replaces CommandsForKey.update on Commit / Stable / Apply / Invalidate
 * (CommandsForKey.java:987-1057, Updating.java:99-358).  Legal moves are CommandsForKeyTest's TRANSITIONS
 * (CommandsForKeyTest.java:235-246): TRANSITIVELY_KNOWN / PREACCEPTED -> PREACCEPTED, ACCEPTED, COMMITTED,
 * STABLE, INVALID; ACCEPTED -> COMMITTED, STABLE, INVALID; COMMITTED -> STABLE; STABLE -> APPLIED.  executeAt
 * >= TxnId once decided and fixed from COMMITTED on.  Every update is checked first; AD_ERR_ARGUMENT (none
 * applied) names the first refused one (not a kept row, illegal move, executeAt rule).  The next ad_cfk_retain
 * prunes rows that became APPLIED below an applied Write's executeAt (Pruning.java:164-233) or INVALID, and
 * ad_exec_levels over the next batch treats APPLIED / INVALID rows as done (AD_LEVEL_DONE). */
int  ad_cfk_update(ad_handle* h, size_t m, const uint32_t* gid, const uint8_t* status, const uint64_t* exec_msb,
                   const uint64_t* exec_lsb, const int32_t* exec_node);
int  ad_cfk_rows(ad_handle* h, size_t* hist_rows /* out */, uint32_t* gid /* [n] global rank per row, or NULL */);

/* CommandsForKey's execution release rule over CFK states as a store holds them (the reference's serialized form,
 * CommandsForKey.SerializerSupport.create(Key, TxnInfo[], Unmanaged[], prunedBefore), local/cfk/CommandsForKey.java
 * :226-232): per key, its byId TxnInfos — TxnId, InternalStatus, executeAt, missing().  Replaces
 * CommandsForKey.notifyManaged (:1208-1289) run over all of committedByExecuteAt with every kind admitted:
 * not_waiting[row] = 1 for each STABLE key Read / Write the rule lets go (NotifySink.notWaiting on this key) — it
 * lies after the last applied Write and at or before the first unapplied Write (executeAt order), and the undecided
 * (status < COMMITTED) Reads / Writes with a lower TxnId than its executeAt that it conflicts with, plus the
 * unapplied committed Reads ahead of it when it is a Write, number exactly its missing entries from minUndecided on
 * (:1237-1280): a Stable txn whose dependency set holds an undecided lower TxnId waits for it to be decided.
 * Undecided rows (status < ACCEPTED) need no executeAt (the fields are not read).  Each key is computed
 * independently (one workgroup per key); pruning state (prunedBefore, loadingPruned) is not taken: the states must
 * not be waiting on pruned TxnIds.  AD_ERR_UNSORTED if a key's TxnIds are not strictly ascending, AD_ERR_ARGUMENT
 * for a missing index outside its key. */
typedef struct ad_cfk_state {
    size_t keys;                    /* CFK states                                                */
    size_t rows;                    /* TxnInfo rows over all keys                                */
    const uint32_t* row_off;        /* [keys+1] rows of key k: [row_off[k], row_off[k+1]), byId (TxnId) order */
    const uint64_t* txn_msb;        /* [rows] TxnId                                              */
    const uint64_t* txn_lsb;
    const int32_t*  txn_node;
    const uint64_t* exec_msb;       /* [rows] executeAt (ACCEPTED .. APPLIED rows)               */
    const uint64_t* exec_lsb;
    const int32_t*  exec_node;
    const uint8_t*  status;         /* [rows] InternalStatus (AD_ST_*)                           */
    const uint32_t* miss_off;       /* [rows+1] TxnInfo.missing() CSR                            */
    const uint32_t* missing;        /* row indices within the key (0 = its first row), ascending */
} ad_cfk_state;
int  ad_cfk_notify(ad_handle* h, const ad_cfk_state* s, uint8_t* not_waiting /* [rows] */);

/* Device-resident CommandsForKey states.  The handle keeps `keys` CFKs of up to `capacity` TxnInfo rows
 * each in HBM -- byId rows (TxnId, InternalStatus, executeAt) and their missing() sets -- and applies the host's
 * stream of CommandsForKey.update calls to them on the device:
 *   CommandsForKey.update / Updating.insertOrUpdate   local/cfk/CommandsForKey.java:987-1057, Updating.java:99-358
 *   (missing() maintained as the reference does: a row with deps misses every undecided txn below its depsKnownBefore
 *   it witnesses and its deps lack; deps unknown to the CFK become TRANSITIVELY_KNOWN rows, :178-227; a newly known
 *   undecided txn joins, a txn that commits or is invalidated leaves, every other row's missing set --
 *   Utils.addToMissingArrays / removeFromMissingArrays, Utils.java:70-172)
 *   Updating.updateUnmanaged's insertAdditionsOnly (:452-514): an event with status TRANSITIVELY_KNOWN
 * Ballots are zero: an event whose InternalStatus does not rise above the row's is ignored.  Events are grouped by key
 * (ev_off[key] .. ev_off[key + 1]) and applied in order per key, keys in parallel (one workgroup each).
 * ad_cfk_store_notify then runs CommandsForKey.notifyManaged's release rule (as ad_cfk_notify) over the resident
 * rows -- nothing is uploaded -- and ad_cfk_store_fetch reads one key back in ad_cfk_state's layout (missing() as byId
 * row indices).  capacity <= 8192 (rounded up to a multiple of 64); AD_ERR_UNSUPPORTED when a key outgrows it.
 * Pruning (local/cfk/Pruning.java) on the resident rows, by event op (op == NULL: every event AD_CFK_OP_UPDATE):
 *   AD_CFK_OP_UPDATE   CommandsForKey.update; deps below the key's prunedBefore that it lacks join its loadingPruned
 *                      table witnessed by the command (Utils.removePrunedAdditions :229-244, Updating.java:111-117)
 *                      instead of becoming rows; a TxnId in loadingPruned takes the LOAD path (:1015-1016)
 *   AD_CFK_OP_LOAD     CommandsForKey.updatePruned (:998-1005): the loaded command's row (no missing(); the TxnId joins
 *                      the other rows' missing() except its loadingPruned witnesses'; the entry leaves the table)
 *   AD_CFK_OP_PRUNE    CommandsForKey.maybePrune(pruneInterval = exec_node, minHlcDelta = exec_msb) (Pruning.java:164-331)
 *   AD_CFK_OP_LOADING  txn joins loadingPruned witnessed by its one dep, if any (an unmanaged's pruned deps,
 *                      Updating.java:806-815)
 *   AD_CFK_OP_UNMANAGED         registerUnmanaged (Updating.updateUnmanaged :715-849, register = true) of unmanaged txn
 *                               txn (a range txn, sync point or ephemeral read; exec = its executeAt) whose Read / Write
 *                               deps at this key are the event's deps: readyToApply -> notified (tag 2), else joins the
 *                               key's unmanaged registry as (APPLY, executesAt) or (COMMIT, its last dep).  The TRANSITIVELY_
 *                               KNOWN rows / LOADING entries of deps the key does not know are the events before it.
 *   AD_CFK_OP_UNMANAGED_RECHECK updateUnmanaged(register = false): an unmanaged notified of commit, re-checked
 * Every UPDATE / LOAD that changes a row then runs PostProcess.notifyUnmanaged (:164-246) over the registry: entries waiting
 * for commits below minUndecided (and the first loadingPruned TxnId) are notified (tag 0) and leave it, and after an apply
 * those whose waitingUntil the contiguous applied prefix reached (tag 1).  ad_cfk_store_notified returns the last apply's
 * notifications, ad_cfk_store_unmanaged a key's registry.
 * ad_cfk_store_notify holds a STABLE txn whose loadingPruned witness entry precedes its executeAt (isWaitingOnPruned,
 * Pruning.java:119-135); ad_cfk_store_pruning reads prunedBefore and the table back.                                 */
#define AD_CFK_OP_UPDATE  0
#define AD_CFK_OP_LOAD    1
#define AD_CFK_OP_PRUNE   2
#define AD_CFK_OP_LOADING 3
#define AD_CFK_OP_UNMANAGED 4
#define AD_CFK_OP_UNMANAGED_RECHECK 5
typedef struct ad_cfk_events {
    size_t m;                       /* events                                                          */
    const uint32_t* ev_off;         /* [keys + 1] events of key k: [ev_off[k], ev_off[k + 1])          */
    const uint64_t* txn_msb;        /* [m] the command's TxnId (lsb: flags with kind and domain)       */
    const uint64_t* txn_lsb;
    const int32_t*  txn_node;
    const uint8_t*  status;         /* [m] its InternalStatus after the update (AD_ST_*)              */
    const uint64_t* exec_msb;       /* [m] executeAt (statuses ACCEPTED .. APPLIED)                   */
    const uint64_t* exec_lsb;
    const int32_t*  exec_node;
    const uint32_t* deps_off;       /* [m + 1] the command's deps at this key (statuses with deps)     */
    const uint64_t* deps_msb;       /*         TxnIds strictly ascending                              */
    const uint64_t* deps_lsb;
    const int32_t*  deps_node;
    const uint8_t*  op;             /* [m] AD_CFK_OP_* per event, or NULL                              */
} ad_cfk_events;
int  ad_cfk_store_open(ad_handle* h, uint32_t keys, uint32_t capacity);
/* Two tiers: every key starts with `capacity` rows (loadingPruned / unmanaged entries alike); a key that an event would
 * take past them stops before that event, moves to one of `big_keys` large-tier slots of `big_capacity` rows (its rows
 * and missing() bitmaps copied and re-strided on the device) and resumes from the event in the same call.  Memory:
 * keys x capacity + big_keys x big_capacity rows, missing() bitmaps quadratic in each tier's capacity.
 * 1 <= capacity <= 8192, capacity < big_capacity <= 16384.  ad_cfk_store_open = no large tier. */
int  ad_cfk_store_open_tiered(ad_handle* h, uint32_t keys, uint32_t capacity, uint32_t big_capacity, uint32_t big_keys);
int  ad_cfk_store_apply(ad_handle* h, const ad_cfk_events* ev);
/* not_waiting: each key's first `capacity` rows (a large-tier key's others: ad_cfk_store_notify_key) */
int  ad_cfk_store_notify(ad_handle* h, uint32_t* rows /* [keys] */, uint8_t* not_waiting /* [keys * capacity] */);
/* after ad_cfk_store_notify: one key's flags for all of its rows (*rows; not_waiting may be NULL: count only) */
int  ad_cfk_store_notify_key(ad_handle* h, uint32_t key, uint8_t* not_waiting, size_t rows_cap, size_t* rows);
/* one key's rows: *rows (and *missing total); arrays may be NULL (two calls); miss_off[rows + 1], missing = byId row
 * indices within the key, ascending per row */
int  ad_cfk_store_fetch(ad_handle* h, uint32_t key, size_t* rows, size_t* missing_total, uint64_t* txn_msb,
                        uint64_t* txn_lsb, int32_t* txn_node, uint64_t* exec_msb, uint64_t* exec_lsb, int32_t* exec_node,
                        uint8_t* status, uint32_t* miss_off, uint32_t* missing);
/* one key's prunedBefore (TxnId.NONE: zeros) and loadingPruned table: *loading entries (and *witness_total); arrays may
 * be NULL (two calls); lp_off[loading + 1], lp_rows = the witnesses that are rows, as byId row indices ascending    */
int  ad_cfk_store_pruning(ad_handle* h, uint32_t key, uint64_t* pruned_msb, uint64_t* pruned_lsb, int32_t* pruned_node,
                          size_t* loading, size_t* witness_total, uint64_t* lp_msb, uint64_t* lp_lsb, int32_t* lp_node,
                          uint32_t* lp_off, uint32_t* lp_rows);
/* one key's unmanaged registry in Unmanaged.compareTo order: *count entries of (pending: 0 COMMIT / 1 APPLY, waitingUntil,
 * TxnId); arrays may be NULL (two calls) */
int  ad_cfk_store_unmanaged(ad_handle* h, uint32_t key, size_t* count, uint8_t* pending, uint64_t* wait_msb,
                            uint64_t* wait_lsb, int32_t* wait_node, uint64_t* txn_msb, uint64_t* txn_lsb, int32_t* txn_node);
/* the last ad_cfk_store_apply's unmanaged notifications, per key in order (counts[keys]), keys concatenated: event = the
 * index among that key's events of the call, tag 0 commit (NotifyUnmanagedOfCommit), 1 applied (NotifyNotWaiting),
 * 2 ready at its (re)registration; arrays may be NULL (two calls) */
int  ad_cfk_store_notified(ad_handle* h, uint32_t* counts, size_t* total, uint32_t* event, uint8_t* tag, uint64_t* txn_msb,
                           uint64_t* txn_lsb, int32_t* txn_node);
/* CommandsForKey.mapReduceActive over the resident rows (local/cfk/CommandsForKey.java:925-983), as
 * PreAccept.calculatePartialDeps (messages/PreAccept.java:245-267) asks it, for a batch of queries: query q's txn on its
 * store keys with bound startedBefore (PreAccept / ExclusiveSyncPoint: its TxnId; Accept / GetDeps: its executeAt, the txn
 * itself then left out), kinds = the txn's Kind.witnesses(); elision against the last committed Write executing before
 * the bound; when startedBefore <= the key's prunedBefore, the earliest committed Write executing at or after it (the
 * future dependency standing in for pruned txns, :967-980).  Per query its PartialDeps' keyDeps (Read / Write deps) and
 * directKeyDeps (sync points) in Deps.Builder's canonical CSR (Deps.java:80-106): keys = store key indices ascending,
 * unique TxnIds ascending, keysToTxnIds.  sizes[2]: keyDeps, directKeyDeps (n = queries).  Errors as ad_cfk_store_apply;
 * AD_ERR_UNSORTED when a query's keys are not strictly ascending. */
typedef struct ad_cfk_queries {
    size_t nq;
    const uint32_t* key_off;        /* [nq + 1] query q's keys: [key_off[q], key_off[q + 1])           */
    const uint32_t* keys;           /* store key indices, strictly ascending per query                 */
    const uint64_t* txn_msb;        /* [nq] the querying txn's TxnId (kind from lsb)                   */
    const uint64_t* txn_lsb;
    const int32_t*  txn_node;
    const uint64_t* bound_msb;      /* [nq] startedBefore                                              */
    const uint64_t* bound_lsb;
    const int32_t*  bound_node;
} ad_cfk_queries;
int  ad_cfk_store_query(ad_handle* h, const ad_cfk_queries* q, ad_csr_sizes* sizes /* [2] */);
/* one class of the last ad_cfk_store_query: out->key_off / keys / k2t_off / k2t / txn_off sized by its sizes (out->txns, if
 * not NULL, gets 0..txns-1); the TxnIds themselves into txn_msb / txn_lsb / txn_node [txns] */
int  ad_cfk_store_query_fetch(ad_handle* h, uint32_t cls, ad_csr_out* out, uint64_t* txn_msb, uint64_t* txn_lsb,
                              int32_t* txn_node);

/* ------------------------------------------------------------------------------------------ */
/* Multi-GPU key-range sharding (one handle = one CommandStore = one GPU).                     */
/*                                                                                             */
/* Replaces CommandStores.mapReduce across stores (local/CommandStores.java:576-593) and       */
/* PreAccept.reduce (messages/PreAccept.java:141-156, Deps.with of the per-store PartialDeps). */
/* Protocol per store:                                                                         */
/*   ad_load_batch(local batch: txns touching the store's key range, keys sliced to it)        */
/*   ad_shard_setup(local row -> global rank, local row -> home store)   then ad_preaccept_deps */
/*   ad_shard_export: per destination store, the deps rows of the local txns homed there (rows  */
/*   without deps are not sent), TxnIds as global ranks -> bytes[d]                             */
/*   exchange: all-to-all (the peers' byte counts give recv_sizes): ad_comm_init +              */
/*   ad_shard_alltoall over RCCL/xGMI, or ad_shard_send_to_host / ad_shard_import_host over a   */
/*   host transport -> ad_shard_merge                                                          */
/*   levels, delta exchange (after ad_shard_set_holders): ad_shard_levels_round appends, per     */
/*   peer store, the levels it raised for txns that peer also holds; ad_shard_levels_exchange   */
/*   (RCCL: all-gather of the per-peer counts + grouped send/recv of the pairs) or              */
/*   ad_shard_levels_deltas / ad_shard_levels_apply over a host transport; repeat until no      */
/*   store sent a pair.  Dense variant (no holders set): all-reduce(max) of the whole global    */
/*   level array (ad_shard_levels_allreduce, or _get/_set).  Then ad_shard_order.               */
/* Home txn = its first key (a range txn: its first range's first key, start + 1) lies in this  */
/* store's range; results are per home txn, TxnIds as global ranks.  Range txns: the host       */
/* slices each range to the store, (max(start, lo-1), min(end, hi-1)] for keys [lo, hi)         */
/* (InMemoryCommandStore.java:758-761); blobs then carry RangeDeps per view (header word         */
/* nvc | nr << 16), and ad_shard_fetch(AD_CLASS_RANGE) returns the store-sliced RangeDeps.      */
/* Range txns, sync points and ephemeral reads take their (b)/(c) level constraints from the    */
/* store's own Deps.merge of its views (first level round); ad_max_conflicts answers range      */
/* footprints per store in global ranks too (fold: sharding.reduce_witnessed).  At most 8 stores.*/
/* ------------------------------------------------------------------------------------------ */
int  ad_shard_bounds(const uint64_t* keys, size_t nkeys, uint32_t shards, uint64_t* bounds_out /* [shards+1] */);
int  ad_shard_setup(ad_handle* h, const uint32_t* gid /* [n] ascending */, const uint8_t* home_store /* [n] */,
                    uint32_t self, uint32_t world, size_t n_global);
int  ad_shard_export(ad_handle* h, uint64_t* bytes /* [world]: blob size per destination */);
int  ad_shard_send_to_host(ad_handle* h, void* dst /* [sum bytes]: blobs in destination order */);
int  ad_shard_import_host(ad_handle* h, const void* src /* blobs in source order */, uint32_t world,
                          const uint64_t* sizes /* [world] */);
int  ad_comm_unique_id(uint8_t* out /* [128] */);
/* Accept / GetDeps (ad_accept_deps) on a sharded store: gq[n] = per local row, the number of TxnIds of the GLOBAL
 * batch below the row's executeAt (the arrival position its executeAt-bound query is answered at; the store holds
 * only its slice).  Messages/Accept.java:113-116 run per store through CommandStores.mapReduce
 * (local/CommandStores.java:576-593).  Required before ad_accept_deps on a sharded handle (not for
 * ad_ephemeral_read_deps: Timestamp.MAX is after every arrival); valid until the next load.  ad_recover works on
 * sharded stores as on any store: each answers from its own slice and its own replicas' merged Deps (the
 * reference's per-store PartialDeps; messages/BeginRecovery.java:118). */
int  ad_shard_query_positions(ad_handle* h, const uint32_t* gq);
int  ad_comm_init(ad_handle* h, uint32_t world, uint32_t rank, const uint8_t* id /* [128] */);
/* Aborts and releases the handle's communicator (a partial init across ranks: the ranks whose init succeeded
 * drop theirs before falling back to a host transport).  No-op without one. */
int  ad_comm_destroy(ad_handle* h);
int  ad_shard_alltoall(ad_handle* h, const uint64_t* recv_sizes /* [world]: peers' bytes[this store] */);
int  ad_shard_merge(ad_handle* h, ad_csr_sizes* sizes /* [(replicas+1)*3]; view == replicas: merged */, size_t* n_home);
int  ad_shard_fetch(ad_handle* h, uint32_t view, uint32_t cls, ad_csr_out* out, uint32_t* home_gid /* [n_home] or NULL */);
/* holders[r]: bitmask of the stores that hold local row r's txn (bit self set; < 1 << world).  Switches
 * the level rounds to the delta exchange: per round only the raised levels of txns shared with a peer
 * travel to that peer, as u64 (global rank << 32 | level) pairs. */
int  ad_shard_set_holders(ad_handle* h, const uint8_t* holders /* [n] */);
int  ad_shard_levels_round(ad_handle* h, int first, uint32_t* changed /* delta mode: this store sent a pair */);
/* The pairs of the last round per destination store: counts[world]; pairs (nullable) receives them
 * concatenated in destination order. */
int  ad_shard_levels_deltas(ad_handle* h, uint32_t* counts /* [world] */, uint64_t* pairs);
int  ad_shard_levels_apply(ad_handle* h, const uint64_t* pairs, size_t m);      /* received pairs, max-folded */
/* RCCL: exchange the last round's pairs with every peer; *any_sent = some store sent a pair this round
 * (0: the levels are final on every store). */
int  ad_shard_levels_exchange(ad_handle* h, uint32_t* any_sent);
int  ad_shard_levels_get(ad_handle* h, uint32_t* G /* [n_global] */);
int  ad_shard_levels_set(ad_handle* h, const uint32_t* G);
int  ad_shard_levels_allreduce(ad_handle* h, uint32_t* any_changed /* out: max of the stores' round flags, or NULL */);
int  ad_shard_order(ad_handle* h, uint32_t* level_out /* [n_home] */, uint32_t* order_out /* [n_home] global ranks */);
/* One-exchange levels (the default protocol): every execution constraint is local to one store, so the
 * batch's level DAG is the union of the stores' constraint graphs.  ad_shard_level_edges gives this store's
 * constraints as explicit edges over global ranks, (src << 32 | dst): the transitive reduction of its key
 * chains (CommandsForKey.notifyManaged's Read/Write rule, CommandsForKey.java:1208-1289) plus its direct /
 * range dependency edges and unmanaged chain bounds (Commands.updateWaitingOn, Commands.java:700-775;
 * Updating.updateUnmanaged, Updating.java:715-800) from the Deps.merge of its own views.  out == NULL: compute
 * and return the count; then again with out[m] to copy them.  Every store gathers every store's edges and
 * solves the union (Kahn wavefronts; deep graphs inside one workgroup): ad_shard_levels_solve from host
 * edges, or ad_shard_levels_gather over RCCL (counts all-gather + grouped send/recv of the edges).  *depth =
 * number of levels.  Then ad_shard_order.  No round count depends on the depth of the graph. */
int  ad_shard_level_edges(ad_handle* h, size_t* m, uint64_t* out);
int  ad_shard_levels_solve(ad_handle* h, const uint64_t* edges, size_t m, uint32_t* depth);
int  ad_shard_levels_gather(ad_handle* h, uint32_t* depth);
/* Distributed Kahn wavefronts (the default for shallow graphs): a txn's level is 1 + the greatest level of its
 * predecessors over the stores holding it (every constraint is local to one store, see above).  Each store sends
 * READY(txn, bound) to every holder of the txn (itself included) once its last local predecessor is released, bound =
 * 1 + the greatest level among them; every holder releases the txn when all holders' READYs are in, at the greatest
 * bound, then decrements its local successors.  Levels ride in the READYs, so a READY may arrive a wave late.  A txn
 * costs holders x holders READYs over the batch (8 bytes each; the store's own by a device copy), and each store
 * touches only its own constraint edges.  Replaces the CommandsForKey.notifyManaged cascade across CommandStores
 * (local/cfk/CommandsForKey.java:1208-1289, local/CommandStores.java:576-593) with the batch's waves.
 *   ad_shard_set_holders, then ad_shard_kahn_begin (the local graph + wave 0's READYs); then either
 *   - ad_shard_kahn_run (RCCL): the whole wave loop with fixed exchange slots of `slot` READYs per (source,
 *     destination) and wave (0: from the queues' capacities, maxed over the stores), no host synchronisation between
 *     waves: every `check_every` waves an all-reduce of the READYs still queued anywhere, read by the host `lag`
 *     checks later; *waves = waves run; AD_ERR_UNSUPPORTED past wave_cap waves (every store together); or
 *   - per wave: exchange (every queued READY; stop when no store sent anything) -> ad_shard_kahn_step (device only;
 *     `level` is not used); over RCCL ad_shard_kahn_exchange (the per-destination counts all-gathered: one host
 *     synchronisation; *any_status = some store sent something; `status` is ignored), over a host transport
 *     ad_shard_kahn_outbox (per-destination counts and messages) -> peers -> ad_shard_kahn_inbox;
 *   then ad_shard_kahn_finish (*unreleased: rows never released, i.e. a cycle), ad_shard_kahn_depth (the greatest
 *   level + 1), ad_shard_order. */
int  ad_shard_kahn_begin(ad_handle* h);
int  ad_shard_kahn_outbox(ad_handle* h, uint32_t* counts /* [world] */, uint64_t* msgs /* or NULL: counts only */);
int  ad_shard_kahn_inbox(ad_handle* h, const uint64_t* msgs, size_t m);
int  ad_shard_kahn_exchange(ad_handle* h, uint32_t status, uint32_t* any_status);
int  ad_shard_kahn_step(ad_handle* h, uint32_t level);
int  ad_shard_kahn_run(ad_handle* h, uint32_t slot, uint32_t check_every, uint32_t lag, uint32_t wave_cap, uint32_t* waves);
int  ad_shard_kahn_finish(ad_handle* h, uint64_t* unreleased);
int  ad_shard_kahn_depth(ad_handle* h, uint32_t* depth);
int  ad_shard_kahn_sent(ad_handle* h, uint64_t* sent);

#ifdef __cplusplus
}
#endif
#endif /* ACCORD_DEPS_H */
