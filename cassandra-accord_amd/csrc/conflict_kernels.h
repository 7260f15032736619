// conflict_kernels.h — the replica's witnessedAt proposal (MaxConflicts) for a key batch (gfx950).
//
// CommandStore.preaccept (local/CommandStore.java:322-347) answers witnessedAt = TxnId when
// TxnId >= maxConflicts.get(keys), else a fresh HLC above it.  MaxConflicts (local/MaxConflicts.java:46-59)
// is a per-key running max of the executeAt of every globally visible txn the store has recorded
// (CommandStore.updateMaxConflicts :282-291, SafeCommandStore.updateMaxConflicts :210-222).  For a batch
// that arrives in TxnId order this is, per (txn i, key) and replica view v, the max executeAt over the
// key's CommandsForKey entries j < i the view holds: out-of-window entries whose final status is recorded
// (category != CAT_SKIP) plus in-flight ones the view did not drop — the same entry set the deps walk
// visits (deps_kernels.h walk_query), without the witness/elision filters.
//
//   MaxConflictOp scan   segmented inclusive prefix max of (executeAt+1, rank) over recorded entries; its
//                        store also inverts the sort permutation (pair -> sorted position)
//   k_mc_txns<NV>        one thread per txn: per pair, the in-flight window walk per view from the pair's
//                        sorted position, then the prefix max of the entry just below the window; max over
//                        the txn's pairs per view, fast-path test (no per-pair intermediate in HBM)
//   k_mc_range_keys<NV>  range-domain txns: the same per CFK key inside their ranges (MaxConflicts is a
//                        ReducingRangeMap: get(ranges) folds every key inside), one wave per txn
//   k_mc_range_entries<NV> every txn vs the batch's range txns: ranges containing one of its keys /
//                        intersecting one of its ranges (the windowed join of k_range_deps), one wave per txn
#pragma once
#include "deps_kernels.h"
#include "range_kernels.h"
#include "union_kernels.h"

namespace ad {

// (executeAt+1, rank) pairs: executeAt+1 = packed ts64 + 1 (0 = Timestamp.NONE), rank = batch row of the txn
// holding it; ordered lexicographically, so equal executeAts go to the larger rank
__device__ inline bool mc_less(uint64_t ae, uint32_t ar, uint64_t be, uint32_t br) {
    return ae < be || (ae == be && ar < br);
}

struct MaxConflictOp {
    struct S {
        uint64_t e;
        uint32_t r;
        uint32_t head;
    };
    const int32_t* seg_start;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const uint32_t* e_txn;
    const uint32_t* sval;      // sorted position -> pair index
    uint64_t* pm_e;
    uint32_t* pm_r;
    uint32_t* inv;             // pair index -> sorted position

    __device__ S load(size_t i) const {
        const uint32_t m = e_meta[i];
        const bool rec = category(m) != CAT_SKIP;
        return S{rec ? e_exec1[i] : 0ull, rec ? e_txn[i] : 0u, seg_start[i] == (int32_t)i ? 1u : 0u};
    }
    __device__ S identity() const { return S{0ull, 0u, 0u}; }
    __device__ S combine(const S& a, const S& b) const {
        if (b.head) return S{b.e, b.r, 1u};
        const bool lt = mc_less(a.e, a.r, b.e, b.r);
        return S{lt ? b.e : a.e, lt ? b.r : a.r, a.head};
    }
    __device__ void store(size_t i, const S&, const S& inc, const S&) const {
        pm_e[i] = inc.e;
        pm_r[i] = inc.r;
        inv[sval[i]] = (uint32_t)i;
    }
};

struct McArgs {
    size_t n, P;
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const int32_t* seg_start;
    const uint32_t* inv;       // pair index -> sorted position
    const uint32_t* gid;       // sharded batches: local row -> global arrival rank (nullable)
    const uint64_t* pm_e;
    const uint32_t* pm_r;
    uint32_t window, thresh;
    uint64_t seed;
    const uint32_t* key_off;
    const uint64_t* tx_ts;
    uint32_t* max_rank;        // [v * n + t]
    uint8_t* fast;             // [v * n + t]
    uint32_t* local_rank;      // [v * n + t] the batch row holding the max (AD_RANK_NONE), or nullptr
};

template <int NV>
static __global__ __launch_bounds__(256) void k_mc_txns(McArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t gi = a.gid ? a.gid[t] : (uint32_t)t;
    const uint32_t lo = a.window == 0 ? gi : (gi > a.window ? gi - a.window : 0u);
    uint64_t be[NV];
    uint32_t br[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) { be[v] = 0; br[v] = 0; }
    for (uint32_t p = a.key_off[t]; p < a.key_off[t + 1]; ++p) {
        const int s = (int)a.inv[p];
        const int seg0 = a.seg_start[s];
        // in-flight window [i - W, i): recorded as PreAccepted by every view that did not drop it
        int q = s - 1;
        for (; q >= seg0; --q) {
            const uint32_t j = a.e_txn[q];
            const uint32_t gj = a.gid ? a.gid[j] : j;
            if (gj < lo) break;
            if (!manages(a.e_meta[q])) continue;
            const uint64_t e = a.e_exec1[q];
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (!(a.thresh && drop_hash(a.seed, (uint32_t)v, gi, gj) < a.thresh) && mc_less(be[v], br[v], e, j)) {
                    be[v] = e; br[v] = j;
                }
        }
        // recorded prefix [seg0, q]: one segmented-scan value, identical for every view
        if (q >= seg0) {
            const uint64_t e = a.pm_e[q];
            const uint32_t r = a.pm_r[q];
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (mc_less(be[v], br[v], e, r)) { be[v] = e; br[v] = r; }
        }
    }
    const uint64_t t1 = a.tx_ts[t] + 1;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        // sharded stores answer in global arrival ranks (ascending with local rows: the tie rule is kept)
        a.max_rank[(size_t)v * a.n + t] = be[v] ? (a.gid ? a.gid[br[v]] : br[v]) : AD_RANK_NONE;
        if (a.local_rank) a.local_rank[(size_t)v * a.n + t] = be[v] ? br[v] : AD_RANK_NONE;
        a.fast[(size_t)v * a.n + t] = (be[v] == 0 || t1 >= be[v]) ? 1 : 0;   // TxnId.compareTo(max) >= 0
    }
}

// ---- range footprints ---------------------------------------------------------------------------------------
struct McRangeArgs {
    size_t n;
    const uint8_t* meta;
    const uint64_t* ex1;       // [n] executeAt + 1 (packed)
    const uint64_t* tx_ts;     // [n] packed TxnId
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint32_t* range_off;
    const uint64_t* rs;
    const uint64_t* re;
    // CFK entries (k_mc_range_keys)
    const uint64_t* ukey;
    const uint32_t* useg;
    uint32_t U;
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const uint64_t* pm_e;
    const uint32_t* pm_r;
    // range entries sorted by (start, end, owner) (k_mc_range_entries)
    size_t Q;
    const uint64_t* es;
    const uint64_t* ee;
    const uint32_t* eown;
    RangeIndex ix;
    uint32_t window, thresh;
    uint64_t seed;
    uint32_t* max_rank;        // [v * n + t] batch rows, folded in place (sharded: the local-row answers,
                               // turned into global ranks by k_mc_globalize afterwards)
    uint8_t* fast;
    const uint32_t* gid;       // sharded stores: local row -> global arrival rank (window, drops; nullable)
};

// sharded stores: the folded local-row answers -> global ranks
static __global__ __launch_bounds__(256) void k_mc_globalize(size_t m, const uint32_t* __restrict__ local,
                                                      const uint32_t* __restrict__ gid, uint32_t* __restrict__ rank) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < m) rank[x] = local[x] == AD_RANK_NONE ? AD_RANK_NONE : gid[local[x]];
}

// wave max of (e, r) per view; lane 0 folds it into the txn's answer and redoes the fast-path test
template <int NV>
__device__ inline void mc_fold_wave(const McRangeArgs& a, size_t t, uint64_t* be, uint32_t* br) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        uint64_t e = be[v];
        uint32_t r = br[v];
#pragma unroll
        for (int o = WAVE / 2; o > 0; o >>= 1) {
            const uint64_t e2 = __shfl_xor(e, o);
            const uint32_t r2 = __shfl_xor(r, o);
            if (mc_less(e, r, e2, r2)) { e = e2; r = r2; }
        }
        if (__lane_id() == 0 && e != 0) {
            const size_t x = (size_t)v * a.n + t;
            const uint32_t cur = a.max_rank[x];
            const uint64_t ce = cur == AD_RANK_NONE ? 0ull : a.ex1[cur];
            if (cur == AD_RANK_NONE || mc_less(ce, cur, e, r)) {
                a.max_rank[x] = r;
                a.fast[x] = a.tx_ts[t] + 1 >= e ? 1 : 0;          // TxnId.compareTo(max) >= 0
            }
        }
    }
}

template <int NV>
static __global__ __launch_bounds__(256) void k_mc_range_keys(McRangeArgs a) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n || meta_domain(a.meta[t]) != AD_DOMAIN_RANGE) return;
    const uint32_t gi = a.gid ? a.gid[t] : (uint32_t)t;     // window and drops: global arrival ranks
    const uint32_t lo_w = a.window == 0 ? gi : (gi > a.window ? gi - a.window : 0u);
    uint64_t be[NV];
    uint32_t br[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) { be[v] = 0; br[v] = 0; }
    for (uint32_t q = a.range_off[t]; q < a.range_off[t + 1]; ++q) {
        // CFK keys inside (start, end]
        const uint32_t ulo = ub_u64(a.ukey, 0, a.U, a.rs[q]), uhi = ub_u64(a.ukey, ulo, a.U, a.re[q]);
        for (uint32_t u = ulo + __lane_id(); u < uhi; u += WAVE) {
            const int s0 = (int)a.useg[u];
            const int pos = (int)ub_u32(a.e_txn, a.useg[u], a.useg[u + 1], (uint32_t)t);   // insertPos(TxnId t)
            int x = pos - 1;
            for (; x >= s0; --x) {                 // in-flight window: per view unless dropped
                const uint32_t j = a.e_txn[x];
                const uint32_t gj = a.gid ? a.gid[j] : j;
                if (gj < lo_w) break;
                if (!manages(a.e_meta[x])) continue;
                const uint64_t e = a.e_exec1[x];
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    if (!(a.thresh && drop_hash(a.seed, (uint32_t)v, gi, gj) < a.thresh) && mc_less(be[v], br[v], e, j)) {
                        be[v] = e; br[v] = j;
                    }
            }
            if (x >= s0) {                         // recorded prefix: one scan value for every view
                const uint64_t e = a.pm_e[x];
                const uint32_t r = a.pm_r[x];
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    if (mc_less(be[v], br[v], e, r)) { be[v] = e; br[v] = r; }
            }
        }
    }
    mc_fold_wave<NV>(a, t, be, br);
}

template <int NV>
static __global__ __launch_bounds__(256) void k_mc_range_entries(McRangeArgs a) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n) return;
    const uint32_t i = (uint32_t)t;
    const bool key_dom = meta_domain(a.meta[i]) == AD_DOMAIN_KEY;
    const uint32_t fb = key_dom ? a.key_off[i] : a.range_off[i];
    const uint32_t fe = key_dom ? a.key_off[i + 1] : a.range_off[i + 1];
    const uint32_t gi = a.gid ? a.gid[i] : i;
    const uint32_t lo_w = a.window == 0 ? gi : (gi > a.window ? gi - a.window : 0u);
    const uint32_t Q = (uint32_t)a.Q;
    uint64_t be[NV];
    uint32_t br[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) { be[v] = 0; br[v] = 0; }
    ri_walk(a.ix, a.es, Q, key_dom, a.keys, a.rs, a.re, fb, fe, [&](uint32_t clo, uint32_t chi) {
        const uint32_t x = clo + __lane_id();
        if (x >= chi) return;
        const uint32_t j = a.eown[x];
        if (j >= i) return;
        const uint32_t mj = a.meta[j];
        const uint32_t kj = meta_kind(mj);
        if (!(kj == AD_KIND_READ || kj == AD_KIND_WRITE || kj == AD_KIND_SYNC_POINT || kj == AD_KIND_EXCLUSIVE_SYNC_POINT))
            return;                                // globally visible kinds only
        // the chunk can hold entries of no footprint element: the exact intersection test
        RangeArgs ra{};
        ra.keys = a.keys; ra.rs = a.rs; ra.re = a.re;
        if (!range_hits(ra, key_dom, fb, fe, a.es[x], a.ee[x])) return;
        const uint32_t gj = a.gid ? a.gid[j] : j;
        const bool inw = gj >= lo_w;
        const uint32_t st = meta_status(mj);
        if (!inw && (st == AD_ST_TRANSITIVELY_KNOWN || st == AD_ST_INVALID)) return;
        const uint64_t ej = a.ex1[j];
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (!(inw && a.thresh && drop_hash(a.seed, (uint32_t)v, gi, gj) < a.thresh) && mc_less(be[v], br[v], ej, j)) {
                be[v] = ej; br[v] = j;
            }
    });
    mc_fold_wave<NV>(a, t, be, br);
}

// ---- MaxConflicts carried across batches (the store's state from its earlier batches) ----------------------
// A store's MaxConflicts map outlives a batch.  The host passes it in as a sorted table (key -> greatest
// executeAt recorded), the witnessedAt inputs then fold it in as timestamps, and the table after the batch is
// exported for the next one.  Timestamps are raw (msb, lsb, node) here: a carried value need not fit the
// batch's packed ts64 range.
struct Ts3 { uint64_t msb, lsb; int32_t node; };
__device__ inline int ts3_cmp(const Ts3& a, const Ts3& b) {          // Timestamp.compareTo (:208-217)
    if (a.msb != b.msb) return a.msb < b.msb ? -1 : 1;
    const uint64_t ah = a.lsb >> 16, bh = b.lsb >> 16;
    if (ah != bh) return ah < bh ? -1 : 1;
    const uint32_t af = (uint32_t)(a.lsb & 0x1E), bf = (uint32_t)(b.lsb & 0x1E);
    if (af != bf) return af < bf ? -1 : 1;
    return a.node < b.node ? -1 : (a.node > b.node ? 1 : 0);
}
// The range part of the carried map (round 3): sorted disjoint intervals (s, e] with a Timestamp each.  A key k
// is the interval (k - 1, k] (Range.EndInclusive over the order-preserving u64 keys), so the point table and the
// interval table together are the reference's ReducingRangeMap (MaxConflicts extends ReducingRangeMap<Timestamp>,
// local/MaxConflicts.java:32-59): get(keys or ranges) folds max over every point and interval the footprint meets;
// update(footprint, executeAt) merges a piece per key / range (ReducingIntervalMap.merge with Timestamp::max).
struct McIntervals {
    size_t m;
    const uint64_t *s, *e, *cm, *cl;
    const int32_t* cn;
};
// Timestamp::max; of two that compare equal the larger raw lsb (a total order: the fold is order-independent).
// Deliberate divergence, documented in DESIGN.md §7: the reference keeps the folded value on a tie in get
// (foldl(.., Timestamp::max, ..) = max(value, acc)) and the existing map's value in merge, i.e. the survivor of a
// tie depends on the fold order.  compareTo-equal timestamps of DIFFERENT txns cannot occur (compareTo covers the
// identity bits epoch, hlc, kind flags, node: Timestamp.java:208-217), so a tie is one txn's timestamp seen twice
// and only bits outside compareTo (domain bit 0, REJECTED 0x8000) can differ — those this rule may pick otherwise.
__device__ inline void ts3_fold(const Ts3& c, Ts3& best, bool& has) {
    const int d = has ? ts3_cmp(c, best) : 1;
    if (d > 0 || (d == 0 && c.lsb > best.lsb)) { best = c; has = true; }
}
// a range txn the store records in MaxConflicts: globally visible kind, not TRANSITIVELY_KNOWN / INVALID
__device__ inline bool mc_range_recorded(uint32_t m) {
    const uint32_t k = meta_kind(m), st = meta_status(m);
    return (k == AD_KIND_READ || k == AD_KIND_WRITE || k == AD_KIND_SYNC_POINT || k == AD_KIND_EXCLUSIVE_SYNC_POINT) &&
           st != AD_ST_TRANSITIVELY_KNOWN && st != AD_ST_INVALID;
}
// the interval containing key k (s < k <= e): the first interval with e >= k
__device__ inline void mci_stab(const McIntervals& r, uint64_t k, Ts3& best, bool& has) {
    size_t lo = 0, hi = r.m;
    while (lo < hi) { const size_t mid = (lo + hi) >> 1; if (r.e[mid] < k) lo = mid + 1; else hi = mid; }
    if (lo < r.m && r.s[lo] < k) ts3_fold(Ts3{r.cm[lo], r.cl[lo], r.cn[lo]}, best, has);
}
// every interval meeting (qs, qe]: from the first with e > qs while s < qe
__device__ inline void mci_span(const McIntervals& r, uint64_t qs, uint64_t qe, Ts3& best, bool& has) {
    size_t lo = 0, hi = r.m;
    while (lo < hi) { const size_t mid = (lo + hi) >> 1; if (r.e[mid] <= qs) lo = mid + 1; else hi = mid; }
    for (size_t x = lo; x < r.m && r.s[x] < qe; ++x) ts3_fold(Ts3{r.cm[x], r.cl[x], r.cn[x]}, best, has);
}

struct McCarryArgs {
    size_t n;
    int nv;
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint32_t* range_off;               // range txns' footprints (nullable: a key batch)
    const uint64_t *rs, *re;
    McIntervals iv;                          // the carried intervals
    const uint64_t *tm, *tl, *em, *el;       // batch TxnId / executeAt
    const int32_t *tn, *en;
    const uint32_t* local_rank;              // [v * n + t]
    size_t m;                                 // carry table
    const uint64_t *ck, *cm, *cl;
    const int32_t* cn;
    uint64_t *om, *ol;                       // [v * n + t] maxConflicts.get(keys) as a timestamp (NONE = 0, 0, 0)
    int32_t* on;
    uint8_t* fast;                           // [v * n + t]
};
static __global__ __launch_bounds__(256) void k_mc_carry(McCarryArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    Ts3 cb{0, 0, 0};
    bool has = false;
    for (uint32_t p = a.key_off[t]; p < a.key_off[t + 1]; ++p) {
        const uint64_t k = a.keys[p];
        if (a.m) {
            size_t lo = 0, hi = a.m;
            while (lo < hi) { const size_t mid = (lo + hi) >> 1; if (a.ck[mid] < k) lo = mid + 1; else hi = mid; }
            if (lo < a.m && a.ck[lo] == k) ts3_fold(Ts3{a.cm[lo], a.cl[lo], a.cn[lo]}, cb, has);
        }
        if (a.iv.m) mci_stab(a.iv, k, cb, has);
    }
    if (a.range_off) {
        // a range footprint: every carried point inside (qs, qe] and every carried interval meeting it
        for (uint32_t q = a.range_off[t]; q < a.range_off[t + 1]; ++q) {
            const uint64_t qs = a.rs[q], qe = a.re[q];
            size_t lo = 0, hi = a.m;
            while (lo < hi) { const size_t mid = (lo + hi) >> 1; if (a.ck[mid] <= qs) lo = mid + 1; else hi = mid; }
            for (size_t x = lo; x < a.m && a.ck[x] <= qe; ++x) ts3_fold(Ts3{a.cm[x], a.cl[x], a.cn[x]}, cb, has);
            if (a.iv.m) mci_span(a.iv, qs, qe, cb, has);
        }
    }
    const Ts3 me{a.tm[t], a.tl[t], a.tn[t]};
    for (int v = 0; v < a.nv; ++v) {
        const size_t o = (size_t)v * a.n + t;
        const uint32_t r = a.local_rank[o];
        Ts3 best = cb;
        bool any = has;
        if (r != AD_RANK_NONE) {
            const Ts3 b{a.em[r], a.el[r], a.en[r]};
            if (!any || ts3_cmp(b, best) > 0) { best = b; any = true; }
        }
        a.om[o] = any ? best.msb : 0ull;
        a.ol[o] = any ? best.lsb : 0ull;
        a.on[o] = any ? best.node : 0;
        a.fast[o] = (!any || ts3_cmp(me, best) >= 0) ? 1 : 0;               // TxnId.compareTo(max) >= 0
    }
}
// The rest of CommandStore.preaccept (local/CommandStore.java:322-347) around maxConflicts.get, as a pass over the
// fast flags either max-conflicts path left ([v * n + t]; the same store state answers every view):
//   isExpired = now - TxnId.hlc >= preAcceptTimeout && !kind.isSyncPoint          (:326)
//            || rejectBefore.foldl(keys, rejectIfBefore > TxnId -> reject)         (:327-328)
//   expired  -> time.uniqueNow(TxnId).asRejected(): fast = AD_FAST_REJECTED          (:330-331)
//   ExclusiveSyncPoint -> TxnId unconditionally (markExclusiveSyncPoint): fast = 1   (:333-337)
// rejectBefore is a ReducingRangeMap<Timestamp> (the greatest ExclusiveSyncPoint TxnId marked over each range,
// markExclusiveSyncPoint :300-306), carried as sorted disjoint intervals (s, e]; a key stabs (k - 1, k].
struct PreacceptRules {
    size_t n;
    int nv;
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint32_t* range_off;               // nullable: a key batch
    const uint64_t *rs, *re;
    const uint64_t *tm, *tl;
    const int32_t* tn;                       // TxnId node: compareTo's last tiebreak (Timestamp.java:208-217)
    McIntervals rb;                          // rejectBefore
    int clock;                               // the timeout test applies
    uint64_t now_hlc, timeout;
    uint8_t* fast;
};
static __global__ __launch_bounds__(256) void k_preaccept_rules(PreacceptRules a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint64_t msb = a.tm[t], lsb = a.tl[t];
    const uint32_t kind = (uint32_t)(lsb >> 1) & 7u;
    const bool sync_point = kind == AD_KIND_SYNC_POINT || kind == AD_KIND_EXCLUSIVE_SYNC_POINT;
    const uint64_t hlc = ((msb & 0x7FFFull) << 48) | (lsb >> 16);
    bool expired = a.clock && !sync_point && (int64_t)(a.now_hlc - hlc) >= (int64_t)a.timeout;
    if (!expired && a.rb.m) {
        Ts3 rb{0, 0, 0};
        bool has = false;
        for (uint32_t p = a.key_off[t]; p < a.key_off[t + 1]; ++p) mci_stab(a.rb, a.keys[p], rb, has);
        if (a.range_off)
            for (uint32_t q = a.range_off[t]; q < a.range_off[t + 1]; ++q) mci_span(a.rb, a.rs[q], a.re[q], rb, has);
        // any rejectIfBefore > TxnId rejects: the max over the footprint decides
        expired = has && ts3_cmp(rb, Ts3{msb, lsb, a.tn[t]}) > 0;   // the real TxnId (CommandStore.java:328)
    }
    if (!expired && kind != AD_KIND_EXCLUSIVE_SYNC_POINT) return;
    for (int v = 0; v < a.nv; ++v) a.fast[(size_t)v * a.n + t] = expired ? AD_FAST_REJECTED : 1;
}

// Export: the union of the carry table and the batch's per-key maxima (the recorded-entry prefix max at each
// key segment's end), merged by key ranks into slots with gaps (a key in both lands on one slot), then
// compacted.  slot[i] of a batch key = i + #carry keys below it; of a carry key = j + #batch keys below it.
static __global__ __launch_bounds__(256) void k_mc_export_slots(uint32_t U, const uint64_t* __restrict__ ukey, const uint32_t* __restrict__ useg,
                                                         const uint64_t* __restrict__ pm_e, const uint32_t* __restrict__ pm_r,
                                                         const uint64_t* __restrict__ em, const uint64_t* __restrict__ el,
                                                         const int32_t* __restrict__ en, size_t m, const uint64_t* __restrict__ ck,
                                                         const uint64_t* __restrict__ cm, const uint64_t* __restrict__ cl,
                                                         const int32_t* __restrict__ cn, uint64_t* __restrict__ sk,
                                                         uint64_t* __restrict__ sm, uint64_t* __restrict__ sl,
                                                         int32_t* __restrict__ sn, uint8_t* __restrict__ used) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < U) {
        const uint64_t k = ukey[i];
        size_t lo = 0, hi = m;
        while (lo < hi) { const size_t mid = (lo + hi) >> 1; if (ck[mid] < k) lo = mid + 1; else hi = mid; }
        const size_t slot = i + lo;
        const uint32_t last = useg[i + 1] - 1;                       // the segment's last entry: prefix max of all
        Ts3 b{0, 0, 0};
        bool any = pm_e[last] != 0;
        if (any) { const uint32_t r = pm_r[last]; b = Ts3{em[r], el[r], en[r]}; }
        if (lo < m && ck[lo] == k) {
            const Ts3 c{cm[lo], cl[lo], cn[lo]};
            if (!any || ts3_cmp(c, b) > 0) { b = c; any = true; }
        }
        sk[slot] = k; sm[slot] = b.msb; sl[slot] = b.lsb; sn[slot] = b.node;
        used[slot] = any ? 1 : 0;                                     // a key with nothing recorded stays out
    } else if (i < U + m) {
        const size_t j = i - U;
        const uint64_t k = ck[j];
        size_t lo = 0, hi = U;
        while (lo < hi) { const size_t mid = (lo + hi) >> 1; if (ukey[mid] < k) lo = mid + 1; else hi = mid; }
        if (lo < U && ukey[lo] == k) return;                          // written by the batch key's thread
        const size_t slot = j + lo;
        sk[slot] = k; sm[slot] = cm[j]; sl[slot] = cl[j]; sn[slot] = cn[j];
        used[slot] = 1;
    }
}
// CompactFlagOp gives out[k] = the k-th used slot: gather them in slot (= key) order
static __global__ __launch_bounds__(256) void k_mc_export_gather(uint32_t count, const uint32_t* __restrict__ slot,
                                                          const uint64_t* __restrict__ sk, const uint64_t* __restrict__ sm,
                                                          const uint64_t* __restrict__ sl, const int32_t* __restrict__ sn,
                                                          uint64_t* __restrict__ ok, uint64_t* __restrict__ om,
                                                          uint64_t* __restrict__ ol, int32_t* __restrict__ on) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    const uint32_t i = slot[k];
    ok[k] = sk[i]; om[k] = sm[i]; ol[k] = sl[i]; on[k] = sn[i];
}

// ---- export of the interval part: the piecewise max of the carried intervals and the batch's range txns ------
// Breakpoints X = every interval endpoint (carried and batch), sorted and unique; the elementary segments
// (X[g], X[g+1]] each take the max of the carried interval and the batch range entries (recorded owners: status not
// TRANSITIVELY_KNOWN / INVALID, as the key scan) that contain X[g+1]; runs of equal values are merged into one
// interval and empty segments dropped (ReducingIntervalMap's normal form).
static __global__ __launch_bounds__(256) void k_mci_points(size_t m, const uint64_t* __restrict__ cs, const uint64_t* __restrict__ ce,
                                                    size_t Q, const uint64_t* __restrict__ rs, const uint64_t* __restrict__ re,
                                                    uint64_t base, uint64_t* __restrict__ x, uint32_t* __restrict__ lo32,
                                                    uint32_t* __restrict__ idx) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t N = 2 * (m + Q);
    if (i >= N) return;
    const size_t j = i >> 1;
    const uint64_t v = j < m ? ((i & 1) ? ce[j] : cs[j]) : ((i & 1) ? re[j - m] : rs[j - m]);
    x[i] = v;
    lo32[i] = (uint32_t)(v - base);
    idx[i] = (uint32_t)i;
}
// second LSD pass over a spread beyond 32 bits: the high halves of the points in their current order
static __global__ __launch_bounds__(256) void k_mci_hi(size_t N, const uint64_t* __restrict__ x, const uint32_t* __restrict__ idx,
                                                uint64_t base, uint32_t* __restrict__ hi32) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) hi32[i] = (uint32_t)((x[idx[i]] - base) >> 32);
}
// unique flags of the sorted points
static __global__ __launch_bounds__(256) void k_mci_unique(size_t N, const uint64_t* __restrict__ x, const uint32_t* __restrict__ idx,
                                                    uint8_t* __restrict__ first) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) first[i] = (i == 0 || x[idx[i]] != x[idx[i - 1]]) ? 1 : 0;
}
static __global__ __launch_bounds__(256) void k_mci_gather_points(uint32_t S, const uint32_t* __restrict__ rows, const uint64_t* __restrict__ x,
                                                           const uint32_t* __restrict__ idx, uint64_t* __restrict__ xu) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < S) xu[k] = x[idx[rows[k]]];
}
struct MciSegArgs {
    uint32_t S;                              // unique breakpoints; segments g = 0 .. S-2
    const uint64_t* xu;
    McIntervals iv;
    size_t Q;                                // batch range entries sorted by (start, end, owner) + their index
    const uint64_t *es, *ee;
    const uint32_t* eown;
    RangeIndex ix;
    const uint8_t* meta;                     // owners' meta (recorded?) and raw executeAt
    const uint64_t *em, *el;
    const int32_t* en;
    uint64_t *vm, *vl;                       // [S] segment values (vm = vl = 0, vn = 0 and has = 0: none)
    int32_t* vn;
    uint8_t* has;
};
// one wave per segment: the carried interval and the batch entries containing y = X[g + 1]
static __global__ __launch_bounds__(256) void k_mci_segments(MciSegArgs a) {
    const size_t g = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (g + 1 >= a.S) return;
    const int lane = __lane_id();
    const uint64_t y = a.xu[g + 1];
    Ts3 best{0, 0, 0};
    bool any = false;
    if (a.Q) {
        ri_walk(a.ix, a.es, (uint32_t)a.Q, true, a.xu, nullptr, nullptr, (uint32_t)(g + 1), (uint32_t)(g + 2),
                [&](uint32_t clo, uint32_t chi) {
            const uint32_t x = clo + (uint32_t)lane;
            if (x < chi && a.es[x] < y && a.ee[x] >= y) {
                const uint32_t j = a.eown[x];
                if (mc_range_recorded(a.meta[j])) ts3_fold(Ts3{a.em[j], a.el[j], a.en[j]}, best, any);
            }
        });
        // the wave's max
#pragma unroll
        for (int o = WAVE / 2; o > 0; o >>= 1) {
            const Ts3 c{__shfl_xor(best.msb, o), __shfl_xor(best.lsb, o), __shfl_xor(best.node, o)};
            const bool ca = __shfl_xor((int)any, o) != 0;
            if (ca) ts3_fold(c, best, any);
        }
    }
    if (lane != 0) return;
    if (a.iv.m) mci_stab(a.iv, y, best, any);
    a.vm[g] = any ? best.msb : 0ull;
    a.vl[g] = any ? best.lsb : 0ull;
    a.vn[g] = any ? best.node : 0;
    a.has[g] = any ? 1 : 0;
}
// piece starts / ends: a segment with a value whose neighbour has no value or another one
static __global__ __launch_bounds__(256) void k_mci_pieces(uint32_t nseg, const uint64_t* __restrict__ vm, const uint64_t* __restrict__ vl,
                                                    const int32_t* __restrict__ vn, const uint8_t* __restrict__ has,
                                                    uint8_t* __restrict__ start, uint8_t* __restrict__ end) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg) return;
    auto same = [&](uint32_t a, uint32_t b) { return has[a] && has[b] && vm[a] == vm[b] && vl[a] == vl[b] && vn[a] == vn[b]; };
    start[g] = (has[g] && !(g > 0 && same(g - 1, g))) ? 1 : 0;
    end[g] = (has[g] && !(g + 1 < nseg && same(g, g + 1))) ? 1 : 0;
}
static __global__ __launch_bounds__(256) void k_mci_emit(uint32_t cnt, const uint32_t* __restrict__ starts, const uint32_t* __restrict__ ends,
                                                  const uint64_t* __restrict__ xu, const uint64_t* __restrict__ vm,
                                                  const uint64_t* __restrict__ vl, const int32_t* __restrict__ vn,
                                                  uint64_t* __restrict__ os, uint64_t* __restrict__ oe, uint64_t* __restrict__ om,
                                                  uint64_t* __restrict__ ol, int32_t* __restrict__ on) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= cnt) return;
    const uint32_t g0 = starts[k], g1 = ends[k];
    os[k] = xu[g0]; oe[k] = xu[g1 + 1]; om[k] = vm[g0]; ol[k] = vl[g0]; on[k] = vn[g0];
}

}  // namespace ad
