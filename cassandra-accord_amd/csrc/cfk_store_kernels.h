// cfk_store_kernels.h — device-resident CommandsForKey states: byId TxnInfos and their missing()
// arrays maintained on the device from a stream of CommandsForKey.update events.
//
// One store = K keys, each with up to `cap` TxnInfo rows.  Per key, in HBM:
//   rows in byId order (TxnId strictly ascending): TxnId (msb, lsb, node), executeAt, InternalStatus, and the row's
//   slot (its insertion index: slots never move, rows shift on insert);
//   per slot a bitmap of `words` u64 over slots: TxnInfo.missing() (CommandsForKey.java:101-113) -- bit s set when
//   the txn in slot s is missing from this row's dependencies.
// The reference keeps `missing` as sorted TxnId[] per TxnInfo and rebuilds arrays copy-on-write per update
// (Updating.insertOrUpdate, local/cfk/Updating.java:99-358; Utils.addToMissingArrays / removeFromMissingArrays
// :70-172).  Here every update is applied in place by one workgroup per key, the missing sets as bit columns: adding a
// newly known undecided txn to every row that witnesses it is one bit per row, removing a txn that committed one bit
// per row, and a row's own missing set (its witnessed undecided TxnIds below depsKnownBefore that its deps lack) is
// built in LDS by the workgroup in one pass over the key's rows.
// Events of one key are applied in order by its workgroup (the reference's per-key sequence of updates); keys run in
// parallel.  The release rule then runs over these rows (k_cfk_notify with the bitmap reader, notify_kernels.h).
// Pruning (local/cfk/Pruning.java): per key prunedBefore's TxnId and the loadingPruned table -- per entry a TxnId and its
// witnessedBy as a bitmap over slots (a witness that is not a row of the key is never read: isWaitingOnPruned asks about
// rows, addToMissingArrays skips rows).  A PRUNE event runs maybePrune / pruneBefore in the workgroup: the candidate
// prune point from order statistics over the committed rows (no committedByExecuteAt array is kept), pruneBefore's
// sequential byId scan with the merged missing() set in LDS, then the rows, their slots and every bitmap are compacted
// (a removed row is Applied or invalidated, so no missing() bit names it).
#pragma once
#include "notify_kernels.h"

namespace ad {

// One wave per key: the per-event folds (maxAppliedWrite, minUndecided, the prune point, ...) are wave reductions with
// no workgroup barrier (a 256-thread fold was ~10 barriers; an event ran ~4 of them: ~9.4 us per event on the hottest
// key's serial chain with the rows already in LDS)
constexpr int CS_T = 64;
constexpr uint32_t CS_MAX_WORDS = NF_MAX_WORDS; // capacity <= 8192 rows per key

struct CfkStoreArgs {
    uint32_t K, cap, words;
    uint32_t* cnt;                            // [K] rows per key
    uint64_t *tm, *tl, *em, *el;              // [K * cap] byId rows
    int32_t *tn, *en;
    uint8_t* st;
    uint32_t* slot;                           // [K * cap] the row's slot
    uint64_t* bits;                           // [(K * cap) * words] missing bitmap of each slot
    // events, grouped by key: key k's are [ev_off[k], ev_off[k + 1])
    const uint32_t* ev_off;
    const uint64_t *etm, *etl, *eem, *eel;
    const int32_t *etn, *een;
    const uint8_t* est;
    const uint32_t* dep_off;                  // [m + 1] the command's deps at this key, TxnId ascending
    const uint64_t *dtm, *dtl;
    const int32_t* dtn;
    uint32_t* overflow;                       // a key ran out of rows
    uint32_t* bad;                            // an event's deps not strictly ascending
    // pruning state
    uint64_t *pbm, *pbl;                      // [K] prunedBefore's TxnId (TxnId.NONE: zeros)
    int32_t* pbn;
    uint32_t* lp_cnt;                         // [K] loadingPruned entries
    uint64_t *lpm, *lpl;                      // [K * cap] their TxnIds
    int32_t* lpn;
    uint64_t* lp_bits;                        // [(K * cap) * words] their witnesses
    uint64_t *lp_xm, *lp_xl;                  // [K * cap] each entry's least witness TxnId, rows or not
    int32_t* lp_xn;                           //   (isAnyPredecessorWaitingOnPruned reads witnessedBy's first)
    uint8_t* lp_xh;
    const uint8_t* eop;                       // [m] event op (CS_OP_*; nullptr: every event an UPDATE)
    // unmanaged registry (CommandsForKey.unmanageds, sorted by Unmanaged.compareTo: pending, waitingUntil, txnId)
    uint32_t* um_cnt;                         // [K]
    uint8_t* um_p;                            // [K * cap] COMMIT (0) / APPLY (1)
    uint64_t *um_wm, *um_wl, *um_tm, *um_tl;
    int32_t *um_wn, *um_tn;
    // this call's unmanaged notifications, key k's at nt_base[k]: (event, tag, TxnId) in order; tag 0 =
    // NotifyUnmanagedOfCommit, 1 = NotifyNotWaiting (applied), 2 = registerUnmanaged / updateUnmanaged found it ready
    const uint32_t* nt_base;
    uint32_t* nt_cnt;                         // [K]
    uint32_t* nt_ev;
    uint8_t* nt_tag;
    uint64_t *nt_tm, *nt_tl;
    int32_t* nt_tn;
    uint64_t* dbg;                            // AD_CS_TIMERS=1: per op class clock64 sums and counts (else nullptr)
    // two tiers (cs_tier): keys outgrowing `cap` rows move to a large-tier slot of capB rows (k_cfk_promote)
    uint32_t* kslot;                          // [K] large-tier slot or ~0u
    uint32_t capB, wordsB, nbig;
    uint32_t* big_used;                       // large-tier slots taken
    const uint32_t* ev_start;                 // [K] first event to apply per key (nullptr: ev_off[key]); a resumed key
                                              //   keeps this call's notifications (nt_cnt not reset)
    uint32_t* kres;                           // [K] out: the event a key stopped at for want of rows (~0u: none)
    const uint32_t* klist;                    // the keys of this launch, one workgroup each (nullptr: every key)
    // the workgroup's view of its key (k_cfk_apply): bitmaps at bbase (LDS copy: 0), the HBM regions of its
    // loadingPruned / registry rows (grbase) and their witness bitmaps (gbbase); cap / words = its tier's
    size_t bbase, grbase, gbbase;
};
// event ops (ad_cfk_events.op)
constexpr uint32_t CS_OP_UPDATE = 0;         // CommandsForKey.update (or insertAdditionsOnly: status TRANSITIVELY_KNOWN)
constexpr uint32_t CS_OP_LOAD = 1;           // CommandsForKey.updatePruned of a loaded pruned command
constexpr uint32_t CS_OP_PRUNE = 2;          // maybePrune(exec_node = pruneInterval, exec_msb = minHlcDelta)
constexpr uint32_t CS_OP_LOADING = 3;        // txn joins loadingPruned, witnessed by the event's deps
constexpr uint32_t CS_OP_UNMANAGED = 4;      // registerUnmanaged: Updating.updateUnmanaged(register = true)
constexpr uint32_t CS_OP_UNMANAGED_RECHECK = 5;   // updateUnmanaged(register = false): a notified commit re-checked
constexpr uint32_t UM_COMMIT = 0, UM_APPLY = 1;

__device__ inline bool cs_has_deps(uint32_t s) {            // InternalStatus.hasExecuteAtOrDeps
    return s == AD_ST_ACCEPTED || s == AD_ST_COMMITTED || s == AD_ST_STABLE || s == AD_ST_APPLIED;
}
__device__ inline bool cs_decided(uint32_t s) { return s == AD_ST_COMMITTED || s == AD_ST_STABLE || s == AD_ST_APPLIED; }
__device__ inline uint32_t cs_kind(uint64_t lsb) { return (uint32_t)(lsb >> 1) & 7u; }

// depsKnownBefore (InternalStatus.depsKnownBefore, CommandsForKey.java:561-580): executeAt once committed, else TxnId
__device__ inline Ts3 cs_dkb(const CfkStoreArgs& a, size_t x) {
    return cs_decided(a.st[x]) ? Ts3{a.em[x], a.el[x], a.en[x]} : Ts3{a.tm[x], a.tl[x], a.tn[x]};
}

// Inserts a row at byId position p of key region [base, base + n): rows [p, n) shift up by one, chunk by chunk from
// the top (each chunk is read, then written one slot higher, so no row is overwritten before it moved).
__device__ inline void cs_shift_up(const CfkStoreArgs& a, size_t base, uint32_t p, uint32_t n) {
    for (int top = (int)n; top > (int)p; top -= CS_T) {
        const int i = top - 1 - (int)threadIdx.x;
        const bool act = i >= (int)p;
        uint64_t vtm = 0, vtl = 0, vem = 0, vel = 0;
        int32_t vtn = 0, ven = 0;
        uint8_t vst = 0;
        uint32_t vsl = 0;
        if (act) {
            const size_t x = base + i;
            vtm = a.tm[x]; vtl = a.tl[x]; vtn = a.tn[x]; vem = a.em[x]; vel = a.el[x]; ven = a.en[x];
            vst = a.st[x]; vsl = a.slot[x];
        }
        __syncthreads();
        if (act) {
            const size_t y = base + i + 1;
            a.tm[y] = vtm; a.tl[y] = vtl; a.tn[y] = vtn; a.em[y] = vem; a.el[y] = vel; a.en[y] = ven;
            a.st[y] = vst; a.slot[y] = vsl;
        }
        __syncthreads();
    }
}

// The byId position of t in the key's rows (binary search by every thread: uniform result), found or not.
__device__ inline uint32_t cs_find(const CfkStoreArgs& a, size_t base, uint32_t n, const Ts3& t, bool& found) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (ts3_cmp(Ts3{a.tm[base + m], a.tl[base + m], a.tn[base + m]}, t) < 0) lo = m + 1; else hi = m;
    }
    found = lo < n && ts3_cmp(Ts3{a.tm[base + lo], a.tl[base + lo], a.tn[base + lo]}, t) == 0;
    return lo;
}

// Utils.addToMissingArrays (:97-172): txn `t` (slot ts) joins the missing set of every row that has deps, witnesses
// it and whose depsKnownBefore is above it -- except t itself, `skip` (the command being updated) and the slots set in
// `dont` (a loaded pruned TxnId's witnessedBy, Updating.java:351).
__device__ inline void cs_add_missing(const CfkStoreArgs& a, size_t base, uint32_t n, const Ts3& t, uint32_t ts,
                                      uint32_t skip_slot, const uint64_t* dont = nullptr) {
    const uint32_t kt = cs_kind(t.lsb);
    for (uint32_t r = threadIdx.x; r < n; r += CS_T) {
        const size_t x = base + r;
        const uint32_t s = a.slot[x];
        if (s == ts || s == skip_slot || !cs_has_deps(a.st[x]) || !witnesses(cs_kind(a.tl[x]), kt)) continue;
        if (dont && ((dont[s >> 6] >> (s & 63)) & 1ull)) continue;
        if (ts3_cmp(cs_dkb(a, x), t) > 0) {
            uint64_t* w = a.bits + (a.bbase + (size_t)s * a.words) + (ts >> 6);
            *w |= 1ull << (ts & 63);
        }
    }
    __syncthreads();
}
// Utils.removeFromMissingArrays (:70-95): slot ts leaves every missing set (it committed, or was invalidated)
__device__ inline void cs_remove_missing(const CfkStoreArgs& a, size_t base, uint32_t n, uint32_t ts) {
    for (uint32_t s = threadIdx.x; s < n; s += CS_T) a.bits[(a.bbase + (size_t)s * a.words) + (ts >> 6)] &= ~(1ull << (ts & 63));
    __syncthreads();
}

// A new row at byId position p with a fresh slot (= the key's row count): TxnId t, status, executeAt, empty missing
__device__ inline uint32_t cs_insert(const CfkStoreArgs& a, size_t base, uint32_t& n, uint32_t p, const Ts3& t,
                                     uint32_t status, const Ts3& ex) {
    const uint32_t s = n;
    cs_shift_up(a, base, p, n);
    for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) a.bits[(a.bbase + (size_t)s * a.words) + w] = 0ull;
    if (threadIdx.x == 0) {
        const size_t x = base + p;
        a.tm[x] = t.msb; a.tl[x] = t.lsb; a.tn[x] = t.node;
        a.em[x] = ex.msb; a.el[x] = ex.lsb; a.en[x] = ex.node;
        a.st[x] = (uint8_t)status; a.slot[x] = s;
    }
    __syncthreads();
    ++n;
    return s;
}

// ---- loadingPruned (Pruning.LoadingPruned, Pruning.java:50-114) ----------------------------------------------------
// the entry of TxnId t in key's table, or -1 (TxnIds are unique in the table)
__device__ inline int cs_lp_find(const CfkStoreArgs& a, uint32_t key, uint32_t L, const Ts3& t, int* s_j) {
    if (L == 0) return -1;                                        // (uniform: L is the workgroup's count)
    if (threadIdx.x == 0) *s_j = -1;
    __syncthreads();
    const size_t lb = a.grbase;
    for (uint32_t j = threadIdx.x; j < L; j += CS_T)
        if (ts3_cmp(Ts3{a.lpm[lb + j], a.lpl[lb + j], a.lpn[lb + j]}, t) == 0) *s_j = (int)j;
    __syncthreads();
    const int j = *s_j;
    __syncthreads();
    return j;
}
// Pruning.loadPruned: t joins the table (or is found there) and slot `w` (if any) joins its witnesses, the witness
// TxnId `wt` (if has_wt; a row or not) its least witness; false: full
__device__ inline bool cs_lp_add(const CfkStoreArgs& a, uint32_t key, uint32_t& L, const Ts3& t, uint32_t w, int* s_j,
                                 const Ts3& wt = Ts3{0, 0, 0}, bool has_wt = false) {
    const size_t lb = a.grbase;
    int j = cs_lp_find(a, key, L, t, s_j);
    if (j < 0) {
        if (L >= a.cap) return false;
        j = (int)L++;
        for (uint32_t q = threadIdx.x; q < a.words; q += CS_T) a.lp_bits[a.gbbase + (size_t)j * a.words + q] = 0ull;
        if (threadIdx.x == 0) { a.lpm[lb + j] = t.msb; a.lpl[lb + j] = t.lsb; a.lpn[lb + j] = t.node; a.lp_xh[lb + j] = 0; }
        __syncthreads();
    }
    if (w != 0xFFFFFFFFu && threadIdx.x == 0) a.lp_bits[a.gbbase + (size_t)j * a.words + (w >> 6)] |= 1ull << (w & 63);
    if (has_wt && threadIdx.x == 0) {
        const size_t x = lb + j;
        if (!a.lp_xh[x] || ts3_cmp(wt, Ts3{a.lp_xm[x], a.lp_xl[x], a.lp_xn[x]}) < 0) {
            a.lp_xm[x] = wt.msb; a.lp_xl[x] = wt.lsb; a.lp_xn[x] = wt.node; a.lp_xh[x] = 1;
        }
    }
    __syncthreads();
    return true;
}
// Pruning.removeLoadingPruned: entry j leaves (the last entry takes its place)
__device__ inline void cs_lp_remove(const CfkStoreArgs& a, uint32_t key, uint32_t& L, int j) {
    const size_t lb = a.grbase;
    const uint32_t last = L - 1;
    if ((uint32_t)j != last) {
        for (uint32_t q = threadIdx.x; q < a.words; q += CS_T)
            a.lp_bits[a.gbbase + (size_t)j * a.words + q] = a.lp_bits[a.gbbase + (size_t)last * a.words + q];
        if (threadIdx.x == 0) {
            a.lpm[lb + j] = a.lpm[lb + last]; a.lpl[lb + j] = a.lpl[lb + last]; a.lpn[lb + j] = a.lpn[lb + last];
            a.lp_xm[lb + j] = a.lp_xm[lb + last]; a.lp_xl[lb + j] = a.lp_xl[lb + last]; a.lp_xn[lb + j] = a.lp_xn[lb + last];
            a.lp_xh[lb + j] = a.lp_xh[lb + last];
        }
    }
    --L;
    __syncthreads();
}

// ---- maybePrune / pruneBefore (Pruning.java:164-331) --------------------------------------------------------------
struct CsPruneLds {
    Ts3 v[CS_T];
    int h[CS_T];
    uint32_t c[CS_T];
    uint64_t merged[CS_MAX_WORDS];            // pruneBefore's mergedMissing (slot bitmap)
    uint64_t gone[CS_MAX_WORDS];              // removed rows (byId index bitmap)
    uint64_t dead[CS_MAX_WORDS];              // their slots
    uint32_t gpc[CS_MAX_WORDS], dpc[CS_MAX_WORDS];   // exclusive prefix popcounts of gone / dead per word
    uint64_t stage[CS_T / 64][CS_MAX_WORDS];  // one remapped bitmap row per wave
    uint32_t idx;
};
__device__ inline uint64_t cs_hlc(const Ts3& t) { return ((t.msb & 0x7FFFull) << 48) | (t.lsb >> 16); }
__device__ inline uint32_t cs_block_sum(uint32_t v, uint32_t*) {
    static_assert(CS_T == 64, "one wave per key");
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
    return v;
}
// the block's greatest (MAX) / least TxnId-ordered value among the lanes that have one (every lane gets it)
template <bool MAX>
__device__ inline void cs_fold(Ts3& v, bool& has) {
    static_assert(CS_T == 64, "one wave per key");
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t mh = (uint32_t)__shfl_xor((int)(uint32_t)(v.msb >> 32), o), ml = (uint32_t)__shfl_xor((int)(uint32_t)v.msb, o);
        const uint32_t lh = (uint32_t)__shfl_xor((int)(uint32_t)(v.lsb >> 32), o), ll = (uint32_t)__shfl_xor((int)(uint32_t)v.lsb, o);
        const int nd = __shfl_xor(v.node, o);
        const bool hu = __shfl_xor(has ? 1 : 0, o) != 0;
        const Ts3 u{((uint64_t)mh << 32) | ml, ((uint64_t)lh << 32) | ll, nd};
        if (hu && (!has || (MAX ? ts3_cmp(u, v) > 0 : ts3_cmp(u, v) < 0))) { v = u; has = true; }
    }
}
// bits below position i that are set in bitmap b (with its exclusive per-word prefix counts pc)
__device__ inline uint32_t cs_rank(const uint64_t* b, const uint32_t* pc, uint32_t i) {
    const uint64_t low = (i & 63) ? (b[i >> 6] & ((1ull << (i & 63)) - 1ull)) : 0ull;
    return pc[i >> 6] + (uint32_t)__popcll(low);
}
// old slot row `src` of a bitmap -> its columns compacted (dead columns dropped) into stage (words), one wave
__device__ inline void cs_remap_row(const CfkStoreArgs& a, const uint64_t* src, uint64_t* stage, const CsPruneLds& s,
                                    int lane) {
    for (uint32_t q = lane; q < a.words; q += 64) stage[q] = 0ull;
    __builtin_amdgcn_wave_barrier();
    for (uint32_t q = lane; q < a.words; q += 64) {
        uint64_t x = src[q] & ~s.dead[q];
        while (x) {
            const uint32_t b = (uint32_t)__builtin_ctzll(x);
            x &= x - 1;
            const uint32_t o = q * 64 + b, ns = o - cs_rank(s.dead, s.dpc, o);
            atomicOr((unsigned long long*)&stage[ns >> 6], 1ull << (ns & 63));
        }
    }
    __builtin_amdgcn_wave_barrier();
}

__device__ inline void cs_maybe_prune(const CfkStoreArgs& a, uint32_t key, size_t base, uint32_t& n, uint32_t L,
                                      uint32_t interval, int64_t min_hlc_delta, CsPruneLds& s) {
    const int tid = threadIdx.x;
    // maxAppliedWriteByExecuteAt: the Applied Write executing last, and its index in committedByExecuteAt
    Ts3 maw{0, 0, 0};
    bool has = false;
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        if (a.st[x] == AD_ST_APPLIED && cs_kind(a.tl[x]) == AD_KIND_WRITE) {
            const Ts3 e{a.em[x], a.el[x], a.en[x]};
            if (!has || ts3_cmp(e, maw) > 0) { maw = e; has = true; }
        }
    }
    cs_fold<true>(maw, has);
    if (!has) return;
    uint32_t below = 0;
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        if (cs_decided(a.st[x]) && ts3_cmp(Ts3{a.em[x], a.el[x], a.en[x]}, maw) < 0) ++below;
    }
    if (cs_block_sum(below, s.c) < interval) return;
    // the prune point: the Applied Write executing last among those before maxAppliedWrite within minHlcDelta of it
    const int64_t lim = (int64_t)cs_hlc(maw) - min_hlc_delta;
    Ts3 pex{0, 0, 0};
    bool hp = false;
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        if (a.st[x] == AD_ST_APPLIED && cs_kind(a.tl[x]) == AD_KIND_WRITE) {
            const Ts3 e{a.em[x], a.el[x], a.en[x]};
            if (ts3_cmp(e, maw) < 0 && (int64_t)cs_hlc(e) <= lim && (!hp || ts3_cmp(e, pex) > 0)) { pex = e; hp = true; }
        }
    }
    cs_fold<true>(pex, hp);
    if (!hp) return;
    if (tid == 0) s.idx = n;
    __syncthreads();
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        if (a.st[x] == AD_ST_APPLIED && cs_kind(a.tl[x]) == AD_KIND_WRITE &&
            ts3_cmp(Ts3{a.em[x], a.el[x], a.en[x]}, pex) == 0) atomicMin(&s.idx, r);
    }
    __syncthreads();
    const uint32_t p = s.idx;                                     // byId position of the new prunedBefore
    __syncthreads();
    if (p >= n) return;
    const Ts3 pt{a.tm[base + p], a.tl[base + p], a.tn[base + p]};
    if (ts3_cmp(pt, Ts3{a.pbm[key], a.pbl[key], a.pbn[key]}) <= 0 || p == 0) return;
    // pruneBefore's byId scan below p
    const uint64_t* pbits = a.bits + a.bbase + (size_t)a.slot[base + p] * a.words;
    for (uint32_t q = tid; q < a.words; q += CS_T) { s.merged[q] = pbits[q]; s.gone[q] = 0ull; s.dead[q] = 0ull; }
    __syncthreads();
    bool any = false;
    for (uint32_t r = 0; r < p; ++r) {
        const size_t x = base + r;
        const uint32_t st = a.st[x];
        bool rm = false;
        if (st == AD_ST_INVALID) {
            rm = true;
        } else if (st == AD_ST_APPLIED) {
            const Ts3 e{a.em[x], a.el[x], a.en[x]};
            if (ts3_cmp(e, pex) < 0) {
                const uint64_t* b = a.bits + a.bbase + (size_t)a.slot[x] * a.words;
                bool extra = false;
                for (uint32_t q = tid; q < a.words; q += CS_T) extra |= (b[q] & ~s.merged[q]) != 0ull;
                extra = __syncthreads_or(extra);
                if (!extra) rm = true;
                else if (ts3_cmp(e, Ts3{a.tm[x], a.tl[x], a.tn[x]}) == 0)
                    for (uint32_t q = tid; q < a.words; q += CS_T) s.merged[q] |= b[q];
            }
        }
        if (rm) {
            any = true;
            if (tid == 0) {
                const uint32_t sl = a.slot[x];
                s.gone[r >> 6] |= 1ull << (r & 63);
                s.dead[sl >> 6] |= 1ull << (sl & 63);
            }
        }
        __syncthreads();
    }
    if (!any) return;                                             // pos == retainCount: nothing changes
    if (tid == 0) {
        a.pbm[key] = pt.msb; a.pbl[key] = pt.lsb; a.pbn[key] = pt.node;
        uint32_t g = 0, d = 0;
        for (uint32_t q = 0; q < a.words; ++q) {
            s.gpc[q] = g; s.dpc[q] = d;
            g += (uint32_t)__popcll(s.gone[q]); d += (uint32_t)__popcll(s.dead[q]);
        }
        s.idx = g;
    }
    __syncthreads();
    const uint32_t removed = s.idx;
    // rows: kept rows move down to their rank among the kept (chunks in ascending order: a row is read before any
    // write can reach its position), their slots renumbered to the rank among the kept slots
    for (uint32_t r0 = 0; r0 < n; r0 += CS_T) {
        const uint32_t r = r0 + tid;
        const bool keep = r < n && !((s.gone[r >> 6] >> (r & 63)) & 1ull);
        uint64_t vtm = 0, vtl = 0, vem = 0, vel = 0;
        int32_t vtn = 0, ven = 0;
        uint8_t vst = 0;
        uint32_t vsl = 0, to = 0;
        if (keep) {
            const size_t x = base + r;
            vtm = a.tm[x]; vtl = a.tl[x]; vtn = a.tn[x]; vem = a.em[x]; vel = a.el[x]; ven = a.en[x]; vst = a.st[x];
            vsl = a.slot[x];
            vsl -= cs_rank(s.dead, s.dpc, vsl);
            to = r - cs_rank(s.gone, s.gpc, r);
        }
        __syncthreads();
        if (keep) {
            const size_t y = base + to;
            a.tm[y] = vtm; a.tl[y] = vtl; a.tn[y] = vtn; a.em[y] = vem; a.el[y] = vel; a.en[y] = ven; a.st[y] = vst;
            a.slot[y] = vsl;
        }
        __syncthreads();
    }
    // missing() bitmaps: each kept slot's row moves to its new slot with its columns compacted (one wave per slot,
    // CS_T / 64 slots per step, every read of a step before its writes)
    const int wv = tid >> 6, lane = tid & 63;
    for (uint32_t s0 = 0; s0 < n; s0 += CS_T / 64) {
        const uint32_t sl = s0 + wv;
        const bool keep = sl < n && !((s.dead[sl >> 6] >> (sl & 63)) & 1ull);
        if (keep) cs_remap_row(a, a.bits + a.bbase + (size_t)sl * a.words, s.stage[wv], s, lane);
        __syncthreads();
        if (keep) {
            uint64_t* dst = a.bits + a.bbase + (size_t)(sl - cs_rank(s.dead, s.dpc, sl)) * a.words;
            for (uint32_t q = lane; q < a.words; q += 64) dst[q] = s.stage[wv][q];
        }
        __syncthreads();
    }
    // loadingPruned witnesses: pruned rows leave, the others renumbered
    const size_t lb = a.grbase;
    for (uint32_t j0 = 0; j0 < L; j0 += CS_T / 64) {
        const uint32_t j = j0 + wv;
        if (j < L) cs_remap_row(a, a.lp_bits + a.gbbase + (size_t)j * a.words, s.stage[wv], s, lane);
        __syncthreads();
        if (j < L) for (uint32_t q = lane; q < a.words; q += 64) a.lp_bits[a.gbbase + (size_t)j * a.words + q] = s.stage[wv][q];
        __syncthreads();
    }
    n -= removed;
}

// ---- unmanaged txns (CommandsForKey.unmanageds; Updating.updateUnmanaged :715-849, PostProcess.notifyUnmanaged :164-246)
__device__ inline bool cs_me(uint64_t lsb) {                   // CommandsForKey.managesExecution: key-domain Read / Write
    const uint32_t k = cs_kind(lsb);
    return (lsb & 1ull) == 0 && (k == AD_KIND_READ || k == AD_KIND_WRITE);
}
// Unmanaged.compareTo: pending, then waitingUntil, then txnId
__device__ inline int cs_um_cmp(uint32_t p1, const Ts3& w1, const Ts3& t1, uint32_t p2, const Ts3& w2, const Ts3& t2) {
    if (p1 != p2) return p1 < p2 ? -1 : 1;
    const int c = ts3_cmp(w1, w2);
    return c != 0 ? c : ts3_cmp(t1, t2);
}
__device__ inline Ts3 cs_um_w(const CfkStoreArgs& a, size_t x) { return Ts3{a.um_wm[x], a.um_wl[x], a.um_wn[x]}; }
__device__ inline Ts3 cs_um_t(const CfkStoreArgs& a, size_t x) { return Ts3{a.um_tm[x], a.um_tl[x], a.um_tn[x]}; }
// (thread 0) one notification of this call
__device__ inline void cs_um_emit(const CfkStoreArgs& a, uint32_t key, uint32_t e, uint32_t tag, const Ts3& t) {
    const uint32_t o = a.nt_base[key] + a.nt_cnt[key]++;
    a.nt_ev[o] = e; a.nt_tag[o] = (uint8_t)tag; a.nt_tm[o] = t.msb; a.nt_tl[o] = t.lsb; a.nt_tn[o] = t.node;
}
// (thread 0) entries [s, e) leave the registry
__device__ inline void cs_um_remove(const CfkStoreArgs& a, size_t ub, uint32_t& U, uint32_t s, uint32_t e) {
    const uint32_t d = e - s;
    for (uint32_t i = e; i < U; ++i) {
        const size_t x = ub + i, y = ub + i - d;
        a.um_p[y] = a.um_p[x]; a.um_wm[y] = a.um_wm[x]; a.um_wl[y] = a.um_wl[x]; a.um_wn[y] = a.um_wn[x];
        a.um_tm[y] = a.um_tm[x]; a.um_tl[y] = a.um_tl[x]; a.um_tn[y] = a.um_tn[x];
    }
    U -= d;
}
// (thread 0) (p, w, t) joins the sorted registry unless present (linearUnion of the sorted arrays); false: full
__device__ inline bool cs_um_insert(const CfkStoreArgs& a, size_t ub, uint32_t cap, uint32_t& U, uint32_t p, const Ts3& w,
                                    const Ts3& t) {
    uint32_t lo = 0, hi = U;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (cs_um_cmp(a.um_p[ub + m], cs_um_w(a, ub + m), cs_um_t(a, ub + m), p, w, t) < 0) lo = m + 1; else hi = m;
    }
    if (lo < U && cs_um_cmp(a.um_p[ub + lo], cs_um_w(a, ub + lo), cs_um_t(a, ub + lo), p, w, t) == 0) return true;
    if (U >= cap) return false;
    for (uint32_t i = U; i > lo; --i) {
        const size_t x = ub + i - 1, y = ub + i;
        a.um_p[y] = a.um_p[x]; a.um_wm[y] = a.um_wm[x]; a.um_wl[y] = a.um_wl[x]; a.um_wn[y] = a.um_wn[x];
        a.um_tm[y] = a.um_tm[x]; a.um_tl[y] = a.um_tl[x]; a.um_tn[y] = a.um_tn[x];
    }
    const size_t x = ub + lo;
    a.um_p[x] = (uint8_t)p; a.um_wm[x] = w.msb; a.um_wl[x] = w.lsb; a.um_wn[x] = w.node;
    a.um_tm[x] = t.msb; a.um_tl[x] = t.lsb; a.um_tn[x] = t.node;
    ++U;
    return true;
}

// PostProcess.notifyUnmanaged after an update that changed the key (new InternalStatus ns, executeAt ex): the unmanageds
// waiting for every managed txn below minUndecided (and below the first loadingPruned TxnId) to commit are notified
// (findCommit, exclusive bound); when the update applied something, the ones waiting for the contiguous applied prefix
// to reach their waitingUntil (maxContiguousManagedApplied, findFirstApply / findApply, inclusive).
__device__ inline void cs_um_notify(const CfkStoreArgs& a, uint32_t key, size_t base, uint32_t n, uint32_t L, uint32_t ns,
                                    const Ts3& ex, uint32_t e, CsPruneLds& s, uint32_t* s_U) {
    const int tid = threadIdx.x;
    if (*s_U == 0) return;                                        // no unmanaged txn waits on this key
    const size_t ub = a.grbase, lb = ub;
    Ts3 b{0, 0, 0};
    bool hb = false;
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        if (a.st[x] < AD_ST_COMMITTED && cs_me(a.tl[x])) {
            const Ts3 u{a.tm[x], a.tl[x], a.tn[x]};
            if (!hb || ts3_cmp(u, b) < 0) { b = u; hb = true; }
        }
    }
    for (uint32_t j = tid; j < L; j += CS_T) {
        const Ts3 u{a.lpm[lb + j], a.lpl[lb + j], a.lpn[lb + j]};
        if (!hb || ts3_cmp(u, b) < 0) { b = u; hb = true; }
    }
    cs_fold<false>(b, hb);
    if (tid == 0) {
        uint32_t U = *s_U, end = 0;
        while (end < U && a.um_p[ub + end] == UM_COMMIT && (!hb || ts3_cmp(b, cs_um_w(a, ub + end)) > 0)) ++end;
        for (uint32_t i = 0; i < end; ++i) cs_um_emit(a, key, e, 0, cs_um_t(a, ub + i));
        if (end) cs_um_remove(a, ub, U, 0, end);
        *s_U = U;
    }
    __syncthreads();
    if (ns < AD_ST_APPLIED) return;
    // maxContiguousManagedApplied (CommandsForKey.java:1419-1436): the last committed txn by executeAt before the first
    // committed, unapplied Read / Write executing after maxAppliedWrite
    Ts3 maw{0, 0, 0}, bl{0, 0, 0}, mca{0, 0, 0};
    bool hm = false, hbl = false, hmca = false;
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        if (a.st[x] == AD_ST_APPLIED && cs_kind(a.tl[x]) == AD_KIND_WRITE) {
            const Ts3 u{a.em[x], a.el[x], a.en[x]};
            if (!hm || ts3_cmp(u, maw) > 0) { maw = u; hm = true; }
        }
    }
    cs_fold<true>(maw, hm);
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        const uint32_t st = a.st[x];
        if (cs_decided(st) && st != AD_ST_APPLIED && cs_me(a.tl[x])) {
            const Ts3 u{a.em[x], a.el[x], a.en[x]};
            if ((!hm || ts3_cmp(u, maw) > 0) && (!hbl || ts3_cmp(u, bl) < 0)) { bl = u; hbl = true; }
        }
    }
    cs_fold<false>(bl, hbl);
    for (uint32_t r = tid; r < n; r += CS_T) {
        const size_t x = base + r;
        if (cs_decided(a.st[x])) {
            const Ts3 u{a.em[x], a.el[x], a.en[x]};
            if ((!hbl || ts3_cmp(u, bl) < 0) && (!hmca || ts3_cmp(u, mca) > 0)) { mca = u; hmca = true; }
        }
    }
    cs_fold<true>(mca, hmca);
    if (hmca && ts3_cmp(mca, ex) < 0) hmca = false;
    if (hmca && tid == 0) {
        uint32_t U = *s_U, st = 0;
        while (st < U && a.um_p[ub + st] == UM_COMMIT) ++st;
        uint32_t end = st;
        while (end < U && ts3_cmp(mca, cs_um_w(a, ub + end)) >= 0) ++end;
        for (uint32_t i = st; i < end; ++i) cs_um_emit(a, key, e, 1, cs_um_t(a, ub + i));
        if (end != st) cs_um_remove(a, ub, U, st, end);
        *s_U = U;
    }
    __syncthreads();
}

// Updating.updateUnmanaged (:715-849) for unmanaged txn t (kind from its TxnId, executeAt wex) whose deps at this key are
// the Read / Write TxnIds dep[d0, d1): readyToApply / waitingToApply / executesAt over the rows it depends on (and, for
// sync points, the managed rows between its first and last dependency); register (registerUnmanaged): a dependency the
// key does not know holds it back (its TRANSITIVELY_KNOWN row or its loadingPruned entry is an earlier event of the
// stream); not ready -> (APPLY, executesAt) or (COMMIT, the last dependency) joins the registry, else it is notified.
// false: the registry is full.
__device__ inline bool cs_um_update(const CfkStoreArgs& a, uint32_t key, size_t base, uint32_t n, uint32_t L, const Ts3& t,
                                    const Ts3& wex, uint32_t d0, uint32_t d1, bool reg, uint32_t e, CsPruneLds& s,
                                    uint32_t* s_U) {
    const int tid = threadIdx.x;
    if (d0 == d1) {
        if (tid == 0) cs_um_emit(a, key, e, 2, t);
        __syncthreads();
        return true;
    }
    const uint32_t wk = cs_kind(t.lsb);
    const bool sync = wk == AD_KIND_SYNC_POINT || wk == AD_KIND_EXCLUSIVE_SYNC_POINT;
    bool ready = true, waiting = true, hx = false;
    Ts3 xm{0, 0, 0};
    auto consider = [&](size_t x) {
        const uint32_t st = a.st[x];
        if (st < AD_ST_COMMITTED) { ready = waiting = false; return; }
        if (st == AD_ST_INVALID) return;
        const Ts3 u{a.em[x], a.el[x], a.en[x]};
        if (ts3_cmp(u, wex) < 0 || wk == AD_KIND_EPHEMERAL_READ ||
            (wk == AD_KIND_EXCLUSIVE_SYNC_POINT && ts3_cmp(Ts3{a.tm[x], a.tl[x], a.tn[x]}, t) < 0)) {
            ready = ready && st == AD_ST_APPLIED;
            if (!hx || ts3_cmp(u, xm) > 0) { xm = u; hx = true; }
        }
    };
    for (uint32_t j = d0 + tid; j < d1; j += CS_T) {
        bool f;
        const uint32_t q = cs_find(a, base, n, Ts3{a.dtm[j], a.dtl[j], a.dtn[j]}, f);
        if (f) consider(base + q);
        else if (reg) ready = waiting = false;
    }
    if (sync) {                                                   // the managed rows between the deps (:760-777)
        bool f0, f1;
        const uint32_t lo = cs_find(a, base, n, Ts3{a.dtm[d0], a.dtl[d0], a.dtn[d0]}, f0);
        uint32_t hi = cs_find(a, base, n, Ts3{a.dtm[d1 - 1], a.dtl[d1 - 1], a.dtn[d1 - 1]}, f1);
        hi += f1 ? 1u : 0u;
        for (uint32_t r = lo + tid; r < hi; r += CS_T)
            if (cs_me(a.tl[base + r])) consider(base + r);
        // Pruning.isAnyPredecessorWaitingOnPruned (:140-157): a loading managed TxnId below t witnessed at or before t
        const size_t lb = a.grbase;
        bool anyp = false;
        for (uint32_t j = tid; j < L; j += CS_T) {
            const size_t x = lb + j;
            anyp |= ts3_cmp(Ts3{a.lpm[x], a.lpl[x], a.lpn[x]}, t) < 0 && cs_me(a.lpl[x]) && a.lp_xh[x] &&
                    ts3_cmp(t, Ts3{a.lp_xm[x], a.lp_xl[x], a.lp_xn[x]}) >= 0;
        }
        if (anyp) ready = waiting = false;
    }
    ready = __syncthreads_and(ready ? 1 : 0) != 0;
    waiting = __syncthreads_and(waiting ? 1 : 0) != 0;
    cs_fold<true>(xm, hx);
    bool ok = true;
    if (tid == 0) {
        const size_t ub = a.grbase;
        uint32_t U = *s_U;
        if (ready) cs_um_emit(a, key, e, 2, t);
        else if (waiting) ok = cs_um_insert(a, ub, a.cap, U, UM_APPLY, xm, t);
        else ok = cs_um_insert(a, ub, a.cap, U, UM_COMMIT, Ts3{a.dtm[d1 - 1], a.dtl[d1 - 1], a.dtn[d1 - 1]}, t);
        *s_U = U;
        s.idx = ok ? 1u : 0u;
    }
    __syncthreads();
    ok = s.idx != 0;
    __syncthreads();
    return ok;
}

// CommandsForKey.update for a stream of commands (ballots all zero: a command updates its TxnInfo only when its
// InternalStatus rises, as in CommandsForKeyTest), Updating.insertOrUpdate's cases (Updating.java:99-358):
//   statuses with deps (ACCEPTED .. APPLIED): the row's missing set is rebuilt from the command's deps (every
//     undecided txn below depsKnownBefore it witnesses and its deps lack, :194-287); deps unknown to the CFK are
//     inserted TRANSITIVELY_KNOWN (:178-227) and join the missing sets of the other rows that witness them
//     (insertOrUpdateWithAdditions :385-450); a new undecided row joins the others' missing sets (insertSelfMissing),
//     a row that becomes decided leaves them (removeSelfMissing);
//   statuses without deps: a new row joins the others' missing sets unless INVALID; an undecided row invalidated
//     leaves them.
// A TRANSITIVELY_KNOWN event is the insertAdditionsOnly path of Updating.updateUnmanaged (:452-514).
// Pruning: deps below prunedBefore that the rows lack join loadingPruned instead of the rows (removePrunedAdditions,
// Utils.java:229-244); a LOAD event, or an update of a TxnId in loadingPruned, is CommandsForKey.update's wasPruned path
// (:1015-1024: no missing(), the TxnId joins the other rows' missing() except its witnesses'); PRUNE / LOADING events
// as CS_OP_* says.
constexpr uint32_t CS_EV_CHUNK = 128, CS_DEP_CHUNK = 512;
struct CsEvChunk {                            // a chunk of the key's events and their deps (k_cfk_apply)
    uint64_t tm[CS_EV_CHUNK], tl[CS_EV_CHUNK], xm[CS_EV_CHUNK], xl[CS_EV_CHUNK];
    int32_t tn[CS_EV_CHUNK], xn[CS_EV_CHUNK];
    uint8_t st[CS_EV_CHUNK], op[CS_EV_CHUNK];
    uint32_t doff[CS_EV_CHUNK + 1];
    uint64_t dm[CS_DEP_CHUNK], dl[CS_DEP_CHUNK];
    int32_t dn[CS_DEP_CHUNK];
    uint32_t m;
};
// (thread 0) the key ran out of rows / loadingPruned / registry entries at event e (global index), before changing
__device__ inline void cs_out_of_rows(const CfkStoreArgs& a, uint32_t key, uint32_t e) {
    if (threadIdx.x == 0) {
        *a.overflow = 1u;
        if (a.kres) a.kres[key] = e;
    }
}
struct CsApplyLds {
    CsEvChunk ev;
    uint64_t miss[CS_MAX_WORDS];
    uint32_t add[CS_T];                       // this event's additions (slots), CS_T at a time
    uint32_t nadd, row, U;
    int j;
    uint64_t t0;
    uint32_t tcls;
    CsPruneLds prune;
};
// The key's events in order (a = the rows' view: HBM, or the LDS copy with base 0).  Returns early when the key runs
// out of rows or loadingPruned / registry entries (overflow flag set); n, L and s.U are the key's counts either way.
__device__ __attribute__((always_inline)) inline bool cs_apply_events(const CfkStoreArgs& a, uint32_t key, size_t base, uint32_t& n, uint32_t& L,
                                       CsApplyLds& sh, uint32_t e_lo, uint32_t e_hi, uint32_t e_id0) {
    uint64_t* s_miss = sh.miss;
    uint32_t* s_add = sh.add;
    uint32_t& s_nadd = sh.nadd;
    int& s_j = sh.j;
    CsPruneLds& s_prune = sh.prune;
    uint32_t& s_U = sh.U;
    for (uint32_t e = e_lo; e < e_hi; ++e) {
        const Ts3 t{a.etm[e], a.etl[e], a.etn[e]};
        const uint32_t op = a.eop ? a.eop[e] : CS_OP_UPDATE;
        if (a.dbg && threadIdx.x == 0) {                          // the previous event's cycles, by its class
            const uint64_t now = clock64();
            if (sh.tcls < 8) {
                atomicAdd((unsigned long long*)&a.dbg[2 * (key % 8) * 8 + 2 * sh.tcls], (unsigned long long)(now - sh.t0));
                atomicAdd((unsigned long long*)&a.dbg[2 * (key % 8) * 8 + 2 * sh.tcls + 1], 1ull);
            }
            sh.t0 = now;
            sh.tcls = op == CS_OP_UPDATE ? (a.dep_off[e + 1] > a.dep_off[e] ? 0u : (cs_has_deps(a.est[e]) ? 1u : 2u)) : 2u + op;
        }
        if (op == CS_OP_PRUNE) {
            cs_maybe_prune(a, key, base, n, L, (uint32_t)a.een[e], (int64_t)a.eem[e], s_prune);
            __syncthreads();
            continue;
        }
        if (op == CS_OP_LOADING) {
            uint32_t w = 0xFFFFFFFFu;
            Ts3 wt{0, 0, 0};
            const bool hw = a.dep_off[e + 1] > a.dep_off[e];
            if (hw) {
                const uint32_t j = a.dep_off[e];
                wt = Ts3{a.dtm[j], a.dtl[j], a.dtn[j]};
                bool f;
                const uint32_t q = cs_find(a, base, n, wt, f);
                if (f) w = a.slot[base + q];
            }
            if (!cs_lp_add(a, key, L, t, w, &s_j, wt, hw)) { cs_out_of_rows(a, key, e + e_id0); return false; }
            continue;
        }
        if (op == CS_OP_UNMANAGED || op == CS_OP_UNMANAGED_RECHECK) {
            if (!cs_um_update(a, key, base, n, L, t, Ts3{a.eem[e], a.eel[e], a.een[e]}, a.dep_off[e], a.dep_off[e + 1],
                              op == CS_OP_UNMANAGED, e + e_id0, s_prune, &s_U)) {
                cs_out_of_rows(a, key, e + e_id0);
                return false;
            }
            continue;
        }
        const uint32_t ns = a.est[e];
        bool found;
        const uint32_t p = cs_find(a, base, n, t, found);
        const uint32_t cur = found ? a.st[base + p] : 0xFFu;
        if (found && ns <= cur) continue;                            // not a higher InternalStatus: no change
        const int jl = cs_lp_find(a, key, L, t, &s_j);
        if (op == CS_OP_LOAD || jl >= 0) {
            // TxnInfo.create: executeAt (statuses with one), no missing(); the loadingPruned entry's witnesses skip it
            const Ts3 ex{a.eem[e], a.eel[e], a.een[e]};
            if (!found && n >= a.cap) { cs_out_of_rows(a, key, e + e_id0); return false; }   // (before any change)
            for (uint32_t w = threadIdx.x; w < a.words; w += CS_T)
                s_miss[w] = jl >= 0 ? a.lp_bits[a.gbbase + (size_t)jl * a.words + w] : 0ull;
            __syncthreads();
            if (jl >= 0) cs_lp_remove(a, key, L, jl);
            uint32_t ts;
            if (!found) {
                ts = cs_insert(a, base, n, p, t, ns, ex);
            } else {
                ts = a.slot[base + p];
                if (threadIdx.x == 0) {
                    const size_t x = base + p;
                    a.st[x] = (uint8_t)ns; a.em[x] = ex.msb; a.el[x] = ex.lsb; a.en[x] = ex.node;
                }
                for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) a.bits[(a.bbase + (size_t)ts * a.words) + w] = 0ull;
                __syncthreads();
            }
            if (cs_decided(ns) && !(found && cs_decided(cur))) cs_remove_missing(a, base, n, ts);
            else if (found && cur < AD_ST_COMMITTED && ns == AD_ST_INVALID) cs_remove_missing(a, base, n, ts);
            else if (!found && ns != AD_ST_INVALID) cs_add_missing(a, base, n, t, ts, 0xFFFFFFFFu, s_miss);
            __syncthreads();
            cs_um_notify(a, key, base, n, L, ns, ex, e + e_id0, s_prune, &s_U);
            continue;
        }
        const uint32_t d0 = a.dep_off[e], d1 = a.dep_off[e + 1];
        if (cs_has_deps(ns)) {
            const Ts3 ex{a.eem[e], a.eel[e], a.een[e]};
            const Ts3 dkb = cs_decided(ns) ? ex : t;
            const uint32_t n_pre = n;
            // room for the event's new rows (its unknown deps at or above prunedBefore, and itself) and loadingPruned
            // entries (its unknown deps below prunedBefore), checked before anything changes: a key that runs out stops
            // at this event with its state intact, and resumes from it in a larger tier
            if (n + (d1 - d0) + (found ? 0u : 1u) > a.cap || L + (d1 - d0) > a.cap) {
                const Ts3 pb0{a.pbm[key], a.pbl[key], a.pbn[key]};
                uint32_t nr = found ? 0u : 1u, nl = 0;
                for (uint32_t j = d0 + threadIdx.x; j < d1; j += CS_T) {
                    const Ts3 d{a.dtm[j], a.dtl[j], a.dtn[j]};
                    bool f;
                    cs_find(a, base, n, d, f);
                    if (f) continue;
                    if (ts3_cmp(d, pb0) >= 0) { ++nr; continue; }
                    bool inl = false;                                  // already loading?
                    for (uint32_t q = 0; q < L && !inl; ++q)
                        inl = ts3_cmp(Ts3{a.lpm[a.grbase + q], a.lpl[a.grbase + q], a.lpn[a.grbase + q]}, d) == 0;
                    if (!inl) ++nl;
                }
                nr = cs_block_sum(nr, nullptr) - (found ? 0u : (uint32_t)(CS_T - 1));   // (the own row counted per lane)
                nl = cs_block_sum(nl, nullptr);
                if (n + nr > a.cap || L + nl > a.cap) { cs_out_of_rows(a, key, e + e_id0); return false; }
            }
            // the row's missing set over the current rows (before the additions: they are in the deps)
            for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) s_miss[w] = 0ull;
            __syncthreads();
            const uint32_t kt = cs_kind(t.lsb);
            for (uint32_t r = threadIdx.x; r < n; r += CS_T) {
                const size_t x = base + r;
                const Ts3 u{a.tm[x], a.tl[x], a.tn[x]};
                if (a.st[x] >= AD_ST_COMMITTED || !witnesses(kt, cs_kind(u.lsb)) || ts3_cmp(u, dkb) >= 0 ||
                    ts3_cmp(u, t) == 0)
                    continue;
                uint32_t lo = d0, hi = d1;                            // u among the deps?
                while (lo < hi) {
                    const uint32_t m = (lo + hi) >> 1;
                    if (ts3_cmp(Ts3{a.dtm[m], a.dtl[m], a.dtn[m]}, u) < 0) lo = m + 1; else hi = m;
                }
                if (lo < d1 && ts3_cmp(Ts3{a.dtm[lo], a.dtl[lo], a.dtn[lo]}, u) == 0) continue;
                const uint32_t s = a.slot[x];
                atomicOr((unsigned long long*)&s_miss[s >> 6], 1ull << (s & 63));
            }
            __syncthreads();
            // deps unknown to the CFK: TRANSITIVELY_KNOWN rows, in deps order (below prunedBefore: loadingPruned).
            // Their missing() joins are applied in chunks of CS_T additions (s_add): a join touches the rows that
            // witness the addition other than the command's own, whose missing() is s_miss (written below)
            if (threadIdx.x == 0) s_nadd = 0;
            __syncthreads();
            const uint32_t cmd_slot = found ? a.slot[base + p] : 0xFFFFFFFFu;
            auto flush_adds = [&](uint32_t skip) {
                const uint32_t nadd = s_nadd;
                for (uint32_t k = 0; k < nadd; ++k) {
                    const uint32_t s = s_add[k];
                    // the addition's TxnId: find its row through the slot (rows shifted since): a scan for the slot
                    for (uint32_t r = threadIdx.x; r < n; r += CS_T) if (a.slot[base + r] == s) sh.row = r;
                    __syncthreads();
                    const size_t x = base + sh.row;
                    const Ts3 ad{a.tm[x], a.tl[x], a.tn[x]};
                    cs_add_missing(a, base, n, ad, s, skip);
                }
                __syncthreads();
                if (threadIdx.x == 0) s_nadd = 0;
                __syncthreads();
            };
            const Ts3 pb{a.pbm[key], a.pbl[key], a.pbn[key]};
            for (uint32_t j = d0; j < d1; ++j) {
                const Ts3 d{a.dtm[j], a.dtl[j], a.dtn[j]};
                if (j > d0 && ts3_cmp(Ts3{a.dtm[j - 1], a.dtl[j - 1], a.dtn[j - 1]}, d) >= 0) {
                    if (threadIdx.x == 0) *a.bad = 1u;
                    break;
                }
                bool f;
                const uint32_t q = cs_find(a, base, n, d, f);
                if (f) continue;
                if (ts3_cmp(d, pb) < 0) continue;                      // a pruned addition: loadingPruned, below
                if (n >= a.cap) { cs_out_of_rows(a, key, e + e_id0); return false; }
                if (s_nadd >= (uint32_t)CS_T) flush_adds(cmd_slot);
                const uint32_t s = cs_insert(a, base, n, q, d, AD_ST_TRANSITIVELY_KNOWN, d);
                if (threadIdx.x == 0) s_add[s_nadd++] = s;
                __syncthreads();
            }
            uint32_t ts;
            bool fnow = found;
            // t's position after the additions (none inserted: where it was)
            const uint32_t p2 = n == n_pre ? p : cs_find(a, base, n, t, fnow);
            if (!fnow) {
                if (n >= a.cap) { cs_out_of_rows(a, key, e + e_id0); return false; }
                ts = cs_insert(a, base, n, p2, t, ns, ex);
            } else {
                ts = a.slot[base + p2];
                if (threadIdx.x == 0) {
                    const size_t x = base + p2;
                    a.st[x] = (uint8_t)ns; a.em[x] = ex.msb; a.el[x] = ex.lsb; a.en[x] = ex.node;
                }
            }
            for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) a.bits[(a.bbase + (size_t)ts * a.words) + w] = s_miss[w];
            __syncthreads();
            // pruned additions (deps below prunedBefore that are not rows): loadingPruned, witnessed by this command
            for (uint32_t j = d0; j < d1; ++j) {
                const Ts3 d{a.dtm[j], a.dtl[j], a.dtn[j]};
                if (ts3_cmp(d, pb) >= 0) break;                       // deps ascend
                bool f;
                cs_find(a, base, n, d, f);
                if (f) continue;
                if (!cs_lp_add(a, key, L, d, ts, &s_j, t, true)) {
                    cs_out_of_rows(a, key, e + e_id0);
                    return false;
                }
            }
            flush_adds(ts);
            if (!found && ns < AD_ST_COMMITTED) cs_add_missing(a, base, n, t, ts, 0xFFFFFFFFu);
            if (found && cur < AD_ST_COMMITTED && ns >= AD_ST_COMMITTED) cs_remove_missing(a, base, n, ts);
            __syncthreads();
            cs_um_notify(a, key, base, n, L, ns, ex, e + e_id0, s_prune, &s_U);
        } else {
            if (!found) {
                if (n >= a.cap) { cs_out_of_rows(a, key, e + e_id0); return false; }
                const uint32_t ts = cs_insert(a, base, n, p, t, ns, t);
                if (ns != AD_ST_INVALID) cs_add_missing(a, base, n, t, ts, 0xFFFFFFFFu);
            } else {
                const uint32_t ts = a.slot[base + p];
                if (threadIdx.x == 0) {
                    const size_t x = base + p;
                    a.st[x] = (uint8_t)ns; a.em[x] = t.msb; a.el[x] = t.lsb; a.en[x] = t.node;
                }
                for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) a.bits[(a.bbase + (size_t)ts * a.words) + w] = 0ull;
                __syncthreads();
                if (cur < AD_ST_COMMITTED && ns == AD_ST_INVALID) cs_remove_missing(a, base, n, ts);
            }
            __syncthreads();
            cs_um_notify(a, key, base, n, L, ns, t, e + e_id0, s_prune, &s_U);
        }
        __syncthreads();
    }
    return true;
}

// One workgroup per key with events.  LDS: the key's rows and missing() bitmaps (capacity <= CS_LDS_CAP) are copied
// into LDS, the events applied there and the result written back once — every row read of an event (the byId
// searches, the missing() rebuild, the notify folds) is then an LDS access instead of an HBM round trip (~10 dependent
// ones per event: ~10 us per event on the hottest key's serial chain).  loadingPruned and the unmanaged registry
// (empty for most keys) stay in HBM.
constexpr uint32_t CS_LDS_CAP = 256;
template <bool LDS>
static __global__ __launch_bounds__(CS_T) void k_cfk_apply(CfkStoreArgs a) {
    __shared__ CsApplyLds sh;
    constexpr uint32_t RC = LDS ? CS_LDS_CAP : 1u, BW = LDS ? CS_LDS_CAP * (CS_LDS_CAP / 64) : 1u;
    __shared__ uint64_t r_tm[RC], r_tl[RC], r_em[RC], r_el[RC], r_bits[BW];
    __shared__ int32_t r_tn[RC], r_en[RC];
    __shared__ uint32_t r_slot[RC];
    __shared__ uint8_t r_st[RC];
    const uint32_t key = a.klist ? a.klist[blockIdx.x] : blockIdx.x;
    if (key >= a.K) return;
    const CsTier tr = cs_tier(key, a.K, a.cap, a.words, a.kslot, a.capB, a.wordsB);
    if (LDS && tr.cap > CS_LDS_CAP) return;                      // a large-tier key: the HBM kernel's
    const uint32_t e_first = a.ev_start ? a.ev_start[key] : a.ev_off[key];
    if (!a.ev_start && threadIdx.x == 0) a.nt_cnt[key] = 0;     // (a resumed key keeps this call's notifications)
    if (e_first >= a.ev_off[key + 1]) return;                    // no events (or none left): the key is unchanged
    const size_t gbase = tr.rbase;
    uint32_t n = a.cnt[key];
    uint32_t L = a.lp_cnt[key];
    if (threadIdx.x == 0) { sh.U = a.um_cnt[key]; sh.tcls = 8; sh.t0 = 0; }
    CfkStoreArgs v = a;
    v.cap = tr.cap; v.words = tr.words; v.bbase = tr.bbase; v.grbase = tr.rbase; v.gbbase = tr.bbase;
    size_t base = gbase;
    if (LDS) {
        for (uint32_t r = threadIdx.x; r < n; r += CS_T) {
            const size_t x = gbase + r;
            r_tm[r] = a.tm[x]; r_tl[r] = a.tl[x]; r_tn[r] = a.tn[x]; r_em[r] = a.em[x]; r_el[r] = a.el[x];
            r_en[r] = a.en[x]; r_st[r] = a.st[x]; r_slot[r] = a.slot[x];
        }
        for (uint32_t i = threadIdx.x; i < n * tr.words; i += CS_T) r_bits[i] = a.bits[tr.bbase + i];
        v.tm = r_tm; v.tl = r_tl; v.tn = r_tn; v.em = r_em; v.el = r_el; v.en = r_en; v.st = r_st; v.slot = r_slot;
        v.bits = r_bits;
        v.bbase = 0;
        base = 0;
    }
    __syncthreads();
    // the events in chunks of <= CS_EV_CHUNK whose deps fit CS_DEP_CHUNK, staged in LDS by one parallel load each (the
    // events' fields, then their deps): per event no dependent HBM read is left on the key's serial path (the deps'
    // searches and the additions scan read one dependency after another).  An event with more deps than a chunk holds
    // runs alone from HBM.
    for (uint32_t e = e_first, end = a.ev_off[key + 1]; e < end;) {
        const uint32_t lim = min(end - e, CS_EV_CHUNK);
        for (uint32_t i = threadIdx.x; i <= lim; i += CS_T) sh.ev.doff[i] = a.dep_off[e + i];
        if (threadIdx.x == 0) sh.ev.m = 0;
        __syncthreads();
        const uint32_t d0 = sh.ev.doff[0];
        for (uint32_t i = threadIdx.x + 1; i <= lim; i += CS_T)
            if (sh.ev.doff[i] - d0 <= CS_DEP_CHUNK) atomicMax(&sh.ev.m, i);
        __syncthreads();
        const uint32_t m = sh.ev.m, nd = m ? sh.ev.doff[m] - d0 : 0u;
        bool ok;
        if (m == 0) {                                             // one event with more deps than a chunk
            ok = cs_apply_events(v, key, base, n, L, sh, e, e + 1, 0);
            e += 1;
        } else {
            for (uint32_t i = threadIdx.x; i < m; i += CS_T) {
                const uint32_t x = e + i;
                sh.ev.tm[i] = a.etm[x]; sh.ev.tl[i] = a.etl[x]; sh.ev.tn[i] = a.etn[x]; sh.ev.st[i] = a.est[x];
                sh.ev.xm[i] = a.eem[x]; sh.ev.xl[i] = a.eel[x]; sh.ev.xn[i] = a.een[x];
                sh.ev.op[i] = a.eop ? a.eop[x] : (uint8_t)CS_OP_UPDATE;
            }
            for (uint32_t j = threadIdx.x; j < nd; j += CS_T) {
                sh.ev.dm[j] = a.dtm[d0 + j]; sh.ev.dl[j] = a.dtl[d0 + j]; sh.ev.dn[j] = a.dtn[d0 + j];
            }
            __syncthreads();
            for (uint32_t i = threadIdx.x; i <= m; i += CS_T) sh.ev.doff[i] -= d0;
            __syncthreads();
            CfkStoreArgs w = v;
            w.etm = sh.ev.tm; w.etl = sh.ev.tl; w.etn = sh.ev.tn; w.est = sh.ev.st; w.eem = sh.ev.xm; w.eel = sh.ev.xl;
            w.een = sh.ev.xn; w.eop = sh.ev.op; w.dep_off = sh.ev.doff; w.dtm = sh.ev.dm; w.dtl = sh.ev.dl; w.dtn = sh.ev.dn;
            ok = cs_apply_events(w, key, base, n, L, sh, 0, m, e);
            e += m;
        }
        __syncthreads();
        if (!ok) break;
    }
    __syncthreads();
    if (LDS) {                                                    // slots are dense: [0, n) rows, [0, n) bitmaps
        for (uint32_t r = threadIdx.x; r < n; r += CS_T) {
            const size_t x = gbase + r;
            a.tm[x] = r_tm[r]; a.tl[x] = r_tl[r]; a.tn[x] = r_tn[r]; a.em[x] = r_em[r]; a.el[x] = r_el[r];
            a.en[x] = r_en[r]; a.st[x] = r_st[r]; a.slot[x] = r_slot[r];
        }
        for (uint32_t i = threadIdx.x; i < n * tr.words; i += CS_T) a.bits[tr.bbase + i] = r_bits[i];
    }
    if (threadIdx.x == 0) { a.cnt[key] = n; a.lp_cnt[key] = L; a.um_cnt[key] = sh.U; }
}

// A key that ran out of rows in the regular tier moves to large-tier slot kslot_new[i]: its rows, loadingPruned and
// registry rows are copied to the slot's region and every bitmap row is re-strided (words -> wordsB words; the new
// words are zero).  One workgroup per moved key (klist).
static __global__ __launch_bounds__(256) void k_cfk_promote(CfkStoreArgs a, const uint32_t* __restrict__ slots) {
    const uint32_t key = a.klist[blockIdx.x];
    const CsTier from = cs_tier(key, a.K, a.cap, a.words, nullptr, a.capB, a.wordsB);
    const size_t r0 = (size_t)a.K * a.cap;
    const uint32_t b = slots[blockIdx.x];
    const CsTier to{r0 + (size_t)b * a.capB, r0 * a.words + (size_t)b * a.capB * a.wordsB, a.capB, a.wordsB};
    const uint32_t n = a.cnt[key], L = a.lp_cnt[key], U = a.um_cnt[key];
    for (uint32_t r = threadIdx.x; r < n; r += blockDim.x) {
        const size_t x = from.rbase + r, y = to.rbase + r;
        a.tm[y] = a.tm[x]; a.tl[y] = a.tl[x]; a.tn[y] = a.tn[x]; a.em[y] = a.em[x]; a.el[y] = a.el[x]; a.en[y] = a.en[x];
        a.st[y] = a.st[x]; a.slot[y] = a.slot[x];
    }
    for (uint32_t j = threadIdx.x; j < L; j += blockDim.x) {
        const size_t x = from.rbase + j, y = to.rbase + j;
        a.lpm[y] = a.lpm[x]; a.lpl[y] = a.lpl[x]; a.lpn[y] = a.lpn[x];
        a.lp_xm[y] = a.lp_xm[x]; a.lp_xl[y] = a.lp_xl[x]; a.lp_xn[y] = a.lp_xn[x]; a.lp_xh[y] = a.lp_xh[x];
    }
    for (uint32_t u = threadIdx.x; u < U; u += blockDim.x) {
        const size_t x = from.rbase + u, y = to.rbase + u;
        a.um_p[y] = a.um_p[x]; a.um_wm[y] = a.um_wm[x]; a.um_wl[y] = a.um_wl[x]; a.um_wn[y] = a.um_wn[x];
        a.um_tm[y] = a.um_tm[x]; a.um_tl[y] = a.um_tl[x]; a.um_tn[y] = a.um_tn[x];
    }
    // bitmaps: the rows' (slots [0, n)) and the loadingPruned entries' ([0, L)), each over the slots
    for (uint32_t i = threadIdx.x; i < n * a.wordsB; i += blockDim.x) {
        const uint32_t sl = i / a.wordsB, w = i - sl * a.wordsB;
        a.bits[to.bbase + i] = w < a.words ? a.bits[from.bbase + (size_t)sl * a.words + w] : 0ull;
    }
    for (uint32_t i = threadIdx.x; i < L * a.wordsB; i += blockDim.x) {
        const uint32_t j = i / a.wordsB, w = i - j * a.wordsB;
        a.lp_bits[to.bbase + i] = w < a.words ? a.lp_bits[from.bbase + (size_t)j * a.words + w] : 0ull;
    }
    if (threadIdx.x == 0) a.kslot[key] = b;
}

}  // namespace ad
