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
#pragma once
#include "notify_kernels.h"

namespace ad {

constexpr int CS_T = 256;
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
};

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
// it and whose depsKnownBefore is above it -- except t itself and `skip` (the command being updated).
__device__ inline void cs_add_missing(const CfkStoreArgs& a, size_t base, uint32_t n, const Ts3& t, uint32_t ts,
                                      uint32_t skip_slot) {
    const uint32_t kt = cs_kind(t.lsb);
    for (uint32_t r = threadIdx.x; r < n; r += CS_T) {
        const size_t x = base + r;
        const uint32_t s = a.slot[x];
        if (s == ts || s == skip_slot || !cs_has_deps(a.st[x]) || !witnesses(cs_kind(a.tl[x]), kt)) continue;
        if (ts3_cmp(cs_dkb(a, x), t) > 0) {
            uint64_t* w = a.bits + ((size_t)(base + s)) * a.words + (ts >> 6);
            *w |= 1ull << (ts & 63);
        }
    }
    __syncthreads();
}
// Utils.removeFromMissingArrays (:70-95): slot ts leaves every missing set (it committed, or was invalidated)
__device__ inline void cs_remove_missing(const CfkStoreArgs& a, size_t base, uint32_t n, uint32_t ts) {
    for (uint32_t s = threadIdx.x; s < n; s += CS_T) a.bits[((size_t)(base + s)) * a.words + (ts >> 6)] &= ~(1ull << (ts & 63));
    __syncthreads();
}

// A new row at byId position p with a fresh slot (= the key's row count): TxnId t, status, executeAt, empty missing
__device__ inline uint32_t cs_insert(const CfkStoreArgs& a, size_t base, uint32_t& n, uint32_t p, const Ts3& t,
                                     uint32_t status, const Ts3& ex) {
    const uint32_t s = n;
    cs_shift_up(a, base, p, n);
    for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) a.bits[((size_t)(base + s)) * a.words + w] = 0ull;
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
static __global__ __launch_bounds__(CS_T) void k_cfk_apply(CfkStoreArgs a) {
    __shared__ uint64_t s_miss[CS_MAX_WORDS];
    __shared__ uint32_t s_add[CS_T];          // this event's additions (slots), CS_T at a time
    __shared__ uint32_t s_nadd;
    const uint32_t key = blockIdx.x;
    if (key >= a.K) return;
    const size_t base = (size_t)key * a.cap;
    uint32_t n = a.cnt[key];
    for (uint32_t e = a.ev_off[key]; e < a.ev_off[key + 1]; ++e) {
        const Ts3 t{a.etm[e], a.etl[e], a.etn[e]};
        const uint32_t ns = a.est[e];
        bool found;
        const uint32_t p = cs_find(a, base, n, t, found);
        const uint32_t cur = found ? a.st[base + p] : 0xFFu;
        if (found && ns <= cur) continue;                            // not a higher InternalStatus: no change
        const uint32_t d0 = a.dep_off[e], d1 = a.dep_off[e + 1];
        if (cs_has_deps(ns)) {
            const Ts3 ex{a.eem[e], a.eel[e], a.een[e]};
            const Ts3 dkb = cs_decided(ns) ? ex : t;
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
            // deps unknown to the CFK: TRANSITIVELY_KNOWN rows, in deps order
            if (threadIdx.x == 0) s_nadd = 0;
            __syncthreads();
            for (uint32_t j = d0; j < d1; ++j) {
                const Ts3 d{a.dtm[j], a.dtl[j], a.dtn[j]};
                if (j > d0 && ts3_cmp(Ts3{a.dtm[j - 1], a.dtl[j - 1], a.dtn[j - 1]}, d) >= 0) {
                    if (threadIdx.x == 0) *a.bad = 1u;
                    break;
                }
                bool f;
                const uint32_t q = cs_find(a, base, n, d, f);
                if (f) continue;
                if (n >= a.cap || s_nadd >= (uint32_t)CS_T) { if (threadIdx.x == 0) *a.overflow = 1u; a.cnt[key] = n; return; }
                const uint32_t s = cs_insert(a, base, n, q, d, AD_ST_TRANSITIVELY_KNOWN, d);
                if (threadIdx.x == 0) s_add[s_nadd++] = s;
                __syncthreads();
            }
            uint32_t ts;
            bool fnow;
            const uint32_t p2 = cs_find(a, base, n, t, fnow);           // t's position after the additions
            if (!fnow) {
                if (n >= a.cap) { if (threadIdx.x == 0) *a.overflow = 1u; a.cnt[key] = n; return; }
                ts = cs_insert(a, base, n, p2, t, ns, ex);
            } else {
                ts = a.slot[base + p2];
                if (threadIdx.x == 0) {
                    const size_t x = base + p2;
                    a.st[x] = (uint8_t)ns; a.em[x] = ex.msb; a.el[x] = ex.lsb; a.en[x] = ex.node;
                }
            }
            for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) a.bits[((size_t)(base + ts)) * a.words + w] = s_miss[w];
            __syncthreads();
            const uint32_t nadd = s_nadd;
            for (uint32_t k = 0; k < nadd; ++k) {
                const uint32_t s = s_add[k];
                bool f2;
                // the addition's TxnId: find its row through the slot (rows shifted since): a scan for the slot
                __shared__ uint32_t s_row;
                for (uint32_t r = threadIdx.x; r < n; r += CS_T) if (a.slot[base + r] == s) s_row = r;
                __syncthreads();
                const size_t x = base + s_row;
                const Ts3 ad{a.tm[x], a.tl[x], a.tn[x]};
                (void)f2;
                cs_add_missing(a, base, n, ad, s, ts);
            }
            if (!found && ns < AD_ST_COMMITTED) cs_add_missing(a, base, n, t, ts, 0xFFFFFFFFu);
            if (found && cur < AD_ST_COMMITTED && ns >= AD_ST_COMMITTED) cs_remove_missing(a, base, n, ts);
        } else {
            if (!found) {
                if (n >= a.cap) { if (threadIdx.x == 0) *a.overflow = 1u; a.cnt[key] = n; return; }
                const uint32_t ts = cs_insert(a, base, n, p, t, ns, t);
                if (ns != AD_ST_INVALID) cs_add_missing(a, base, n, t, ts, 0xFFFFFFFFu);
            } else {
                const uint32_t ts = a.slot[base + p];
                if (threadIdx.x == 0) {
                    const size_t x = base + p;
                    a.st[x] = (uint8_t)ns; a.em[x] = t.msb; a.el[x] = t.lsb; a.en[x] = t.node;
                }
                for (uint32_t w = threadIdx.x; w < a.words; w += CS_T) a.bits[((size_t)(base + ts)) * a.words + w] = 0ull;
                __syncthreads();
                if (cur < AD_ST_COMMITTED && ns == AD_ST_INVALID) cs_remove_missing(a, base, n, ts);
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) a.cnt[key] = n;
}

}  // namespace ad
