// history_kernels.h — a store's CommandsForKey state carried from one batch to the next (gfx950).
//
// A batch is the store's txns in TxnId (= arrival) order; the next batch continues that order.  Instead of a
// closed world per batch, the store keeps the CFK entries a later query can still see: after the deps stage,
// ad_cfk_retain marks every txn that, on some key, is not prunable for all later queries, and keeps those txns
// (their TxnId, executeAt, status and keys) on the device; the next ad_load_batch puts them in front of the new
// txns, with their global arrival ranks, and the whole pipeline runs over the combined rows.
//
// The statuses of kept rows are current: ad_cfk_update moves them along CommandsForKeyTest's transition table
// (Commit, Stable, Apply, Invalidate) between batches, and the levels over a batch with history treat APPLIED /
// INVALID rows as done.  So a row is dropped only when nothing can need it again (Pruning.java:164-233 prunes
// applied txns below an applied Write): it is out of every later query's in-flight window (global rank <
// next - W) and on every key either
//   * INVALID (terminal, skipped by mapReduceActive and by the execution order), or
//   * APPLIED and never seen again by a later mapReduceActive (CommandsForKey.java:925-983): not in the CFK at
//     all (unmanaged kinds), or a Read/Write executing before M_k = the greatest executeAt of the key's
//     committed Writes that execute before every later TxnId — maxCommittedWriteBefore(bound) >= M_k for every
//     later bound, so the elision (:951-962) drops it.  The Write achieving M_k is itself kept.
// TRANSITIVELY_KNOWN rows are kept (they may still be preaccepted), and so are committed rows that have not
// applied (they still execute and constrain the order).  A txn is kept when one of its entries is not
// prunable (keeping a txn's other, prunable entries changes no answer: they are elided or skipped where they
// sit).  MaxConflicts over the kept entries is unchanged too: every dropped entry executes below a kept one on
// its key.
#pragma once
#include "deps_kernels.h"

namespace ad {

// per key segment (indexed by its head position): greatest executeAt+1 of a committed Write executing at or
// before `last_ts` (the batch's last TxnId: every later TxnId is larger)
static __global__ __launch_bounds__(256) void k_hist_seg_wmax(size_t P, const int32_t* __restrict__ seg_start,
                                                       const uint8_t* __restrict__ e_meta, const uint64_t* __restrict__ e_exec1,
                                                       uint64_t last_ts1, unsigned long long* __restrict__ segmax) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t m = e_meta[q];
    const uint64_t e = e_exec1[q];
    if (category(m) == CAT_ELIDABLE && meta_kind(m) == AD_KIND_WRITE && e <= last_ts1)
        atomicMax(segmax + seg_start[q], (unsigned long long)e);
}

static __global__ __launch_bounds__(256) void k_hist_keep(size_t P, const int32_t* __restrict__ seg_start,
                                                   const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                                   const uint64_t* __restrict__ e_exec1, const unsigned long long* __restrict__ segmax,
                                                   const uint32_t* __restrict__ gid, uint64_t window_lo, uint8_t* __restrict__ keep) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t j = e_txn[q];
    const uint64_t gj = gid ? gid[j] : j;
    bool k = gj >= window_lo;                           // in flight for some later query
    if (!k) {
        const uint32_t m = e_meta[q], st = meta_status(m), c = category(m);
        const bool prunable = st == AD_ST_INVALID ||
                              (st == AD_ST_APPLIED && (c == CAT_SKIP || (c == CAT_ELIDABLE && e_exec1[q] < segmax[seg_start[q]])));
        k = !prunable;
    }
    if (k) keep[j] = 1;                                 // every writer stores the same value
}

// kept rows -> the history arrays (row-wise fields and the per-row key counts)
struct HistGather {
    size_t H;
    const uint32_t* rows;
    const uint64_t *tm, *tl, *em, *el;
    const int32_t *tn, *en;
    const uint8_t* st;
    const uint32_t* key_off;
    const uint32_t* gid;                                // nullable: rows are global ranks
    uint64_t *otm, *otl, *oem, *oel;
    int32_t *otn, *oen;
    uint8_t* ost;
    uint32_t* ocnt;                                     // [H] keys per kept row
    uint32_t* ogid;
};
static __global__ __launch_bounds__(256) void k_hist_gather_rows(HistGather g) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= g.H) return;
    const uint32_t r = g.rows[x];
    g.otm[x] = g.tm[r]; g.otl[x] = g.tl[r]; g.otn[x] = g.tn[r];
    g.oem[x] = g.em[r]; g.oel[x] = g.el[r]; g.oen[x] = g.en[r];
    g.ost[x] = g.st[r];
    g.ocnt[x] = g.key_off[r + 1] - g.key_off[r];
    g.ogid[x] = g.gid ? g.gid[r] : r;
}
static __global__ __launch_bounds__(256) void k_hist_gather_keys(size_t H, const uint32_t* __restrict__ rows,
                                                          const uint32_t* __restrict__ key_off, const uint64_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ okoff, uint64_t* __restrict__ okeys) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= H) return;
    const uint32_t r = rows[x];
    const uint32_t b = key_off[r], e = key_off[r + 1];
    uint32_t o = okoff[x];
    for (uint32_t p = b; p < e; ++p) okeys[o++] = keys[p];
}

// the next batch: rows [H, H + n) get global ranks next + i, their key offsets shift past the history's keys
static __global__ __launch_bounds__(256) void k_hist_new_rows(size_t H, size_t n, uint64_t next, uint32_t hp,
                                                       uint32_t* __restrict__ gid, uint32_t* __restrict__ key_off) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) gid[H + i] = (uint32_t)(next + i);
    if (i <= n) key_off[H + i] += hp;
}

// ---- status transitions of kept rows between batches (ad_cfk_update) --------------------------------------
// CommandsForKeyTest's transition table (CommandsForKeyTest.java:235-246) over CommandsForKey.InternalStatus
// (CommandsForKey.java:493-611): NotDefined -> PreAccepted / AcceptedInvalidate / Accepted / Committed / Stable /
// Invalidated; PreAccepted -> AcceptedInvalidate / Accepted / Committed / Stable / Invalidated; Accepted ->
// Committed / Stable / Invalidated; AcceptedInvalidate -> Invalidated; Committed -> Stable; Stable -> Applied.
// AcceptedInvalidate is PREACCEPTED_OR_ACCEPTED_INVALIDATE internally, so PREACCEPTED -> PREACCEPTED is allowed.
// executeAt: given with ACCEPTED / COMMITTED / STABLE (>= TxnId), fixed from COMMITTED on.
enum : uint32_t { CU_OK = 0, CU_NOT_HELD = 1, CU_TRANSITION = 2, CU_EXECUTE_AT = 3 };
__host__ __device__ inline bool cfk_transition_ok(uint32_t from, uint32_t to) {
    switch (from) {
        case AD_ST_TRANSITIVELY_KNOWN:
            return to == AD_ST_PREACCEPTED || to == AD_ST_ACCEPTED || to == AD_ST_COMMITTED || to == AD_ST_STABLE || to == AD_ST_INVALID;
        case AD_ST_PREACCEPTED:
            return to == AD_ST_PREACCEPTED || to == AD_ST_ACCEPTED || to == AD_ST_COMMITTED || to == AD_ST_STABLE || to == AD_ST_INVALID;
        case AD_ST_ACCEPTED: return to == AD_ST_COMMITTED || to == AD_ST_STABLE || to == AD_ST_INVALID;
        case AD_ST_COMMITTED: return to == AD_ST_STABLE;
        case AD_ST_STABLE: return to == AD_ST_APPLIED;
        default: return false;                       // HISTORICAL, APPLIED, INVALID: no further transition
    }
}
// Timestamp.compareTo (Timestamp.java:208-217): msb unsigned, lsb >>> 16, identity flags, node signed
__device__ inline int ts3_cmp(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn) {
    if (am != bm) return am < bm ? -1 : 1;
    if ((al >> 16) != (bl >> 16)) return (al >> 16) < (bl >> 16) ? -1 : 1;
    if ((al & 0x1E) != (bl & 0x1E)) return (al & 0x1E) < (bl & 0x1E) ? -1 : 1;
    return an < bn ? -1 : (an > bn ? 1 : 0);
}
struct CfkUpdate {
    size_t m, H;
    const uint32_t* ugid;                 // [m] ascending global ranks
    const uint8_t* ust;                   // [m] new InternalStatus
    const uint64_t *um, *ul;              // [m] new executeAt (nullable)
    const int32_t* un;
    const uint32_t* hgid;                 // [H] kept rows' global ranks (ascending)
    const uint64_t *htm, *htl;
    const int32_t* htn;
    uint8_t* hst;
    uint64_t *hem, *hel;
    int32_t* hen;
    uint32_t* row;                        // [m] kept row, or CU_* reason | 0x80000000
    uint32_t* bad;                        // [0] some update is refused
};
static __global__ __launch_bounds__(256) void k_cfk_update_check(CfkUpdate a) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool b = false;
    if (i < a.m) {
        const uint32_t g = a.ugid[i];
        size_t lo = 0, hi = a.H;
        while (lo < hi) { const size_t h = (lo + hi) >> 1; if (a.hgid[h] < g) lo = h + 1; else hi = h; }
        uint32_t why = CU_OK;
        if (lo == a.H || a.hgid[lo] != g) {
            why = CU_NOT_HELD;
        } else {
            const uint32_t from = a.hst[lo], to = a.ust[i];
            if (!cfk_transition_ok(from, to)) {
                why = CU_TRANSITION;
            } else if (a.um) {
                const bool fixed = from == AD_ST_COMMITTED || from == AD_ST_STABLE;
                const bool decided = to == AD_ST_ACCEPTED || to == AD_ST_COMMITTED || to == AD_ST_STABLE || to == AD_ST_APPLIED;
                if (fixed && ts3_cmp(a.um[i], a.ul[i], a.un[i], a.hem[lo], a.hel[lo], a.hen[lo]) != 0) why = CU_EXECUTE_AT;
                if (decided && ts3_cmp(a.um[i], a.ul[i], a.un[i], a.htm[lo], a.htl[lo], a.htn[lo]) < 0) why = CU_EXECUTE_AT;
            }
        }
        a.row[i] = why == CU_OK ? (uint32_t)lo : (0x80000000u | why);
        b = why != CU_OK;
    }
    wave_set_flag(b, a.bad);
}
static __global__ __launch_bounds__(256) void k_cfk_update_apply(CfkUpdate a) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.m) return;
    const uint32_t r = a.row[i];
    const uint32_t from = a.hst[r], to = a.ust[i];
    a.hst[r] = to;
    // executeAt is written only where the move decides it: not for PREACCEPTED / INVALID (no executeAt,
    // CommandsForKey.InternalStatus.hasExecuteAtOrDeps), and not once it is fixed (COMMITTED / STABLE: the check
    // proved the given one compares equal; the stored raw bits, flags included, stay)
    const bool fixed = from == AD_ST_COMMITTED || from == AD_ST_STABLE;
    const bool decided = to == AD_ST_ACCEPTED || to == AD_ST_COMMITTED || to == AD_ST_STABLE || to == AD_ST_APPLIED;
    if (a.um && decided && !fixed) { a.hem[r] = a.um[i]; a.hel[r] = a.ul[i]; a.hen[r] = a.un[i]; }
}

}  // namespace ad
