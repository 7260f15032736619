// history_kernels.h — a store's CommandsForKey state carried from one batch to the next (gfx950).
//
// A batch is the store's txns in TxnId (= arrival) order; the next batch continues that order.  Instead of a
// closed world per batch, the store keeps the CFK entries a later query can still see: after the deps stage,
// ad_cfk_retain marks every txn that, on some key, is not prunable for all later queries, and keeps those txns
// (their TxnId, executeAt, status and keys) on the device; the next ad_load_batch puts them in front of the new
// txns, with their global arrival ranks, and the whole pipeline runs over the combined rows.
//
// Prunable (Pruning.java:164-233 restated for final statuses; the oracle's FLAG_PRUNE, tests/test_oracle_prune.py):
// an entry j of key k is never emitted, nor counted, by any later mapReduceActive (CommandsForKey.java:925-983)
// when it is out of every later query's in-flight window (global rank < next - W) and either
//   * TRANSITIVELY_KNOWN / INVALID, or not in the CFK at all (unmanaged kinds): skipped outright, or
//   * a committed Read/Write executing before M_k = the greatest executeAt of the key's committed Writes that
//     execute before every later TxnId: maxCommittedWriteBefore(bound) >= M_k for every later bound, so the
//     elision (:951-962) drops it.  The Write achieving M_k is itself kept, so later prefix maxima still see it.
// A txn is kept when one of its entries is not prunable (keeping a txn's other, prunable entries changes no
// answer: they are elided or skipped where they sit).  MaxConflicts over the kept entries is unchanged too: every
// dropped entry executes below a kept one on its key.
#pragma once
#include "deps_kernels.h"

namespace ad {

// per key segment (indexed by its head position): greatest executeAt+1 of a committed Write executing at or
// before `last_ts` (the batch's last TxnId: every later TxnId is larger)
__global__ __launch_bounds__(256) void k_hist_seg_wmax(size_t P, const int32_t* __restrict__ seg_start,
                                                       const uint8_t* __restrict__ e_meta, const uint64_t* __restrict__ e_exec1,
                                                       uint64_t last_ts1, unsigned long long* __restrict__ segmax) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t m = e_meta[q];
    const uint64_t e = e_exec1[q];
    if (category(m) == CAT_ELIDABLE && meta_kind(m) == AD_KIND_WRITE && e <= last_ts1)
        atomicMax(segmax + seg_start[q], (unsigned long long)e);
}

__global__ __launch_bounds__(256) void k_hist_keep(size_t P, const int32_t* __restrict__ seg_start,
                                                   const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                                   const uint64_t* __restrict__ e_exec1, const unsigned long long* __restrict__ segmax,
                                                   const uint32_t* __restrict__ gid, uint64_t window_lo, uint8_t* __restrict__ keep) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t j = e_txn[q];
    const uint64_t gj = gid ? gid[j] : j;
    bool k = gj >= window_lo;                           // in flight for some later query
    if (!k) {
        const uint32_t c = category(e_meta[q]);
        const bool prunable = c == CAT_SKIP || (c == CAT_ELIDABLE && e_exec1[q] < segmax[seg_start[q]]);
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
__global__ __launch_bounds__(256) void k_hist_gather_rows(HistGather g) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= g.H) return;
    const uint32_t r = g.rows[x];
    g.otm[x] = g.tm[r]; g.otl[x] = g.tl[r]; g.otn[x] = g.tn[r];
    g.oem[x] = g.em[r]; g.oel[x] = g.el[r]; g.oen[x] = g.en[r];
    g.ost[x] = g.st[r];
    g.ocnt[x] = g.key_off[r + 1] - g.key_off[r];
    g.ogid[x] = g.gid ? g.gid[r] : r;
}
__global__ __launch_bounds__(256) void k_hist_gather_keys(size_t H, const uint32_t* __restrict__ rows,
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
__global__ __launch_bounds__(256) void k_hist_new_rows(size_t H, size_t n, uint64_t next, uint32_t hp,
                                                       uint32_t* __restrict__ gid, uint32_t* __restrict__ key_off) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) gid[H + i] = (uint32_t)(next + i);
    if (i <= n) key_off[H + i] += hp;
}

}  // namespace ad
