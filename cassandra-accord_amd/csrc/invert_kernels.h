// invert_kernels.h — the txn -> keys inverse of batched Deps CSRs.
//
// Replaces RelationMultiMap.invert (utils/RelationMultiMap.java:907-938) as KeyDeps.txnIdsToKeys
// (primitives/KeyDeps.java:362-367) and RangeDeps.txnIdsToRanges (primitives/RangeDeps.java:576-582) build it
// lazily per Deps: from keysToTxnIds (nKeys end offsets, then per key its ascending TxnId indices) to
// txnIdsToKeys (nTxnIds end offsets based at nTxnIds, then per TxnId its ascending key indices).
//
// The reference inverts one Deps at a time with a counting sort.  Here every txn of a row window is inverted at
// once as ONE stable sort: each (txn i, key k, TxnId index t) entry becomes the pair (global TxnId slot
// tb[i] + t, k), emitted in keysToTxnIds order — ascending (i, k) — so a stable LSD radix sort by the slot
// leaves every slot's keys ascending (radix_sort.h).  In the sorted array txn i's entries occupy
// [eb[i], eb[i+1]) (the slot order keeps txns in order), and txn i's inverse lives at off[i] = tb[i] + eb[i]:
//   header  out[off[i] + t] = nt_i + (upper_bound(slots in txn i's entries, tb[i] + t) - eb[i])
//   body    out[off[i] + nt_i + (q - eb[i])] = out[tb[i + 1] + q] = key of sorted entry q
// A TxnId index without entries (legal in SerializerSupport input, never produced by the builder) gets an empty
// run, as the reference's cursor loop gives it.  All integer, HBM-streaming except the per-slot binary searches.
#pragma once
#include "common.h"

namespace ad {

struct InvArgs {
    size_t m;                 // rows in the window
    size_t lo;                // first row
    const uint32_t *key_off, *k2t_off, *tcnt;
    const int32_t* k2t;
    uint32_t *nt, *ne;        // [m] per-row TxnId count, entry count
    const uint32_t *tb, *eb;  // [m + 1] exclusive scans of nt / ne
    uint32_t *skey, *sval;    // [E] (slot, key index) pairs
    uint32_t* bad;            // [0] an entry's TxnId index is out of range (malformed CSR)
    int32_t* out;
    size_t total_nt, E;
};

static __global__ __launch_bounds__(256) void k_inv_counts(InvArgs a) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.m) return;
    const size_t r = a.lo + i;
    const uint32_t nk = a.key_off[r + 1] - a.key_off[r];
    const uint32_t len = a.k2t_off[r + 1] - a.k2t_off[r];
    a.nt[i] = a.tcnt[r];
    a.ne[i] = len > nk ? len - nk : 0u;
}

// one wave per row: lanes over the row's entries; an entry's key = how many key end offsets are <= its
// position (binary search over the row's nk end offsets, which start at nk: KeyDeps.java:153-169)
static __global__ __launch_bounds__(256) void k_inv_expand(InvArgs a) {
    const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    const uint32_t lane = threadIdx.x % WAVE;
    if (i >= a.m) return;
    const size_t r = a.lo + i;
    const uint32_t nk = a.key_off[r + 1] - a.key_off[r];
    const int32_t* src = a.k2t + a.k2t_off[r];
    const uint32_t ne = a.ne[i], nt = a.nt[i], tbase = a.tb[i], ebase = a.eb[i];
    bool b = false;
    for (uint32_t j = lane; j < ne; j += WAVE) {
        const uint32_t pos = nk + j;
        uint32_t lo = 0, hi = nk;                      // first key whose end offset > pos
        while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if ((uint32_t)src[mid] <= pos) lo = mid + 1; else hi = mid; }
        const int32_t t = src[pos];
        b |= t < 0 || (uint32_t)t >= nt;
        a.skey[ebase + j] = tbase + (uint32_t)(t < 0 ? 0 : (uint32_t)t < nt ? t : nt - 1);
        a.sval[ebase + j] = lo;
    }
    wave_set_flag(b, a.bad);
}

// the row holding global TxnId slot g: tb[row] <= g < tb[row + 1]
__device__ inline size_t inv_row_of(const uint32_t* tb, size_t m, uint32_t g) {
    size_t lo = 0, hi = m;
    while (lo < hi) { const size_t mid = (lo + hi) >> 1; if (tb[mid + 1] <= g) lo = mid + 1; else hi = mid; }
    return lo;
}

static __global__ __launch_bounds__(256) void k_inv_body(InvArgs a, const uint32_t* __restrict__ sk,
                                                         const uint32_t* __restrict__ sv) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.E) return;
    const size_t row = inv_row_of(a.tb, a.m, sk[q]);
    a.out[a.tb[row + 1] + q] = (int32_t)sv[q];
}

static __global__ __launch_bounds__(256) void k_inv_header(InvArgs a, const uint32_t* __restrict__ sk) {
    const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= a.total_nt) return;
    const size_t row = inv_row_of(a.tb, a.m, (uint32_t)g);
    const uint32_t tbase = a.tb[row], nt = a.tb[row + 1] - tbase;
    uint32_t lo = a.eb[row], hi = a.eb[row + 1];        // first sorted entry of the row with slot > g
    while (lo < hi) { const uint32_t mid = (lo + hi) >> 1; if (sk[mid] <= (uint32_t)g) lo = mid + 1; else hi = mid; }
    a.out[(size_t)tbase + a.eb[row] + (g - tbase)] = (int32_t)(nt + lo - a.eb[row]);
}

}  // namespace ad
