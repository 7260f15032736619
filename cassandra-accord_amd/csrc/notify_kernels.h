// notify_kernels.h — CommandsForKey's execution release rule over CFK states in their serialized layout.
//
// Replaces CommandsForKey.notifyManaged (local/cfk/CommandsForKey.java:1208-1289), run over the whole of
// committedByExecuteAt with every kind admitted: the STABLE Read/Write txns of a key that are no longer waiting on it.
// The reference walks committedByExecuteAt from the last applied Write, stops after the first unapplied Write, and
// lets a STABLE txn go when the count of undecided lower-TxnId txns it conflicts with, plus the unapplied committed
// ones before it, equals the count of its `missing` entries from minUndecided on (:1237-1280).  The scan is sequential;
// its outcome is a set of order statistics, so one workgroup per key computes it without sorting anything:
//   maxAW  = the greatest executeAt of an APPLIED Write                      (maxAppliedWriteByExecuteAt, :671-678)
//   W*     = the least executeAt above maxAW of an unapplied Write           (the scan's stopping point, :1286-1287)
//   R*     = unapplied committed Reads with executeAt in (maxAW, W*)         (counters before W*, :1285)
//   und(e) = undecided Read / Write rows (status < COMMITTED) with TxnId < e  (the byId backfill, :1237-1247): a
//            prefix count over byId, read at the first row with TxnId >= e (binary search)
//   miss   = the txn's missing entries at or after minUndecided that are Reads / Writes (:1256-1272)
// A STABLE Read/Write txn T with maxAW < e_T <= W* is released iff
//   Read:  und_writes(e_T)      == miss_T      (unappliedCount: the Write count, :1326-1327)
//   Write: R* + und_rw(e_T)     == miss_T      (only W* itself can be an eligible STABLE Write)
// Rows: byId order (TxnId strictly ascending) per key; executeAt is read only for ACCEPTED..APPLIED rows, so an
// undecided row's executeAt may be anything (the release rule never needs it).
#pragma once
#include "conflict_kernels.h"

namespace ad {

struct NotifyArgs {
    size_t K;                                // keys (CFK states)
    const uint32_t* row_off;                 // [K + 1]
    const uint64_t *tm, *tl, *em, *el;       // [rows] TxnId, executeAt
    const int32_t *tn, *en;
    const uint8_t* st;                       // [rows] InternalStatus
    const uint32_t* miss_off;                // [rows + 1] missing CSR
    const uint32_t* miss;                    // segment-relative row indices
    uint32_t* pre;                           // [2 * rows] scratch: per row the undecided Writes / Reads+Writes below it
    uint8_t* out;                            // [rows] 1: notWaiting on this key
    uint32_t* bad_order;                     // TxnIds not strictly ascending within a key
    uint32_t* bad_miss;                      // a missing index outside its key / not below its txn's bound
    // device-resident store (cfk_store_kernels.h; row_off == nullptr): key k's rows are [k * cap, k * cap + cnt[k]),
    // missing() as a bitmap over the key's slots (bits[(k * cap + slot) * words ...]) instead of the CSR
    const uint32_t* cnt;
    uint32_t cap, words;
    const uint32_t* kslot;                   // two-tier stores: per key its large-tier slot (or ~0u); nullptr: one tier
    uint32_t capB, wordsB;
    const uint32_t* slot;
    const uint64_t* bits;
    // the store's loadingPruned tables (nullptr: none): a STABLE txn that witnessed a pruned Read / Write TxnId below its
    // executeAt that is still loading is not released (Pruning.isWaitingOnPruned, Pruning.java:119-135; :1222)
    const uint32_t* lp_cnt;
    const uint64_t *lpm, *lpl;
    const int32_t* lpn;
    const uint64_t* lp_bits;
};
constexpr uint32_t NF_MAX_WORDS = 256;       // the bitmap reader: at most 16384 rows per key

// A device store's key region (cfk_store_kernels.h): the K keys' regular tier (cap rows, words-word bitmaps each) first,
// then the large tier (capB rows, wordsB-word bitmaps per slot) that keys outgrowing cap move to.  Rows, loadingPruned
// and registry rows at rbase; missing() / witness bitmaps at bbase, one bitmap row of `words` words per slot.
struct CsTier { size_t rbase, bbase; uint32_t cap, words; };
__device__ inline CsTier cs_tier(uint32_t key, size_t K, uint32_t cap, uint32_t words, const uint32_t* kslot, uint32_t capB,
                                 uint32_t wordsB) {
    const uint32_t b = kslot ? kslot[key] : 0xFFFFFFFFu;
    if (b == 0xFFFFFFFFu) return CsTier{(size_t)key * cap, (size_t)key * cap * words, cap, words};
    const size_t r0 = K * cap;
    return CsTier{r0 + (size_t)b * capB, r0 * words + (size_t)b * capB * wordsB, capB, wordsB};
}

__device__ inline bool nf_rw(uint64_t lsb) {             // managesExecution: key-domain Read / Write
    const uint32_t k = (uint32_t)(lsb >> 1) & 7u;
    return (lsb & 1ull) == 0 && (k == AD_KIND_READ || k == AD_KIND_WRITE);
}
__device__ inline bool nf_write(uint64_t lsb) { return (lsb & 1ull) == 0 && ((uint32_t)(lsb >> 1) & 7u) == AD_KIND_WRITE; }
__device__ inline bool nf_read(uint64_t lsb) { return (lsb & 1ull) == 0 && ((uint32_t)(lsb >> 1) & 7u) == AD_KIND_READ; }

constexpr int NF_T = 256;

// block-wide fold of one Ts3 (has flag) with `better(a, b)` = a should replace b
template <bool MAX>
__device__ inline void nf_block_fold(Ts3& v, bool& has, Ts3* s_v, int* s_h) {
    const int tid = threadIdx.x;
    s_v[tid] = v; s_h[tid] = has;
    __syncthreads();
    for (int o = NF_T / 2; o > 0; o >>= 1) {
        if (tid < o && s_h[tid + o]) {
            const int c = s_h[tid] ? ts3_cmp(s_v[tid + o], s_v[tid]) : (MAX ? 1 : -1);
            if (MAX ? c > 0 : c < 0) { s_v[tid] = s_v[tid + o]; s_h[tid] = 1; }
        }
        __syncthreads();
    }
    v = s_v[0]; has = s_h[0];
    __syncthreads();
}

static __global__ __launch_bounds__(NF_T) void k_cfk_notify(NotifyArgs a) {
    __shared__ Ts3 s_v[NF_T];
    __shared__ int s_h[NF_T];
    __shared__ uint32_t s_c[NF_T];
    __shared__ uint32_t s_c2[NF_T];
    const size_t key = blockIdx.x;
    if (key >= a.K) return;
    const int tid = threadIdx.x;
    const CsTier tr = cs_tier((uint32_t)key, a.K, a.cap, a.words, a.row_off ? nullptr : a.kslot, a.capB, a.wordsB);
    const size_t lo = a.row_off ? a.row_off[key] : tr.rbase;
    const size_t hi = a.row_off ? a.row_off[key + 1] : lo + a.cnt[key];
    const uint32_t L = (uint32_t)(hi - lo);
    const uint32_t words = tr.words;
    __shared__ uint64_t s_mask[NF_MAX_WORDS];
    // pass 1: maxAW, order check, minUndecided
    Ts3 maw{0, 0, 0};
    bool has_maw = false, bad = false, bad_m = false;
    uint32_t minund = L;
    for (uint32_t r = tid; r < L; r += NF_T) {
        const size_t x = lo + r;
        const uint8_t s = a.st[x];
        const uint64_t lsb = a.tl[x];
        if (s == AD_ST_APPLIED && nf_write(lsb)) {
            const Ts3 e{a.em[x], a.el[x], a.en[x]};
            if (!has_maw || ts3_cmp(e, maw) > 0) { maw = e; has_maw = true; }
        }
        if (s < AD_ST_COMMITTED && nf_rw(lsb) && r < minund) minund = r;
        if (r > 0 && ts3_cmp(Ts3{a.tm[x - 1], a.tl[x - 1], a.tn[x - 1]}, Ts3{a.tm[x], lsb, a.tn[x]}) >= 0) bad = true;
    }
    nf_block_fold<true>(maw, has_maw, s_v, s_h);
    s_c[tid] = minund;
    __syncthreads();
    for (int o = NF_T / 2; o > 0; o >>= 1) {
        if (tid < o && s_c[tid + o] < s_c[tid]) s_c[tid] = s_c[tid + o];
        __syncthreads();
    }
    minund = s_c[0];
    __syncthreads();
    // pass 2: W* = least executeAt above maxAW of an unapplied committed Write
    Ts3 ws{0, 0, 0};
    bool has_ws = false;
    for (uint32_t r = tid; r < L; r += NF_T) {
        const size_t x = lo + r;
        const uint8_t s = a.st[x];
        if ((s == AD_ST_COMMITTED || s == AD_ST_STABLE) && nf_write(a.tl[x])) {
            const Ts3 e{a.em[x], a.el[x], a.en[x]};
            if ((!has_maw || ts3_cmp(e, maw) > 0) && (!has_ws || ts3_cmp(e, ws) < 0)) { ws = e; has_ws = true; }
        }
    }
    nf_block_fold<false>(ws, has_ws, s_v, s_h);
    // pass 3: R* and the undecided prefix counts over byId (exclusive; Writes, Reads + Writes)
    uint32_t rstar = 0, carry_w = 0, carry_rw = 0;
    for (uint32_t base = 0; base < L; base += NF_T) {
        const uint32_t r = base + tid;
        uint32_t uw = 0, urw = 0;
        if (r < L) {
            const size_t x = lo + r;
            const uint8_t s = a.st[x];
            const uint64_t lsb = a.tl[x];
            if (s < AD_ST_COMMITTED && nf_rw(lsb)) { urw = 1; uw = nf_write(lsb) ? 1 : 0; }
            if ((s == AD_ST_COMMITTED || s == AD_ST_STABLE) && nf_read(lsb)) {
                const Ts3 e{a.em[x], a.el[x], a.en[x]};
                if ((!has_maw || ts3_cmp(e, maw) > 0) && (!has_ws || ts3_cmp(e, ws) < 0)) ++rstar;
            }
        }
        // block exclusive scans of uw and urw (Hillis-Steele in LDS)
        s_c[tid] = uw; s_c2[tid] = urw;
        __syncthreads();
        for (int o = 1; o < NF_T; o <<= 1) {
            const uint32_t yw = tid >= o ? s_c[tid - o] : 0u, yrw = tid >= o ? s_c2[tid - o] : 0u;
            __syncthreads();
            s_c[tid] += yw; s_c2[tid] += yrw;
            __syncthreads();
        }
        if (r < L) {
            const uint32_t ew = carry_w + s_c[tid] - uw, erw = carry_rw + s_c2[tid] - urw;
            a.pre[(lo + r) * 2] = ew;
            a.pre[(lo + r) * 2 + 1] = erw;
        }
        carry_w += s_c[NF_T - 1]; carry_rw += s_c2[NF_T - 1];
        __syncthreads();
    }
    s_c[tid] = rstar;
    __syncthreads();
    for (int o = NF_T / 2; o > 0; o >>= 1) {
        if (tid < o) s_c[tid] += s_c[tid + o];
        __syncthreads();
    }
    rstar = s_c[0];
    __syncthreads();
    // bitmap reader: the slots whose missing bit counts -- Read / Write rows at or after minUndecided
    if (a.bits) {
        for (uint32_t w = tid; w < words; w += NF_T) s_mask[w] = 0ull;
        __syncthreads();
        for (uint32_t r = tid; r < L; r += NF_T)
            if (r >= (minund == L ? 0u : minund) && nf_rw(a.tl[lo + r])) {
                const uint32_t sl = a.slot[lo + r];
                atomicOr((unsigned long long*)&s_mask[sl >> 6], 1ull << (sl & 63));
            }
        __syncthreads();
    }
    // pass 4: per STABLE Read / Write row, the release test
    for (uint32_t r = tid; r < L; r += NF_T) {
        const size_t x = lo + r;
        uint8_t rel = 0;
        const uint8_t s = a.st[x];
        const uint64_t lsb = a.tl[x];
        // missing indices must lie in the segment
        if (!a.bits)
            for (uint32_t m = a.miss_off[x]; m < a.miss_off[x + 1]; ++m) if (a.miss[m] >= L) bad_m = true;
        if (s == AD_ST_STABLE && nf_rw(lsb)) {
            const Ts3 e{a.em[x], a.el[x], a.en[x]};
            const bool eligible = (!has_maw || ts3_cmp(e, maw) > 0) && (!has_ws || ts3_cmp(e, ws) <= 0);
            if (eligible) {
                uint32_t blo = 0, bhi = L;                 // first byId row with TxnId >= executeAt
                while (blo < bhi) {
                    const uint32_t mid = (blo + bhi) >> 1;
                    const size_t y = lo + mid;
                    if (ts3_cmp(Ts3{a.tm[y], a.tl[y], a.tn[y]}, e) < 0) blo = mid + 1; else bhi = mid;
                }
                const uint32_t und_w = blo < L ? a.pre[(lo + blo) * 2] : carry_w;
                const uint32_t und_rw = blo < L ? a.pre[(lo + blo) * 2 + 1] : carry_rw;
                const uint32_t expect = nf_write(lsb) ? rstar + und_rw : und_w;
                uint32_t mc = 0;
                if (a.bits) {
                    const uint64_t* row = a.bits + tr.bbase + (size_t)a.slot[x] * words;
                    for (uint32_t w = 0; w < words; ++w) mc += (uint32_t)__popcll(row[w] & s_mask[w]);
                } else {
                    for (uint32_t m = a.miss_off[x]; m < a.miss_off[x + 1]; ++m) {
                        const uint32_t j = a.miss[m];
                        if (j < L && j >= (minund == L ? 0u : minund) && nf_rw(a.tl[lo + j])) ++mc;   // minUndecided null: from 0
                    }
                }
                rel = expect == mc ? 1 : 0;
                if (rel && a.lp_cnt) {
                    const size_t lb = tr.rbase;
                    const uint32_t sl = a.slot[x];
                    for (uint32_t j = 0; j < a.lp_cnt[key]; ++j)
                        if (nf_rw(a.lpl[lb + j]) && ts3_cmp(Ts3{a.lpm[lb + j], a.lpl[lb + j], a.lpn[lb + j]}, e) < 0 &&
                            ((a.lp_bits[tr.bbase + (size_t)j * words + (sl >> 6)] >> (sl & 63)) & 1ull)) { rel = 0; break; }
                }
            }
        }
        a.out[x] = rel;
    }
    if (bad && *(volatile uint32_t*)a.bad_order == 0u) *(volatile uint32_t*)a.bad_order = 1u;
    if (bad_m && *(volatile uint32_t*)a.bad_miss == 0u) *(volatile uint32_t*)a.bad_miss = 1u;
}

}  // namespace ad
