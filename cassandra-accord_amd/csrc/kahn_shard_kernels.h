// kahn_shard_kernels.h — execution levels of a key-range sharded batch as distributed Kahn wavefronts
// (round 4, one exchange per wave since round 5).
//
// Every execution constraint is local to one store (global_levels.h): an (a) key-chain edge lives with the key's
// store, a (b) direct / range dependency edge and a (c) unmanaged chain bound with a store whose slice both ends
// touch.  So a txn's level is 1 + the greatest level of its predecessors over the stores that hold it: it is
// released at wave l once EVERY holder has released all of its local predecessors by wave l - 1.  Per wave l:
//   1. exchange: every store's READY(txn) messages reach the txn's holders (the store itself included: its own
//      region is a device copy);
//   2. every holder counts the READYs of its rows; a row whose count reaches its txn's holder count is released at
//      level l -- on every holder in the same wave, since every holder receives the same READYs -- its local
//      successors' remaining in-degrees drop, and those reaching zero send READY to all of their txn's holders
//      (wave l + 1's messages).
// Waves stop at the first exchange that moves nothing anywhere (every store sees the same count matrix).  One
// exchange and one host synchronisation (the count all-gather that sizes the receives) per wave; the round-4 protocol
// sent READY to one coordinating holder and RELEASE back (two exchanges and four host round trips per wave).  A txn
// costs holders x holders READYs over the batch (holders x (holders - 1) over the network).  Messages are u64 (global
// rank in the low word); the region for destination d holds at most one READY per local row d also holds, so appends
// never overflow.
#pragma once
#include "shard_kernels.h"

namespace ad {

constexpr uint32_t KS_UNRELEASED = 0xFFFFFFFFu;

// One message per lane to the region of `dest` (wave-aggregated append; every lane of the wave must call it).
__device__ inline void ks_append(bool want, uint32_t dest, uint64_t msg, const uint32_t* __restrict__ base,
                                 uint32_t* __restrict__ cnt, uint64_t* __restrict__ out) {
    const int lane = (int)__lane_id();
#pragma unroll
    for (int d = 0; d < MAX_STORES; ++d) {
        const bool w = want && dest == (uint32_t)d;
        const uint64_t b = __ballot(w);
        if (!b) continue;
        const int leader = __ffsll((unsigned long long)b) - 1;
        uint32_t at = 0;
        if (lane == leader) at = atomicAdd(cnt + d, (uint32_t)__popcll(b));
        at = __builtin_amdgcn_readlane(at, leader);
        if (w) out[base[d] + at + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = msg;
    }
}

// local row of global rank g (rows ascend by global rank); n if absent
__device__ inline size_t ks_row(const uint32_t* __restrict__ gid, size_t n, uint32_t g) {
    size_t lo = 0, hi = n;
    while (lo < hi) { const size_t m = (lo + hi) >> 1; if (gid[m] < g) lo = m + 1; else hi = m; }
    return (lo < n && gid[lo] == g) ? lo : n;
}

// READY(g) of row r to every holder of its txn (this store included), one wave-aggregated append per destination
__device__ inline void ks_ready_all(bool want, uint32_t holders, uint64_t msg, const uint32_t* __restrict__ base,
                                    uint32_t* __restrict__ cnt, uint64_t* __restrict__ out) {
#pragma unroll
    for (int d = 0; d < MAX_STORES; ++d) ks_append(want && ((holders >> d) & 1u), (uint32_t)d, msg, base, cnt, out);
}

// Wave 0: every row starts unreleased; rows without local predecessors are ready.
static __global__ __launch_bounds__(256) void k_ks_init(size_t n, const uint32_t* __restrict__ gid, const uint8_t* __restrict__ holders,
                                                 const uint32_t* __restrict__ rem, uint32_t* __restrict__ lvl,
                                                 uint32_t* __restrict__ rcnt, const uint32_t* __restrict__ base,
                                                 uint32_t* __restrict__ cnt, uint64_t* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool want = false;
    uint32_t hm = 0;
    uint64_t msg = 0;
    if (i < n) {
        lvl[i] = KS_UNRELEASED;
        rcnt[i] = 0;
        if (rem[i] == 0) { want = true; hm = holders[i]; msg = gid[i]; }
    }
    ks_ready_all(want, hm, msg, base, cnt, out);
}

// One wave: the READYs received in; a row whose count reaches its holder count is released at `level`, its local
// successors' remaining in-degrees drop, and the rows reaching zero send READY to every holder (the next wave).
// flag[1] += rows released; bad[0]: a READY for a row this store does not hold, or for a released row.
static __global__ __launch_bounds__(256) void k_ks_step(size_t m, const uint64_t* __restrict__ in, size_t n, uint32_t level,
                                                 const uint32_t* __restrict__ gid, const uint8_t* __restrict__ holders,
                                                 const uint64_t* __restrict__ xoff, const uint32_t* __restrict__ xs,
                                                 uint32_t* __restrict__ rem, uint32_t* __restrict__ lvl,
                                                 uint32_t* __restrict__ rcnt, const uint32_t* __restrict__ base,
                                                 uint32_t* __restrict__ cnt, uint64_t* __restrict__ out,
                                                 uint32_t* __restrict__ flag, uint32_t* __restrict__ bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t beg = 0, end = 0;
    bool b = false, got = false;
    if (i < m) {
        const size_t r = ks_row(gid, n, (uint32_t)in[i]);
        if (r >= n || lvl[r] != KS_UNRELEASED) {
            b = true;
        } else if (atomicAdd(&rcnt[r], 1u) + 1u == (uint32_t)__popc(holders[r])) {
            lvl[r] = level;
            beg = xoff[r]; end = xoff[r + 1];
            got = true;
        }
    }
    const uint64_t gb = __ballot(got);
    if ((int)__lane_id() == __ffsll((unsigned long long)gb) - 1) atomicAdd(flag + 1, (uint32_t)__popcll(gb));
    for (uint64_t k = 0;; ++k) {
        const bool has = beg + k < end;
        if (!__ballot(has)) break;
        bool want = false;
        uint32_t hm = 0;
        uint64_t msg = 0;
        if (has) {
            const uint32_t s = xs[beg + k];
            if (atomicSub(&rem[s], 1u) == 1u) { want = true; hm = holders[s]; msg = gid[s]; }
        }
        ks_ready_all(want, hm, msg, base, cnt, out);
    }
    wave_set_flag(b, bad);
}

}  // namespace ad
