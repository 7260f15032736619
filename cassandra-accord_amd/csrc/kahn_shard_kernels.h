// kahn_shard_kernels.h — execution levels of a key-range sharded batch as distributed Kahn wavefronts
// (SURVEY §8e, round 4).
//
// Every execution constraint is local to one store (global_levels.h): an (a) key-chain edge lives with the key's
// store, a (b) direct / range dependency edge and a (c) unmanaged chain bound with a store whose slice both ends
// touch.  So a txn's level is 1 + the greatest level of its predecessors over the stores that hold it, and it can
// be released at level l once EVERY holder has released all of its local predecessors by level l - 1.  Per wave
// (level) l, each store
//   1. sends READY(txn) to the txn's coordinator (one of its holders, ks_coord) for every local row whose last
//      local predecessor was released at level l - 1 (level 0: the rows without local predecessors);
//   2. coordinators count READYs; a txn whose count reaches its holder count is released at level l, and
//      RELEASE(txn) goes to every holder (itself included);
//   3. every store applies the RELEASEs: the row's level is l, its local successors' remaining in-degrees drop, and
//      those reaching zero are step 1 of wave l + 1.
// Waves stop when one released nothing.  Each txn costs (holders) READY + (holders) RELEASE messages in total, once
// per batch -- not once per round as the delta exchange's raised levels, nor every store's edges on every store as
// the one-exchange gather -- and each store touches only its own edges.  Messages are u64 (global rank in the low
// word); regions per destination are sized by what can be sent there at most (a row is ready once; a coordinated
// txn released once), so appends never overflow.
#pragma once
#include "shard_kernels.h"

namespace ad {

constexpr uint32_t KS_UNRELEASED = 0xFFFFFFFFu;

// The store that counts a txn's READYs and sends its RELEASEs: one of its holders, picked by global rank (the
// (g mod holders)-th set bit of the holder mask), so the coordination spreads evenly over the stores.  (The txn's
// home store -- its first key's -- would coordinate ~41 % of C5's txns on store 0 at N = 8.)
__host__ __device__ inline uint32_t ks_coord(uint32_t g, uint32_t holders) {
    uint32_t k = g % (uint32_t)__builtin_popcount(holders), m = holders;
    for (; k > 0; --k) m &= m - 1u;
    return (uint32_t)__builtin_ctz(m);
}

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

// Wave 0: every row starts unreleased; rows without local predecessors are ready.
static __global__ __launch_bounds__(256) void k_ks_init(size_t n, const uint32_t* __restrict__ gid, const uint8_t* __restrict__ holders,
                                                 const uint32_t* __restrict__ rem, uint32_t* __restrict__ lvl,
                                                 uint32_t* __restrict__ rcnt, const uint32_t* __restrict__ base,
                                                 uint32_t* __restrict__ cnt, uint64_t* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool want = false;
    uint32_t dest = 0;
    uint64_t msg = 0;
    if (i < n) {
        lvl[i] = KS_UNRELEASED;
        rcnt[i] = 0;
        if (rem[i] == 0) { want = true; dest = ks_coord(gid[i], holders[i]); msg = gid[i]; }
    }
    ks_append(want, dest, msg, base, cnt, out);
}

// Coordinator: READYs in; a txn whose count reaches its holder count is released at `level` -> RELEASE to every
// holder.  bad[0]: a message for a row this store does not coordinate; flag[0]: released something.
static __global__ __launch_bounds__(256) void k_ks_decide(size_t m, const uint64_t* __restrict__ in, size_t n,
                                                   const uint32_t* __restrict__ gid, uint32_t self,
                                                   const uint8_t* __restrict__ holders, uint32_t* __restrict__ rcnt,
                                                   const uint32_t* __restrict__ base, uint32_t* __restrict__ cnt,
                                                   uint64_t* __restrict__ out, uint32_t* __restrict__ flag,
                                                   uint32_t* __restrict__ bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t mask = 0;
    uint64_t msg = 0;
    bool b = false;
    if (i < m) {
        const uint32_t g = (uint32_t)in[i];
        const size_t r = ks_row(gid, n, g);
        if (r >= n || ks_coord(g, holders[r]) != self) {
            b = true;
        } else {
            const uint32_t hm = holders[r];
            if (atomicAdd(&rcnt[r], 1u) + 1u == (uint32_t)__popc(hm)) { mask = hm; msg = g; }
        }
    }
#pragma unroll
    for (int d = 0; d < MAX_STORES; ++d) ks_append((mask >> d) & 1u, (uint32_t)d, msg, base, cnt, out);
    wave_set_flag(mask != 0, flag);
    wave_set_flag(b, bad);
}

// Every holder: RELEASEs in -> the row's level, then its local successors' remaining in-degrees; rows reaching
// zero send READY to their coordinator (the next wave).  flag[1] += rows released here.
static __global__ __launch_bounds__(256) void k_ks_apply(size_t m, const uint64_t* __restrict__ in, size_t n, uint32_t level,
                                                  const uint32_t* __restrict__ gid, const uint8_t* __restrict__ holders,
                                                  const uint64_t* __restrict__ xoff, const uint32_t* __restrict__ xs,
                                                  uint32_t* __restrict__ rem, uint32_t* __restrict__ lvl,
                                                  const uint32_t* __restrict__ base, uint32_t* __restrict__ cnt,
                                                  uint64_t* __restrict__ out, uint32_t* __restrict__ flag,
                                                  uint32_t* __restrict__ bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t beg = 0, end = 0;
    bool b = false, got = false;
    if (i < m) {
        const size_t r = ks_row(gid, n, (uint32_t)in[i]);
        if (r >= n || lvl[r] != KS_UNRELEASED) {
            b = true;
        } else {
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
        uint32_t dest = 0;
        uint64_t msg = 0;
        if (has) {
            const uint32_t s = xs[beg + k];
            if (atomicSub(&rem[s], 1u) == 1u) { want = true; dest = ks_coord(gid[s], holders[s]); msg = gid[s]; }
        }
        ks_append(want, dest, msg, base, cnt, out);
    }
    wave_set_flag(b, bad);
}

}  // namespace ad
