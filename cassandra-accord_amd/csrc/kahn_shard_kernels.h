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
// A READY carries its sender's level bound (1 + the greatest level of the row's local predecessors, 0 without any)
// in its high word; a txn's level is the greatest bound over its holders' READYs, so it does not depend on the wave
// that delivers them: a READY may be late (a bounded exchange slot full) and the levels are still exact.
// The outbox is a queue per destination (tail: appended, head: sent).  Exchanges:
//   * host transports / ad_shard_kahn_exchange: every queued READY each wave (waves stop at the first exchange that
//     moves nothing anywhere; with full delivery the wave of a release is its level);
//   * ad_shard_kahn_run (RCCL): fixed slots of S READYs per (source, destination) and wave, so the receive sizes are
//     known without asking the host: the waves are enqueued back to back with no host synchronisation between them;
//     every few waves an all-reduce of the READYs still queued anywhere goes to a pinned word, and the host reads it
//     `lag` checks later (the device has those waves queued meanwhile); every store sees the same sums, so all stop
//     after the same wave.
// The round-4 protocol sent READY to one coordinating holder and RELEASE back (two exchanges and four host round trips
// per wave).  A txn costs holders x holders READYs over the batch (holders x (holders - 1) over the network).  The
// region for destination d holds at most one READY per local row d also holds, so appends never overflow.
#pragma once
#include "shard_kernels.h"

namespace ad {

constexpr uint32_t KS_UNRELEASED = 0xFFFFFFFFu;
__device__ inline uint64_t ks_msg(uint32_t g, uint32_t lb) { return (uint64_t)g | ((uint64_t)lb << 32); }

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
                                                 uint32_t* __restrict__ rcnt, uint32_t* __restrict__ lacc,
                                                 uint32_t* __restrict__ plv, const uint32_t* __restrict__ base,
                                                 uint32_t* __restrict__ cnt, uint64_t* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool want = false;
    uint32_t hm = 0;
    uint64_t msg = 0;
    if (i < n) {
        lvl[i] = KS_UNRELEASED;
        rcnt[i] = 0;
        lacc[i] = 0;
        plv[i] = 0;
        if (rem[i] == 0) { want = true; hm = holders[i]; msg = ks_msg(gid[i], 0); }
    }
    ks_ready_all(want, hm, msg, base, cnt, out);
}

// One wave: the READYs received in (S == 0: m messages in a row; else the slots of `world` sources, S + 1 words each:
// a count, then the READYs); a row whose count reaches its holder count is released at the greatest level bound of
// its READYs; its local successors' level bounds rise to its level + 1 and their remaining in-degrees drop, and the rows
// reaching zero send READY (with their bound) to every holder.  flag[1] += rows released, flag[3] = max(level + 1);
// bad[0]: a READY for a row this store does not hold, or for a released row.  (Each bound is raised before the count
// that publishes it, with a device fence between: the thread that completes a count reads every bound raised before.)
static __global__ __launch_bounds__(256) void k_ks_step(size_t m, uint32_t S, const uint64_t* __restrict__ in, size_t n,
                                                 const uint32_t* __restrict__ gid, const uint8_t* __restrict__ holders,
                                                 const uint64_t* __restrict__ xoff, const uint32_t* __restrict__ xs,
                                                 uint32_t* __restrict__ rem, uint32_t* __restrict__ lvl,
                                                 uint32_t* __restrict__ rcnt, uint32_t* lacc, uint32_t* plv,
                                                 const uint32_t* __restrict__ base,
                                                 uint32_t* __restrict__ cnt, uint64_t* __restrict__ out,
                                                 uint32_t* __restrict__ flag, uint32_t* __restrict__ bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t beg = 0, end = 0;
    bool b = false, got = false;
    uint32_t L = 0;
    bool has_msg = false;
    uint64_t msg = 0;
    if (i < m) {
        if (S == 0) {
            has_msg = true;
            msg = in[i];
        } else {
            const size_t src = i / S, k = i - src * S;
            const uint64_t* slot = in + src * (S + 1);
            has_msg = k < slot[0];
            if (has_msg) msg = slot[1 + k];
        }
    }
    if (has_msg) {
        const size_t r = ks_row(gid, n, (uint32_t)msg);
        if (r >= n || lvl[r] != KS_UNRELEASED) {
            b = true;
        } else {
            atomicMax(&lacc[r], (uint32_t)(msg >> 32));
            __threadfence();
            if (atomicAdd(&rcnt[r], 1u) + 1u == (uint32_t)__popc(holders[r])) {
                __threadfence();
                L = atomicMax(&lacc[r], 0u);
                lvl[r] = L;
                atomicMax(&flag[3], L + 1u);
                beg = xoff[r]; end = xoff[r + 1];
                got = true;
            }
        }
    }
    const uint64_t gb = __ballot(got);
    if ((int)__lane_id() == __ffsll((unsigned long long)gb) - 1) atomicAdd(flag + 1, (uint32_t)__popcll(gb));
    for (uint64_t k = 0;; ++k) {
        const bool has = beg + k < end;
        if (!__ballot(has)) break;
        bool want = false;
        uint32_t hm = 0;
        uint64_t mo = 0;
        if (has) {
            const uint32_t s_ = xs[beg + k];
            atomicMax(&plv[s_], L + 1u);
            __threadfence();
            if (atomicSub(&rem[s_], 1u) == 1u) {
                __threadfence();
                want = true; hm = holders[s_]; mo = ks_msg(gid[s_], atomicMax(&plv[s_], 0u));
            }
        }
        ks_ready_all(want, hm, mo, base, cnt, out);
    }
    wave_set_flag(b, bad);
}

// ad_shard_kahn_run: this wave's slot per destination d (one workgroup each): up to S queued READYs from the head of
// d's queue, the count first; the head advances past them.  sent[0] += the READYs for other stores.
static __global__ __launch_bounds__(256) void k_ks_pack(uint32_t S, uint32_t self, const uint32_t* __restrict__ base,
                                                 const uint32_t* __restrict__ tail, uint32_t* __restrict__ head,
                                                 const uint64_t* __restrict__ out, uint64_t* __restrict__ stage,
                                                 unsigned long long* __restrict__ sent) {
    const uint32_t d = blockIdx.x;
    const uint32_t h0 = head[d], q = tail[d] - h0, c = q < S ? q : S;
    uint64_t* slot = stage + (size_t)d * (S + 1);
    for (uint32_t k = threadIdx.x; k < c; k += blockDim.x) slot[1 + k] = out[base[d] + h0 + k];
    __syncthreads();
    if (threadIdx.x == 0) {
        slot[0] = c;
        head[d] = h0 + c;
        if (d != self && c) atomicAdd(sent, (unsigned long long)c);
    }
}
// ad_shard_kahn_exchange: this wave's count per destination (the queues' lengths)
static __global__ void k_ks_lengths(uint32_t W, const uint32_t* __restrict__ tail, const uint32_t* __restrict__ head,
                                    uint32_t* __restrict__ len) {
    const uint32_t d = threadIdx.x;
    if (d < W) len[d] = tail[d] - head[d];
    if (d == W) len[d] = 0;
}
// the READYs still queued on this store (after a wave's step): pending[0]
static __global__ void k_ks_pending(uint32_t W, const uint32_t* __restrict__ tail, const uint32_t* __restrict__ head,
                                    unsigned long long* __restrict__ pending) {
    if (threadIdx.x != 0) return;
    unsigned long long p = 0;
    for (uint32_t d = 0; d < W; ++d) p += tail[d] - head[d];
    pending[0] = p;
}

}  // namespace ad
