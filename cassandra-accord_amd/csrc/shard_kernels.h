// shard_kernels.h — key-range sharding across GPUs (BASELINE C5).
//
// One CommandStore per GPU owns a contiguous key range (ShardDistributor.EvenSplit,
// local/ShardDistributor.java:32-80).  Each store resolves, for every txn touching its range, the part of
// the PreAccept deps that its keys produce (its local batch: the txns, with their keys sliced to the range,
// in global TxnId order; row -> global arrival rank through `gid`).  PreAccept.reduce across stores
// (messages/PreAccept.java:141-156: Deps.with of the per-store PartialDeps) becomes:
//   export    each store packs its per-(view, class) CSRs, TxnIds rewritten to global ranks, into one blob;
//   exchange  all-gather of the blobs (RCCL over xGMI, or host staging over gloo);
//   merge     each store's home txns (first key in its range) merge the fragments of every store, per view
//             (k_merge with per-source row indirection), then Deps.merge across the replica views.
// Execution levels: each store runs the chain fixpoint over its own keys on a replicated global level
// array; stores exchange it with an all-reduce(max) until no store raises a level.
#pragma once
#include "level_kernels.h"

namespace ad {

// txns lists of a capacity-form CSR: local row -> global rank (valid entries only; the capacity slack
// past tcnt is never read)
__global__ __launch_bounds__(256) void k_txns_to_global(size_t n, const uint32_t* __restrict__ ent_off, const uint32_t* __restrict__ tcnt,
                                                        uint32_t* __restrict__ txns, const uint32_t* __restrict__ gid) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t b = ent_off[t], e = b + tcnt[t];
    for (uint32_t x = b; x < e; ++x) txns[x] = gid[txns[x]];
}

struct Segment { const void* src; void* dst; uint64_t bytes; };
constexpr int MAX_SEGS = 160;
struct SegTable { Segment s[MAX_SEGS]; int count; };

// batched device memcpy: blockIdx.y = segment, blocks stride over its 16-byte words
__global__ __launch_bounds__(256) void k_copy_segments(SegTable tab) {
    const int k = blockIdx.y;
    if (k >= tab.count) return;
    const Segment sg = tab.s[k];
    const uint64_t words = sg.bytes / 4;
    const uint32_t* src = (const uint32_t*)sg.src;
    uint32_t* dst = (uint32_t*)sg.dst;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < words; x += (uint64_t)gridDim.x * blockDim.x)
        dst[x] = src[x];
}

struct CompactFlagOp {            // rows with flag -> out[] (exclusive-scan scatter)
    using S = uint32_t;
    const uint8_t* flag;
    uint32_t* out;
    uint32_t* total;
    size_t n;
    __device__ S load(size_t i) const { return flag[i] ? 1u : 0u; }
    __device__ S identity() const { return 0u; }
    __device__ S combine(S a, S b) const { return a + b; }
    __device__ void store(size_t i, S ex, S inc, S el) const {
        if (el) out[ex] = (uint32_t)i;
        if (i + 1 == n) *total = inc;
    }
};

// home txns: global ids
__global__ __launch_bounds__(256) void k_home_gid(size_t H, const uint32_t* __restrict__ rows, const uint32_t* __restrict__ gid,
                                                  uint32_t* __restrict__ hg) {
    const size_t h = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h < H) hg[h] = gid[rows[h]];
}

// row of each home txn in source s (binary search over the source's ascending global ids; -1 = absent)
__global__ __launch_bounds__(256) void k_source_rows(size_t H, const uint32_t* __restrict__ hg, const uint32_t* __restrict__ sgid,
                                                     uint32_t ns, int32_t* __restrict__ row) {
    const size_t h = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= H) return;
    const uint32_t g = hg[h];
    uint32_t lo = 0, hi = ns;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (sgid[m] < g) lo = m + 1; else hi = m;
    }
    row[h] = (lo < ns && sgid[lo] == g) ? (int32_t)lo : -1;
}

// levels: local rows <- replicated global array; and back (max), flagging any raise
__global__ __launch_bounds__(256) void k_levels_gather(size_t n, const uint32_t* __restrict__ gid, const uint32_t* __restrict__ G,
                                                       uint32_t* __restrict__ L) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) L[i] = G[gid[i]];
}
__global__ __launch_bounds__(256) void k_levels_scatter(size_t n, const uint32_t* __restrict__ gid, uint32_t* __restrict__ G,
                                                        const uint32_t* __restrict__ L, uint32_t* __restrict__ changed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool up = false;
    if (i < n) {
        const uint32_t g = gid[i], l = L[i];
        if (l > G[g]) { G[g] = l; up = true; }
    }
    wave_set_flag(up, changed);
}

}  // namespace ad
