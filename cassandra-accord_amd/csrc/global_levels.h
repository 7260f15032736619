// global_levels.h — execution levels of a key-range-sharded batch in ONE exchange (gfx950).
//
// Every execution constraint is local to one store: an (a) key-chain edge belongs to the store
// owning the key, a (b) direct / range dependency edge to a store whose slice both txns touch, a (c) unmanaged
// bound to one key's chain.  So the level DAG of the whole batch is the union of the stores' constraint
// graphs.  Each store therefore exports its constraints as explicit edges over global arrival ranks,
// (src << 32 | dst) — the transitive reduction of its key chains plus its (b)/(c) edges — every store gathers
// all of them, and solves the union with the Kahn wavefronts: one exchange, whatever the depth of the graph
// (the per-round delta exchange this replaces needed as many rounds as the graph is deep).
//
//   (a) per key chain in executeAt order over the managesExecution entries (CommandsForKey.notifyManaged,
//       CommandsForKey.java:1208-1289): a Read waits for the last Write before it; a Write for the Reads
//       since the last Write, else for that Write (level = 1 + max over earlier entries, and Write levels
//       increase along the chain, so those edges carry the maximum);
//   (b)/(c) as the Kahn path's explicit edges (xedges_visit, level_kernels.h).
#pragma once
#include "level_kernels.h"

namespace ad {

__device__ inline uint64_t edge_of(const uint32_t* gid, uint32_t src, uint32_t dst) {
    return ((uint64_t)(gid ? gid[src] : src) << 32) | (uint64_t)(gid ? gid[dst] : dst);
}

// Batches carrying CFK history (current statuses): APPLIED / INVALID txns are done — they wait for nothing and
// nothing waits for them (Commands.updateWaitingOn drops applied / invalidated deps, Commands.java:700-775).
// Applied txns form an executeAt prefix of each key's chain (a txn applies only once everything it waits for
// has), so the reduction below stays exact with them removed.
__device__ inline bool row_done(uint32_t m) {
    const uint32_t s = meta_status(m);
    return s == AD_ST_APPLIED || s == AD_ST_INVALID;
}

// (a) edges, one thread per chain position q (executeAt order inside each key segment); last_w[q] = position of
// the last Write before q in its segment (-1: none; WriteLinkOp<false>).  Count pass: cnt[q]; fill: at off[q].
// done_aware: no edge into or out of a done txn (batches with CFK history).
template <bool FILL>
static __global__ __launch_bounds__(256) void k_chain_edges(size_t P, const int32_t* __restrict__ seg_start,
                                                            const uint32_t* __restrict__ c_txn, const uint8_t* __restrict__ c_meta,
                                                            const int32_t* __restrict__ last_w, const uint32_t* __restrict__ gid,
                                                            int done_aware, unsigned long long* __restrict__ cnt,
                                                            const unsigned long long* __restrict__ off, uint64_t* __restrict__ out) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t m = c_meta[q];
    uint32_t k = 0;
    if (manages_execution(m) && !(done_aware && row_done(m))) {
        const uint32_t t = c_txn[q];
        const int32_t lw = last_w[q], s0 = seg_start[q];
        auto live = [&](int32_t pos) { return !(done_aware && row_done(c_meta[pos])); };
        auto emit = [&](int32_t pos) {
            if (FILL) out[off[q] + k] = edge_of(gid, c_txn[pos], t);
            ++k;
        };
        if (meta_kind(m) == AD_KIND_WRITE) {
            // no Write between lw and q: the managed entries there are Reads
            for (int32_t x = (lw + 1 > s0 ? lw + 1 : s0); x < (int32_t)q; ++x)
                if (manages_execution(c_meta[x]) && live(x)) emit(x);
            if (k == 0 && lw >= 0 && live(lw)) emit(lw);
        } else if (lw >= 0 && live(lw)) {
            emit(lw);
        }
    }
    if (!FILL) cnt[q] = k;
}

// (b)/(c) edges of txn t (k_xedges' sources), as (src, t) pairs: count pass cnt[t], fill at off[t]
template <bool FILL>
static __global__ __launch_bounds__(256) void k_xedge_pairs(XEdgeArgs a, const uint32_t* __restrict__ gid,
                                                            unsigned long long* __restrict__ cnt,
                                                            const unsigned long long* __restrict__ off, uint64_t* __restrict__ out) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.e.n) return;
    uint64_t k = 0;
    xedges_visit(a, t, [&](uint32_t src) {
        if (FILL) out[off[t] + k] = edge_of(gid, src, (uint32_t)t);
        ++k;
    });
    if (!FILL) cnt[t] = k;
}

// ---- the global solve over the gathered edges (every store holds all of them) -------------------------
static __global__ __launch_bounds__(256) void k_edges_split(size_t m, const uint64_t* __restrict__ e, uint32_t* __restrict__ src,
                                                            uint32_t* __restrict__ dst, uint32_t* __restrict__ indeg, uint32_t n,
                                                            uint32_t* __restrict__ bad) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool b = false;
    if (i < m) {
        const uint64_t x = e[i];
        const uint32_t s = (uint32_t)(x >> 32), d = (uint32_t)x;
        if (s >= n || d >= n || s == d) {
            b = true;
        } else {
            src[i] = s;
            dst[i] = d;
            atomicAdd(&indeg[d], 1u);
        }
    }
    wave_set_flag(b, bad);
}
// successor offsets of the src-sorted edges: xoff[v] = first edge with src >= v (v in [0, n])
static __global__ __launch_bounds__(256) void k_xoff_bounds(size_t m, const uint32_t* __restrict__ src, uint32_t n,
                                                            uint64_t* __restrict__ xoff) {
    const size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (v > n) return;
    size_t lo = 0, hi = m;
    while (lo < hi) { const size_t h = (lo + hi) >> 1; if (src[h] < (uint32_t)v) lo = h + 1; else hi = h; }
    xoff[v] = lo;
}

// CFK history batches: an INVALID entry is no part of its key's execution chain (it never executes, so it neither
// waits nor carries the chain's Write order): its chain copy is marked unmanaged before the last-Write scan
static __global__ __launch_bounds__(256) void k_chain_mask_invalid(size_t P, uint8_t* __restrict__ c_meta) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t m = c_meta[q];
    if (meta_status(m) == AD_ST_INVALID) c_meta[q] = (uint8_t)((m & ~7u) | AD_KIND_LOCAL_ONLY);
}

// CFK history batches: done rows (APPLIED / INVALID) report AD_LEVEL_DONE and sort first (key 0); the others
// sort by level + 1, then executeAt (order_rows)
static __global__ __launch_bounds__(256) void k_done_levels(size_t n, const uint8_t* __restrict__ meta, uint32_t* __restrict__ lvl,
                                                            uint32_t* __restrict__ key) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const bool done = row_done(meta[t]);
    key[t] = done ? 0u : lvl[t] + 1u;
    if (done) lvl[t] = AD_LEVEL_DONE;
}

// every txn was released (a cycle would leave some in-degree unconsumed)
static __global__ __launch_bounds__(256) void k_rem_check(size_t n, const uint32_t* __restrict__ rem, uint32_t* __restrict__ bad) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    wave_set_flag(t < n && rem[t] != 0u, bad);
}

}  // namespace ad
