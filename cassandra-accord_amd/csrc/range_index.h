// range_index.h — the interval index over the sorted range entries (gfx950).
//
// Replaces SearchableRangeList / CheckpointIntervalArray (utils/SearchableRangeList.java:33-131,
// utils/CheckpointIntervalArray.java:28-219, CheckpointIntervalArrayBuilder.java): stabbing and overlap
// queries over the range commands of a store, O(log N + k) per query instead of a scan of every range
// whose start could reach the query.
//
// CINTIA keeps, every few entries of the start-sorted array, a checkpoint list of the earlier ranges
// that still reach past it.  On a 64-wide wavefront the natural shape is a 64-ary tree of maximum ends
// over the same (start, end, owner)-sorted array: level 0 is the entries' ends, node x of level l+1 is
// the maximum of nodes [64x, 64x + 64) of level l, up to a top level of at most 64 nodes.  The ranges
// that contain a point k (Range.EndInclusive (s, e], Range.java:48-55) are the entries with s < k
// (a prefix [0, lb(start >= k)) of the array) and e >= k, and those that intersect (qs, qe] are the
// entries with s < qe and e > qs (compareIntersecting, Range.java:296-305): every query is "entries
// x < hi with end >= thr".  ri_next finds the next such entry with one coalesced 64-lane load and ballot
// per tree level: climb while the aligned group of 64 holds no node >= thr, then descend into the first
// node that does.  Entries come out in array order, i.e. RangeDeps key order, so the joins below keep
// their ordered, duplicate-free output.  Memory: Q·8/63 bytes over the entries; build: one pass per
// level, one wave per node.
#pragma once
#include "common.h"

namespace ad {

constexpr int RI_MAXLEV = 7;           // 64^6 = 2^36 entries > any u32 count

struct RangeIndex {
    const uint64_t* lv[RI_MAXLEV];     // lv[0] = entry ends (ee), lv[l] = maxima of 64 nodes of lv[l-1]
    uint32_t cnt[RI_MAXLEV];
    int top;                           // cnt[top] <= 64
};

// host: node counts of levels 1..top for Q entries, and the total (one buffer holds all upper levels)
inline int ri_levels(size_t Q, uint32_t* cnt, size_t* total) {
    int top = 0;
    size_t c = Q, sum = 0;
    cnt[0] = (uint32_t)Q;
    while (c > (size_t)WAVE) {
        c = (c + WAVE - 1) / WAVE;
        cnt[++top] = (uint32_t)c;
        sum += c;
    }
    *total = sum;
    return top;
}

// one wave per output node: max of its 64 children
static __global__ __launch_bounds__(256) void k_ri_level(size_t nout, uint32_t nin, const uint64_t* __restrict__ in, uint64_t* __restrict__ out) {
    const size_t x = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (x >= nout) return;
    const size_t c = x * WAVE + __lane_id();
    uint64_t m = c < nin ? in[c] : 0ull;
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) {
        const uint64_t y = __shfl_xor(m, o);
        m = y > m ? y : m;
    }
    if (__lane_id() == 0) out[x] = m;
}

// Smallest x in [lo, hi) with lv[0][x] >= thr, else hi.  Arguments wave-uniform; every lane calls.
__device__ inline uint32_t ri_next(const RangeIndex& ix, uint32_t lo, uint32_t hi, uint64_t thr) {
    if (lo >= hi) return hi;
    const uint32_t lane = (uint32_t)__lane_id();
    uint32_t pos = lo;
    int lev = 0;
    while (true) {
        if (((uint64_t)pos << (6 * lev)) >= hi) return hi;       // everything left lies at or past hi
        const uint32_t base = pos & ~(uint32_t)(WAVE - 1);
        const uint32_t idx = base + lane;
        const bool hit = idx >= pos && idx < ix.cnt[lev] && ix.lv[lev][idx] >= thr;
        const uint64_t m = __ballot(hit);
        if (m) {
            const uint32_t c = base + (uint32_t)__builtin_ctzll(m);
            if (lev == 0) return c < hi ? c : hi;
            --lev;
            pos = c << 6;                                         // first child: its group holds a hit
            continue;
        }
        if (lev == ix.top) return hi;
        pos = (base >> 6) + 1;                                    // the next node of the parent level
        ++lev;
    }
}

// Visit, in entry order, every chunk [x, chi) (chi - x <= 64) that can hold an entry intersecting a
// sorted footprint: keys strictly ascending (hit: s < k <= e), or sorted disjoint ranges (hit: s < qe &&
// e > qs).  Each element f needs entries below hi_f with end >= thr_f, and both bounds are non-decreasing
// in f, so one forward cursor serves the whole footprint; entries it skips cannot hit any later element.
// The visitor gets wave-uniform chunk bounds and evaluates the exact predicate itself.
template <class Visit>
__device__ inline void ri_walk(const RangeIndex& ix, const uint64_t* __restrict__ es, uint32_t Q, bool key_dom,
                               const uint64_t* __restrict__ keys, const uint64_t* __restrict__ rs,
                               const uint64_t* __restrict__ re, uint32_t fb, uint32_t fe, Visit&& visit) {
    uint32_t x = 0;
    for (uint32_t f = fb; f < fe; ++f) {
        uint64_t thr, top;
        if (key_dom) { thr = keys[f]; top = keys[f]; }
        else {
            if (rs[f] == ~0ull) continue;
            thr = rs[f] + 1; top = re[f];
        }
        // entries with start < top (the prefix [0, hi)); lb over es from the cursor on
        uint32_t lo = x, hi = Q;
        while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (es[m] < top) lo = m + 1; else hi = m; }
        hi = lo;
        while (x < hi) {
            x = ri_next(ix, x, hi, thr);
            if (x >= hi) break;
            const uint32_t chi = x + WAVE < hi ? x + WAVE : hi;
            visit(x, chi);
            x = chi;
        }
    }
}

}  // namespace ad
