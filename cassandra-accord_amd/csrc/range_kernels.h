// range_kernels.h — RangeDeps: the range-interval overlap join (gfx950).
//
// Replaces InMemoryCommandStore.mapReduceRangesInternal (impl/InMemoryCommandStore.java:884-1017), the
// brute-force scan of every range command per query, and its TreeMap<Range, List<TxnInfo>> collection
// (keyed by Range::compare = (start, end), Range.java:310-317).  Semantics per query txn i: every range
// txn j < i with a witnessed kind, not Erased (here: final status INVALID outside the in-flight window),
// and not dropped by the replica view; each of j's ranges r that intersects i's footprint — a key k
// with r.start < k <= r.end (Range.EndInclusive, Range.java:48-55) or a range q with
// !(r.start >= q.end) && !(r.end <= q.start) (compareIntersecting :296-305) — contributes (r, j).
//
// Device algorithm:
//   * range entries (start, end, owner) of all range txns are radix-sorted by (start, end, owner) once
//     per batch (stable LSD on end then start over the input order, which is owner order);
//   * a 64-ary max-end tree over the sorted entries (range_index.h, the device form of CINTIA's
//     checkpoints) gives, per footprint element, the entries below its bound whose end reaches it:
//     O(log Q + hits) per query whatever the width distribution (one very wide range no longer widens
//     every query's window);
//   * one wave per query txn walks the chunks the index yields for its whole footprint 64 entries at a
//     time, evaluates the predicate per lane, and ballots per replica view: popcounts give the counts,
//     prefix popcounts the output slots, and the matched entries come out already in (start, end,
//     owner) order — the RangeDeps key order — so equal ranges are adjacent and the distinct-range
//     count falls out of a lane-to-previous-match comparison (shuffle from the highest lower match).
//   * the per-txn TxnId union/remap is k_union_lds.
// Bytes per query: the visited entries (16 B range + 4 B owner + 1 B meta) + 512 B per index step; per
// emitted entry 4 B (+16 B per distinct range).
#pragma once
#include "range_index.h"
#include "union_kernels.h"

namespace ad {

// per range entry: owner txn + sort keys (end, start relative to rbase)
static __global__ __launch_bounds__(256) void k_range_prep(size_t n, const uint8_t* __restrict__ meta, const uint32_t* __restrict__ range_off,
                                                    const uint64_t* __restrict__ rs, const uint64_t* __restrict__ re,
                                                    uint64_t rbase, uint32_t* __restrict__ rowner,
                                                    uint32_t* __restrict__ k_end, uint32_t* __restrict__ v_idx) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    for (uint32_t q = range_off[t]; q < range_off[t + 1]; ++q) {
        rowner[q] = (uint32_t)t;
        k_end[q] = (uint32_t)(re[q] - rbase);
        v_idx[q] = q;
    }
}

static __global__ __launch_bounds__(256) void k_range_startkey(size_t Q, const uint64_t* __restrict__ rs, const uint32_t* __restrict__ idx,
                                                        uint64_t rbase, uint32_t* __restrict__ k_start) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < Q) k_start[x] = (uint32_t)(rs[idx[x]] - rbase);
}

// 64-bit range spreads: sort key = (src[idx[x]] - rbase) >> shift, truncated to 32 bits (one LSD half)
static __global__ __launch_bounds__(256) void k_range_key_half(size_t Q, const uint64_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                        uint64_t rbase, int shift, uint32_t* __restrict__ k_out) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < Q) k_out[x] = (uint32_t)((src[idx[x]] - rbase) >> shift);
}

static __global__ __launch_bounds__(256) void k_range_gather(size_t Q, const uint32_t* __restrict__ idx, const uint64_t* __restrict__ rs,
                                                      const uint64_t* __restrict__ re, const uint32_t* __restrict__ rowner,
                                                      uint64_t* __restrict__ es, uint64_t* __restrict__ ee,
                                                      uint32_t* __restrict__ eown) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= Q) return;
    const uint32_t q = idx[x];
    es[x] = rs[q];
    ee[x] = re[q];
    eown[x] = rowner[q];
}

struct RangeArgs {
    size_t n, Q;
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint32_t* range_off;
    const uint64_t* rs;
    const uint64_t* re;
    const uint8_t* meta;
    const uint64_t* es;          // sorted entries
    const uint64_t* ee;
    const uint32_t* eown;
    RangeIndex ix;               // max-end tree over the sorted entries (range_index.h)
    const Params* prm;           // range_kinds: a query whose kind witnesses none of them walks nothing (nullable)
    uint32_t window, thresh;
    uint64_t seed;
    uint32_t* rnk;               // [v * n + t]  distinct ranges (count pass)
    uint32_t* rne;               // [v * n + t]  entries
    const uint32_t* key_off_v[MAXV];   // fill pass: per-view RangeDeps CSR
    const uint32_t* k2t_off_v[MAXV];
    uint64_t* keys_v[MAXV];      // (start, end) interleaved
    int32_t* k2t_v[MAXV];
    const uint32_t* qpos;        // executeAt-bound queries: per txn the bound's arrival position (nullable)
    const uint32_t* gqpos;       // sharded stores: the bound's global arrival position (window; nullable = qpos)
    const uint32_t* gid;         // sharded stores: local row -> global arrival rank (window, drops; nullable)
};

// does entry [s, e) intersect txn t's footprint (sorted keys, or sorted disjoint ranges)?
__device__ inline bool range_hits(const RangeArgs& a, bool key_dom, uint32_t fb, uint32_t fe, uint64_t s, uint64_t e) {
    if (key_dom) {
        // first key > s, then <= e ?
        const uint32_t x = ub_u64(a.keys, fb, fe, s);
        return x < fe && a.keys[x] <= e;
    }
    // ranges sorted and disjoint: first q with q.end > s; intersects iff q.start < e
    uint32_t lo = fb, hi = fe;
    while (lo < hi) {
        uint32_t m = (lo + hi) >> 1;
        if (a.re[m] <= s) lo = m + 1; else hi = m;
    }
    return lo < fe && a.rs[lo] < e;
}

template <int NV, bool FILL>
static __global__ __launch_bounds__(256) void k_range_deps(RangeArgs a) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n) return;
    const int lane = __lane_id();
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t i = (uint32_t)t;
    const uint32_t mi = a.meta[i];
    const uint32_t qk = meta_kind(mi);
    const bool key_dom = meta_domain(mi) == AD_DOMAIN_KEY;
    const uint32_t fb = key_dom ? a.key_off[i] : a.range_off[i];
    const uint32_t fe = key_dom ? a.key_off[i + 1] : a.range_off[i + 1];
    // the arrival position the query is answered at (PreAccept: i; Accept: its executeAt's), the window below it
    const uint32_t qi = a.qpos ? a.qpos[i] : i;
    // window and drop decisions use global arrival ranks (shard-invariant); emitted ids stay local rows
    const uint32_t gi = a.gid ? a.gid[i] : i;
    const uint32_t gq = a.qpos ? (a.gqpos ? a.gqpos[i] : qi) : gi;
    const uint32_t lo_w = a.window == 0 ? gq : (gq > a.window ? gq - a.window : 0u);
    uint32_t ecount[NV], kcount[NV];
    uint64_t cs[NV], ce[NV];
    bool chas[NV];
    uint32_t kb[NV], mb[NV], nkt[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        ecount[v] = 0; kcount[v] = 0; cs[v] = 0; ce[v] = 0; chas[v] = false;
        if (FILL) {
            kb[v] = a.key_off_v[v][i];
            nkt[v] = a.key_off_v[v][i + 1] - kb[v];
            mb[v] = a.k2t_off_v[v][i];
        }
    }
    uint32_t wk = 0;                                   // the range kinds this query's kind witnesses
#pragma unroll
    for (uint32_t k = 0; k <= AD_KIND_EXCLUSIVE_SYNC_POINT; ++k) wk |= witnesses(qk, k) ? 1u << k : 0u;
    const bool query = qk <= AD_KIND_EXCLUSIVE_SYNC_POINT && fe > fb && a.Q > 0 && (!a.prm || (wk & a.prm->range_kinds));
    if (query) {
        // the index walk visits, in entry order, the chunks that can hold a hit; the predicate is exact
        ri_walk(a.ix, a.es, (uint32_t)a.Q, key_dom, a.keys, a.rs, a.re, fb, fe, [&](uint32_t clo, uint32_t chi) {
            const uint32_t x = clo + lane;
            const bool valid = x < chi;
            uint64_t s = 0, e = 0;
            uint32_t j = 0xFFFFFFFFu, gj = 0xFFFFFFFFu;
            bool cond = false;
            if (valid) {
                j = a.eown[x];
                if (j < qi && j != i) {
                    const uint32_t mj = a.meta[j];
                    gj = a.gid ? a.gid[j] : j;
                    const bool inw = gj >= lo_w;
                    cond = witnesses(qk, meta_kind(mj)) && (inw || meta_status(mj) != AD_ST_INVALID);
                    if (cond) {
                        s = a.es[x];
                        e = a.ee[x];
                        cond = range_hits(a, key_dom, fb, fe, s, e);
                    }
                }
            }
            const bool inw = gj >= lo_w;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const bool ok = cond && !(inw && a.thresh && drop_hash(a.seed, (uint32_t)v, gi, gj) < a.thresh);
                const uint64_t mask = __ballot(ok);
                if (mask == 0) continue;
                const uint64_t lower = mask & below;
                const int pl = lower ? 63 - __clzll(lower) : lane;
                const uint64_t ps = __shfl(s, pl), pe = __shfl(e, pl);
                const bool has_prev = lower ? true : chas[v];
                const uint64_t prs = lower ? ps : cs[v], pre = lower ? pe : ce[v];
                const bool newkey = ok && !(has_prev && prs == s && pre == e);
                const uint64_t nmask = __ballot(newkey);
                if (FILL) {
                    const uint32_t epos = ecount[v] + (uint32_t)__popcll(lower);
                    if (ok) a.k2t_v[v][mb[v] + nkt[v] + epos] = (int32_t)j;
                    if (newkey) {
                        const uint32_t kpos = kcount[v] + (uint32_t)__popcll(nmask & below);
                        a.keys_v[v][2 * (size_t)(kb[v] + kpos)] = s;
                        a.keys_v[v][2 * (size_t)(kb[v] + kpos) + 1] = e;
                        if (kpos > 0) a.k2t_v[v][mb[v] + kpos - 1] = (int32_t)(nkt[v] + epos);
                    }
                }
                ecount[v] += (uint32_t)__popcll(mask);
                kcount[v] += (uint32_t)__popcll(nmask);
                const int hl = 63 - __clzll(mask);
                cs[v] = __shfl(s, hl);
                ce[v] = __shfl(e, hl);
                chas[v] = true;
            }
        });
    }
    if (lane == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if (FILL) {
                if (nkt[v] > 0) a.k2t_v[v][mb[v] + nkt[v] - 1] = (int32_t)(nkt[v] + ecount[v]);
            } else {
                a.rnk[(size_t)v * a.n + t] = kcount[v];
                a.rne[(size_t)v * a.n + t] = ecount[v];
            }
        }
    }
}

}  // namespace ad
