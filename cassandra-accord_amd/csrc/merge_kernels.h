// merge_kernels.h — Deps.merge of R replica replies, per txn (gfx950).
//
// Replaces KeyDeps.merge / RelationMultiMap.LinearMerger (primitives/KeyDeps.java:115-135,
// utils/RelationMultiMap.java:284-406), which folds the replies pairwise with linearUnion
// (RelationMultiMap.java:562-816).  Because every reply is canonical (sorted unique keys, sorted
// unique TxnIds, sorted per-key index lists), the fold equals the canonical CSR of the union of the
// (key, TxnId) relations, which this kernel builds in one R-way merge-path pass per txn:
//   1. TxnIds: R-way merge of the replies' sorted TxnId lists (SortedArrays.linearUnion :198-333)
//   2. keys:   R-way merge of the sorted key lists; for each merged key, R-way merge of the replies'
//              per-key lists mapped to TxnIds, then to indices in (1) (remapToSuperset :1249-1275)
// Two launches: count (key / entry / TxnId totals per txn), then write into scanned offsets.
#pragma once
#include "range_kernels.h"

namespace ad {

struct MergeArgs {
    size_t n;
    int nv;
    const uint32_t* spec_bad;    // write pass launched before the merged sizes reached the host: exit when set
    const uint32_t* key_off[MAXV];
    const uint64_t* keys[MAXV];
    const uint32_t* k2t_off[MAXV];
    const int32_t* k2t[MAXV];
    const uint32_t* ent_off[MAXV];
    const uint32_t* txns[MAXV];
    const uint32_t* tcnt[MAXV];
    const int32_t* row[MAXV];    // optional per-part row indirection (nullptr = identity)
    uint32_t *mk, *me, *mu;      // count pass outputs
    const uint32_t* o_key_off;
    uint64_t* o_keys;
    const uint32_t* o_k2t_off;
    int32_t* o_k2t;
    const uint32_t* o_ent_off;
    uint32_t* o_txns;
    uint32_t* o_tcnt;
    // heavy txns (long lists: range txns' KeyDeps, key txns' RangeDeps) go to k_merge_heavy
    uint32_t* hcount;            // [1] appended by the count pass
    uint32_t* hlist;             // [n]
    uint8_t* hsame;              // [n] heavy txn whose replies are identical in every view (count pass -> write pass)
};

// A txn whose replies hold more than MERGE_HEAVY TxnIds + keys in total is merged by one workgroup
// (k_merge_heavy) instead of one thread: its serial merge would be thousands of dependent loads long.
constexpr uint32_t MERGE_HEAVY = MERGE_HEAVY_HINT;

// KW = u64 words per key: 1 for KeyDeps keys, 2 for RangeDeps (start, end) compared as Range::compare.
template <int KW>
struct MKey {
    uint64_t a, b;
    __device__ static MKey load(const uint64_t* k, size_t x) {
        MKey r;
        r.a = k[KW * x];
        r.b = KW == 2 ? k[KW * x + 1] : 0ull;
        return r;
    }
    __device__ bool operator<(const MKey& o) const { return a < o.a || (a == o.a && b < o.b); }
    __device__ bool operator==(const MKey& o) const { return a == o.a && b == o.b; }
};

template <int NV, bool WRITE, int KW>
static __global__ __launch_bounds__(256) void k_merge(MergeArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    if (WRITE && a.spec_bad && *a.spec_bad) return;   // speculative write into too-small buffers: re-run after sizing
    constexpr uint32_t INF = 0xFFFFFFFFu;
    // ---- 1. union of TxnId rank lists
    // input row of output txn t in each part (shard merge: a global txn's row in each source, -1 = absent)
    int64_t rv[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) rv[v] = a.row[v] ? (int64_t)a.row[v][t] : (int64_t)t;
    // a txn without deps in every reply (no TxnIds => no keys in a canonical CSR) merges to nothing:
    // settle it from the TxnId counts alone (C2: about half the txns)
    uint32_t tc[NV], any_tc = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) { tc[v] = rv[v] >= 0 ? a.tcnt[v][rv[v]] : 0u; any_tc |= tc[v]; }
    if (any_tc == 0) {
        if (WRITE) a.o_tcnt[t] = 0;
        else { a.mk[t] = 0; a.me[t] = 0; a.mu[t] = 0; }
        return;
    }
    if (a.hlist) {
        uint32_t w = 0;
#pragma unroll
        for (int v = 0; v < NV; ++v) w += tc[v] + (rv[v] >= 0 ? a.key_off[v][rv[v] + 1] - a.key_off[v][rv[v]] : 0u);
        const bool hv = w > MERGE_HEAVY;
        if (!WRITE) {
            const uint64_t m = __ballot(hv);
            if (hv) {                     // wave-aggregated append
                const int leader = __ffsll((unsigned long long)m) - 1;
                uint32_t base = 0;
                if ((int)__lane_id() == leader) base = atomicAdd(a.hcount, (uint32_t)__popcll(m));
                base = __builtin_amdgcn_readlane(base, leader);
                a.hlist[base + (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull))] = (uint32_t)t;
            }
        }
        if (hv) return;
    }
    uint32_t cur[NV], end[NV], head[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        cur[v] = rv[v] >= 0 ? a.ent_off[v][rv[v]] : 0u;
        end[v] = cur[v] + tc[v];
        head[v] = cur[v] < end[v] ? a.txns[v][cur[v]] : INF;
    }
    uint32_t* out = WRITE ? a.o_txns + a.o_ent_off[t] : nullptr;
    uint32_t mu = 0;
    while (true) {
        uint32_t mn = INF;
#pragma unroll
        for (int v = 0; v < NV; ++v) mn = head[v] < mn ? head[v] : mn;
        if (mn == INF) break;
        if (WRITE) out[mu] = mn;
        ++mu;
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (head[v] == mn) { ++cur[v]; head[v] = cur[v] < end[v] ? a.txns[v][cur[v]] : INF; }
    }
    // ---- 2. union of keys; per merged key union of the per-key TxnId lists
    uint32_t kc[NV], ke[NV], mb[NV], tb[NV], nkv[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const bool has = rv[v] >= 0;
        kc[v] = has ? a.key_off[v][rv[v]] : 0u;
        ke[v] = has ? a.key_off[v][rv[v] + 1] : 0u;
        nkv[v] = ke[v] - kc[v];
        mb[v] = has ? a.k2t_off[v][rv[v]] : 0u;
        tb[v] = has ? a.ent_off[v][rv[v]] : 0u;
    }
    const uint32_t okb = WRITE ? a.o_key_off[t] : 0;
    const uint32_t onk = WRITE ? a.o_key_off[t + 1] - okb : 0;
    const uint32_t omb = WRITE ? a.o_k2t_off[t] : 0;
    uint32_t mk = 0, me = 0;
    uint32_t ep = omb + onk;         // next entry slot (write pass)
    while (true) {
        bool any = false;
        MKey<KW> kmin{0ull, 0ull};
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if (kc[v] < ke[v]) {
                MKey<KW> k = MKey<KW>::load(a.keys[v], kc[v]);
                if (!any || k < kmin) { kmin = k; any = true; }
            }
        }
        if (!any) break;
        // per-view list bounds for this key
        uint32_t lc[NV], le[NV], lh[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            lc[v] = 0; le[v] = 0; lh[v] = INF;
            if (kc[v] < ke[v] && MKey<KW>::load(a.keys[v], kc[v]) == kmin) {
                const uint32_t ki = kc[v] - a.key_off[v][rv[v]];
                lc[v] = mb[v] + (ki == 0 ? nkv[v] : (uint32_t)a.k2t[v][mb[v] + ki - 1]);
                le[v] = mb[v] + (uint32_t)a.k2t[v][mb[v] + ki];
                lh[v] = lc[v] < le[v] ? a.txns[v][tb[v] + (uint32_t)a.k2t[v][lc[v]]] : INF;
                ++kc[v];
            }
        }
        uint32_t x = 0;   // position in the merged TxnId list (monotone)
        while (true) {
            uint32_t mn = INF;
#pragma unroll
            for (int v = 0; v < NV; ++v) mn = lh[v] < mn ? lh[v] : mn;
            if (mn == INF) break;
            if (WRITE) {
                while (out[x] < mn) ++x;
                a.o_k2t[ep++] = (int32_t)x;
            }
            ++me;
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (lh[v] == mn) { ++lc[v]; lh[v] = lc[v] < le[v] ? a.txns[v][tb[v] + (uint32_t)a.k2t[v][lc[v]]] : INF; }
        }
        if (WRITE) {
            a.o_keys[KW * (size_t)(okb + mk)] = kmin.a;
            if (KW == 2) a.o_keys[KW * (size_t)(okb + mk) + 1] = kmin.b;
            a.o_k2t[omb + mk] = (int32_t)(ep - omb);
        }
        ++mk;
    }
    if (WRITE) a.o_tcnt[t] = mu;
    else { a.mk[t] = mk; a.me[t] = me; a.mu[t] = mu; }
}

// ---------------------------------------------------------------------------------------------------
// Heavy txns: one 256-thread workgroup per txn (grid-stride over the heavy list).  The txn's TxnId lists
// are cut into chunks at every mch-th TxnId of the reply holding the most (mch: the longer list over the
// workgroup, at least MCH_MIN), its key lists likewise by keys;
// each chunk is a value interval, so the R-way merge of one chunk (the same loops as k_merge) is
// independent of the others.  Thread j takes a contiguous run of chunks; a block scan of the per-thread
// totals gives each thread its output offsets.  Write pass: TxnIds first (a barrier), then keys and
// per-key lists, whose TxnIds are remapped by binary search in the txn's merged TxnId list.
constexpr int MCH_MIN = 2, MH_T = 256, MH_GRID = 8192;
// write pass: the txn's merged TxnId list is staged in LDS for the per-entry remap (binary searches in LDS
// instead of HBM round trips) when it fits
constexpr uint32_t MH_LDS = 12288;

template <int KW>
__device__ inline uint32_t lb_key(const uint64_t* k, uint32_t lo, uint32_t hi, const MKey<KW>& v) {
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (MKey<KW>::load(k, m) < v) lo = m + 1; else hi = m; }
    return lo;
}
// exclusive block scan of three counters (MH_T threads); returns the block totals in tot[]
__device__ inline void block_scan3(uint32_t x[3], uint32_t tot[3]) {
    __shared__ uint32_t sh[3][MH_T / WAVE];
    const int lane = (int)__lane_id(), w = (int)threadIdx.x / WAVE;
    uint32_t inc[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        uint32_t v = x[c];
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
            const uint32_t y = __shfl_up(v, d);
            if (lane >= d) v += y;
        }
        inc[c] = v;
        if (lane == WAVE - 1) sh[c][w] = v;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        uint32_t before = 0, all = 0;
        for (int k = 0; k < MH_T / WAVE; ++k) { if (k < w) before += sh[c][k]; all += sh[c][k]; }
        x[c] = before + inc[c] - x[c];
        tot[c] = all;
    }
    __syncthreads();
}

template <int NV, bool WRITE, int KW>
static __global__ __launch_bounds__(MH_T) void k_merge_heavy(MergeArgs a) {
    constexpr uint32_t INF = 0xFFFFFFFFu;
    __shared__ uint32_t sU[WRITE ? MH_LDS : 1];
    if (WRITE && a.spec_bad && *a.spec_bad) return;
    const uint32_t H = *a.hcount;
    for (uint32_t hi = blockIdx.x; hi < H; hi += gridDim.x) {
        const uint32_t t = a.hlist[hi];
        int64_t rv[NV];
        uint32_t tb[NV], tc[NV], kb[NV], nk[NV], mb[NV];
        int pv = 0, pk = 0;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            rv[v] = a.row[v] ? (int64_t)a.row[v][t] : (int64_t)t;
            const bool has = rv[v] >= 0;
            tc[v] = has ? a.tcnt[v][rv[v]] : 0u;
            tb[v] = has ? a.ent_off[v][rv[v]] : 0u;
            kb[v] = has ? a.key_off[v][rv[v]] : 0u;
            nk[v] = has ? a.key_off[v][rv[v] + 1] - kb[v] : 0u;
            mb[v] = has ? a.k2t_off[v][rv[v]] : 0u;
            if (tc[v] > tc[pv]) pv = v;
            if (nk[v] > nk[pk]) pk = v;
        }
        // replies identical in every view (the usual case for long lists: they differ only where a view dropped an
        // in-flight dependency, and a txn's in-window deps are few): the union is any one of them — a streaming
        // compare of the views, then a copy of view 0 with its own offsets (the merged TxnId list is the same list,
        // so the per-key entries' TxnId indices carry over unchanged)
        {
            bool same = rv[0] >= 0;
#pragma unroll
            for (int v = 1; v < NV; ++v) same = same && rv[v] >= 0 && tc[v] == tc[0] && nk[v] == nk[0];
            const uint32_t klen = nk[0] ? (uint32_t)a.k2t[0][mb[0] + nk[0] - 1] : 0u;   // header + entries
#pragma unroll
            for (int v = 1; v < NV; ++v) same = same && (nk[v] ? (uint32_t)a.k2t[v][mb[v] + nk[v] - 1] : 0u) == klen;
            if (same && WRITE && a.hsame) {
                same = a.hsame[t] != 0;                      // the count pass compared the views
            } else if (same) {
                bool diff = false;
                for (uint32_t i = threadIdx.x; i < tc[0] && !diff; i += MH_T) {
                    const uint32_t x = a.txns[0][tb[0] + i];
#pragma unroll
                    for (int v = 1; v < NV; ++v) diff |= a.txns[v][tb[v] + i] != x;
                }
                for (uint32_t i = threadIdx.x; i < KW * nk[0] && !diff; i += MH_T) {
                    const uint64_t x = a.keys[0][(size_t)KW * kb[0] + i];
#pragma unroll
                    for (int v = 1; v < NV; ++v) diff |= a.keys[v][(size_t)KW * kb[v] + i] != x;
                }
                for (uint32_t i = threadIdx.x; i < klen && !diff; i += MH_T) {
                    const int32_t x = a.k2t[0][mb[0] + i];
#pragma unroll
                    for (int v = 1; v < NV; ++v) diff |= a.k2t[v][mb[v] + i] != x;
                }
                same = !__syncthreads_or(diff ? 1 : 0);
                if (!WRITE && a.hsame && threadIdx.x == 0) a.hsame[t] = same ? 1 : 0;
            }
            if (same) {
                if (!WRITE) {
                    if (threadIdx.x == 0) { a.mk[t] = nk[0]; a.me[t] = klen - nk[0]; a.mu[t] = tc[0]; }
                } else {
                    uint32_t* ot = a.o_txns + a.o_ent_off[t];
                    for (uint32_t i = threadIdx.x; i < tc[0]; i += MH_T) ot[i] = a.txns[0][tb[0] + i];
                    uint64_t* okk = a.o_keys + (size_t)KW * a.o_key_off[t];
                    for (uint32_t i = threadIdx.x; i < KW * nk[0]; i += MH_T) okk[i] = a.keys[0][(size_t)KW * kb[0] + i];
                    int32_t* ok2 = a.o_k2t + a.o_k2t_off[t];
                    for (uint32_t i = threadIdx.x; i < klen; i += MH_T) ok2[i] = a.k2t[0][mb[0] + i];
                    if (threadIdx.x == 0) a.o_tcnt[t] = tc[0];
                }
                __syncthreads();
                continue;
            }
        }
        // chunk size: spread the larger of the two lists over the whole workgroup (a key Write's ~10^2-10^3 RangeDeps
        // used to keep 19 of 256 threads busy with fixed 32-item chunks), at least MCH_MIN items per chunk
        const uint32_t big = tc[pv] > nk[pk] ? tc[pv] : nk[pk];
        const uint32_t mch = max((uint32_t)MCH_MIN, (big + MH_T - 1) / MH_T);
        const uint32_t nT = (tc[pv] + mch - 1) / mch, nK = (nk[pk] + mch - 1) / mch;
        const uint32_t nch = nT > nK ? nT : nK;
        const uint32_t cpt = (nch + MH_T - 1) / MH_T;
        const uint32_t c0 = threadIdx.x * cpt, c1 = min(nch, c0 + cpt);
        // chunk c of the TxnIds: [T_pv[c*mch], T_pv[(c+1)*mch]) in every reply
        auto t_bounds = [&](uint32_t c, uint32_t* cur, uint32_t* end) {
            const uint32_t lo = c == 0 ? 0u : a.txns[pv][tb[pv] + c * mch];
            const uint32_t hiv = (c + 1) * mch < tc[pv] ? a.txns[pv][tb[pv] + (c + 1) * mch] : INF;
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const uint32_t b = tb[v], e = tb[v] + tc[v];
                cur[v] = c == 0 ? b : lb_u32(a.txns[v], b, e, lo);
                end[v] = hiv == INF ? e : lb_u32(a.txns[v], cur[v], e, hiv);
            }
        };
        auto k_bounds = [&](uint32_t c, uint32_t* kc, uint32_t* ke) {
            const bool first = c == 0, last = (c + 1) * mch >= nk[pk];
            const MKey<KW> lo = first ? MKey<KW>{0ull, 0ull} : MKey<KW>::load(a.keys[pk], kb[pk] + c * mch);
            const MKey<KW> hv = last ? MKey<KW>{0ull, 0ull} : MKey<KW>::load(a.keys[pk], kb[pk] + (c + 1) * mch);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                const uint32_t b = kb[v], e = kb[v] + nk[v];
                kc[v] = first ? b : lb_key<KW>(a.keys[v], b, e, lo);
                ke[v] = last ? e : lb_key<KW>(a.keys[v], kc[v], e, hv);
            }
        };
        // TxnId union of one chunk (count, or write at out[pos..])
        auto t_union = [&](uint32_t c, uint32_t* out) -> uint32_t {
            if (c >= nT) return 0u;
            uint32_t cur[NV], end[NV], head[NV];
            t_bounds(c, cur, end);
#pragma unroll
            for (int v = 0; v < NV; ++v) head[v] = cur[v] < end[v] ? a.txns[v][cur[v]] : INF;
            uint32_t m = 0;
            while (true) {
                uint32_t mn = INF;
#pragma unroll
                for (int v = 0; v < NV; ++v) mn = head[v] < mn ? head[v] : mn;
                if (mn == INF) break;
                if (out) out[m] = mn;
                ++m;
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    if (head[v] == mn) { ++cur[v]; head[v] = cur[v] < end[v] ? a.txns[v][cur[v]] : INF; }
            }
            return m;
        };
        // key union of one chunk: (keys, entries); write: keys at okey, header slots from kpos, entries from
        // ep (absolute k2t positions), TxnIds remapped into U[0, mu)
        auto k_union = [&](uint32_t c, bool wr, uint32_t kpos, uint32_t ep, const uint32_t* U, uint32_t mu,
                           uint32_t okb, uint32_t omb, uint32_t onk, uint32_t* n_e) -> uint32_t {
            *n_e = 0;
            if (c >= nK) return 0u;
            uint32_t kc[NV], ke[NV];
            k_bounds(c, kc, ke);
            uint32_t mk = 0, me = 0;
            while (true) {
                bool any = false;
                MKey<KW> kmin{0ull, 0ull};
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    if (kc[v] < ke[v]) {
                        MKey<KW> k = MKey<KW>::load(a.keys[v], kc[v]);
                        if (!any || k < kmin) { kmin = k; any = true; }
                    }
                }
                if (!any) break;
                uint32_t lc[NV], le[NV], lh[NV];
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    lc[v] = 0; le[v] = 0; lh[v] = INF;
                    if (kc[v] < ke[v] && MKey<KW>::load(a.keys[v], kc[v]) == kmin) {
                        const uint32_t ki = kc[v] - kb[v];
                        lc[v] = mb[v] + (ki == 0 ? nk[v] : (uint32_t)a.k2t[v][mb[v] + ki - 1]);
                        le[v] = mb[v] + (uint32_t)a.k2t[v][mb[v] + ki];
                        lh[v] = lc[v] < le[v] ? a.txns[v][tb[v] + (uint32_t)a.k2t[v][lc[v]]] : INF;
                        ++kc[v];
                    }
                }
                uint32_t x = 0;
                while (true) {
                    uint32_t mn = INF;
#pragma unroll
                    for (int v = 0; v < NV; ++v) mn = lh[v] < mn ? lh[v] : mn;
                    if (mn == INF) break;
                    if (wr) {
                        x = lb_u32(U, x, mu, mn);       // U: the LDS copy when it fits
                        a.o_k2t[ep++] = (int32_t)x;
                    }
                    ++me;
#pragma unroll
                    for (int v = 0; v < NV; ++v)
                        if (lh[v] == mn) { ++lc[v]; lh[v] = lc[v] < le[v] ? a.txns[v][tb[v] + (uint32_t)a.k2t[v][lc[v]]] : INF; }
                }
                if (wr) {
                    a.o_keys[KW * (size_t)(okb + kpos + mk)] = kmin.a;
                    if (KW == 2) a.o_keys[KW * (size_t)(okb + kpos + mk) + 1] = kmin.b;
                    a.o_k2t[omb + kpos + mk] = (int32_t)(ep - omb);
                }
                ++mk;
            }
            (void)onk;
            *n_e = me;
            return mk;
        };
        uint32_t x[3] = {0, 0, 0}, tot[3];
        if (!WRITE) {
            for (uint32_t c = c0; c < c1; ++c) {
                x[2] += t_union(c, nullptr);
                uint32_t ne;
                x[0] += k_union(c, false, 0, 0, nullptr, 0, 0, 0, 0, &ne);
                x[1] += ne;
            }
            block_scan3(x, tot);
            if (threadIdx.x == 0) { a.mk[t] = tot[0]; a.me[t] = tot[1]; a.mu[t] = tot[2]; }
        } else {
            uint32_t* Ug = a.o_txns + a.o_ent_off[t];
            for (uint32_t c = c0; c < c1; ++c) x[2] += t_union(c, nullptr);
            block_scan3(x, tot);
            uint32_t pos = x[2];
            for (uint32_t c = c0; c < c1; ++c) pos += t_union(c, Ug + pos);
            const uint32_t mu = tot[2];
            __threadfence_block();
            __syncthreads();
            const uint32_t* U = Ug;
            if (mu <= MH_LDS) {
                for (uint32_t i = threadIdx.x; i < mu; i += MH_T) sU[i] = Ug[i];
                __syncthreads();
                U = sU;
            }
            // keys: per-thread (keys, entries) totals, then the writes
            x[0] = x[1] = x[2] = 0;
            for (uint32_t c = c0; c < c1; ++c) {
                uint32_t ne;
                x[0] += k_union(c, false, 0, 0, nullptr, 0, 0, 0, 0, &ne);
                x[1] += ne;
            }
            block_scan3(x, tot);
            const uint32_t okb = a.o_key_off[t], omb = a.o_k2t_off[t];
            const uint32_t onk = a.o_key_off[t + 1] - okb;
            uint32_t kpos = x[0], ep = omb + onk + x[1];
            for (uint32_t c = c0; c < c1; ++c) {
                uint32_t ne;
                kpos += k_union(c, true, kpos, ep, U, mu, okb, omb, onk, &ne);
                ep += ne;
            }
            if (threadIdx.x == 0) a.o_tcnt[t] = mu;
        }
        __syncthreads();
    }
}

// Offsets of K merged outputs from the count pass, in one scan: state (keys, entries, TxnIds) x K.
template <int K>
struct MultiOffsetsOp {
    struct S { uint32_t k[K], e[K], u[K]; };
    size_t n;
    const uint32_t* mk;           // [k * n + t]
    const uint32_t* me;
    const uint32_t* mu;
    uint32_t* key_off[K];
    uint32_t* ent_off[K];
    uint32_t* k2t_off[K];
    __device__ S identity() const {
        S s;
#pragma unroll
        for (int c = 0; c < K; ++c) { s.k[c] = 0; s.e[c] = 0; s.u[c] = 0; }
        return s;
    }
    __device__ S load(size_t t) const {
        S s;
#pragma unroll
        for (int c = 0; c < K; ++c) { s.k[c] = mk[c * n + t]; s.e[c] = me[c * n + t]; s.u[c] = mu[c * n + t]; }
        return s;
    }
    __device__ S combine(const S& x, const S& y) const {
        S r;
#pragma unroll
        for (int c = 0; c < K; ++c) { r.k[c] = x.k[c] + y.k[c]; r.e[c] = x.e[c] + y.e[c]; r.u[c] = x.u[c] + y.u[c]; }
        return r;
    }
    __device__ void store(size_t t, const S& ex, const S& inc, const S&) const {
#pragma unroll
        for (int c = 0; c < K; ++c) {
            key_off[c][t] = ex.k[c];
            ent_off[c][t] = ex.u[c];
            k2t_off[c][t] = ex.k[c] + ex.e[c];
            if (t + 1 == n) { key_off[c][n] = inc.k[c]; ent_off[c][n] = inc.u[c]; k2t_off[c][n] = inc.k[c] + inc.e[c]; }
        }
    }
};

// Uploaded replies (ad_merge_host): per-txn unique-TxnId counts from the compacted txn_off.
static __global__ __launch_bounds__(256) void k_tcnt_from_off(size_t n, const uint32_t* __restrict__ off, uint32_t* __restrict__ tcnt) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) tcnt[t] = off[t + 1] - off[t];
}

template <int NV>
inline void merge_launch_nv(const MergeArgs& a, bool write, int kw, hipStream_t st) {
    const int g = ceil_div((long)a.n, 256);
    {
    KScope ks(write ? K_MERGE_WRITE : K_MERGE_COUNT, a.n);
    if (kw == 2) {
        if (write) k_merge<NV, true, 2><<<g, 256, 0, st>>>(a);
        else k_merge<NV, false, 2><<<g, 256, 0, st>>>(a);
    } else {
        if (write) k_merge<NV, true, 1><<<g, 256, 0, st>>>(a);
        else k_merge<NV, false, 1><<<g, 256, 0, st>>>(a);
    }
    }
    if (!a.hlist) return;
    const int gh = std::min<int>(g, MH_GRID);
    KScope kh(write ? K_MERGE_HEAVY_WRITE : K_MERGE_HEAVY_COUNT);
    if (kw == 2) {
        if (write) k_merge_heavy<NV, true, 2><<<gh, MH_T, 0, st>>>(a);
        else k_merge_heavy<NV, false, 2><<<gh, MH_T, 0, st>>>(a);
    } else {
        if (write) k_merge_heavy<NV, true, 1><<<gh, MH_T, 0, st>>>(a);
        else k_merge_heavy<NV, false, 1><<<gh, MH_T, 0, st>>>(a);
    }
}

// ---------------------------------------------------------------------------------------------------
// Deps.merge of the R replies in one pass without a count pass, offsets scan or host round trip (k_merge_ref; key
// classes of batches whose deps stage saw no heavy txn).
//
// LinearMerger / linearUnion return an input unchanged when it already is the union (RelationMultiMap.java:583-589:
// "one side is a superset").  Replies differ only where a replica dropped an in-flight dependency, so for nearly every
// txn (C2: all but ~12 of 1M) the replies that have deps are identical: k_merge_ref, one thread per txn, compares them
// word for word and records the txn's merged row as a REFERENCE to that reply's row (src[t] = its view; MC_EMPTY when
// no reply has deps).  Every other txn is merged by its own thread right after (such txns are rare: a wave that holds one
// runs the merge, the others do not) — in registers for small replies (<= 8 TxnIds, <= 4 keys, <= 12 keysToTxnIds words
// per view):
//   - TxnId union: an id is OWNED by the first view that lists it; its merged position is the number of owned
//     ids below it (compares only, no data-dependent register indexing);
//   - keys: the same ownership / rank on the keys;
//   - per merged key the set of merged TxnId positions is a bitmask: each view's per-key index list (the
//     keysToTxnIds entries between two header ends) becomes a mask over its own ids, remapped through the ranks
//     (remapToSuperset, SortedArrays.java:1249-1275) and OR-ed into the merged key's mask (the per-key
//     linearUnion, RelationMultiMap.java:562-816); set bits in ascending order are the sorted index list;
// else with k_merge's serial R-way merge-path loops — into a region whose space each wave claims with one atomic per
// counter, the txn's place recorded in the list arrays (lidx[t] -> l_*).  merged_ready() turns references + merged rows into the exact CSR when something reads it (fetch, levels over
// merged deps, recovery, inverse); a key batch's pipeline reads nothing of it.  Merged entries per workgroup go to
// part[] (the host sums them lazily).
// ---------------------------------------------------------------------------------------------------
constexpr uint8_t MC_EMPTY = 0xFE, MC_LIST = 0xFF;
struct MergeCapArgs {
    size_t n;
    const uint32_t* key_off[MAXV];
    const uint64_t* keys[MAXV];
    const uint32_t* k2t_off[MAXV];
    const int32_t* k2t[MAXV];
    const uint32_t* ent_off[MAXV];
    const uint32_t* txns[MAXV];
    const uint32_t* tcnt[MAXV];
    uint8_t* src;                                   // [n] the reply the merged row equals, MC_EMPTY or MC_LIST
    uint32_t* lidx;                                 // [n] a merged txn's index in the list arrays
    uint32_t* list;                                 // (unused)
    uint32_t* cnt;                                  // this call's counters: [0] merged txns, [1..3] region keys / words / ids
    uint32_t* cnt_next;                             // the next call's (this call zeroes them)
    uint32_t *l_koff, *l_moff, *l_toff;             // [list] a merged row's place in the region
    uint32_t *l_kcnt, *l_ment, *l_tcnt;             // [list] its keys / keysToTxnIds entries / TxnIds
    uint64_t* o_keys;                               // the region (capacity: the replies' totals summed)
    int32_t* o_k2t;
    uint32_t* o_txns;
    uint32_t* part;                                 // [gridDim.x] merged entries per workgroup
    uint32_t part2;
};
constexpr int MC_T = 8, MC_K = 4, MC_S = 12;

// Serial merge of one txn's replies into its capacity region (any sizes).
template <int NV>
__device__ inline void merge_cap_serial(const MergeCapArgs& a, const uint32_t* kb, const uint32_t* nk, const uint32_t* mb,
                                        const uint32_t* tb, const uint32_t* tc, uint32_t okb, uint32_t omb, uint32_t otb,
                                        uint32_t& okc, uint32_t& oent, uint32_t& otc) {
    constexpr uint32_t INF = 0xFFFFFFFFu;
    uint32_t cur[NV], head[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) { cur[v] = tb[v]; head[v] = tc[v] ? a.txns[v][cur[v]] : INF; }
    uint32_t* out = a.o_txns + otb;
    uint32_t mu = 0;
    while (true) {
        uint32_t mn = INF;
#pragma unroll
        for (int v = 0; v < NV; ++v) mn = head[v] < mn ? head[v] : mn;
        if (mn == INF) break;
        out[mu++] = mn;
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (head[v] == mn) { ++cur[v]; head[v] = cur[v] < tb[v] + tc[v] ? a.txns[v][cur[v]] : INF; }
    }
    // merged key count first: the keysToTxnIds header (one end offset per key) precedes the entries
    uint32_t kc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) kc[v] = kb[v];
    uint32_t mk = 0;
    while (true) {
        bool any = false;
        uint64_t kmin = 0;
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (kc[v] < kb[v] + nk[v]) { const uint64_t k = a.keys[v][kc[v]]; if (!any || k < kmin) { kmin = k; any = true; } }
        if (!any) break;
#pragma unroll
        for (int v = 0; v < NV; ++v) if (kc[v] < kb[v] + nk[v] && a.keys[v][kc[v]] == kmin) ++kc[v];
        ++mk;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) kc[v] = kb[v];
    uint32_t ep = omb + mk, j = 0;
    while (true) {
        bool any = false;
        uint64_t kmin = 0;
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (kc[v] < kb[v] + nk[v]) { const uint64_t k = a.keys[v][kc[v]]; if (!any || k < kmin) { kmin = k; any = true; } }
        if (!any) break;
        uint32_t lc[NV], le[NV], lh[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            lc[v] = 0; le[v] = 0; lh[v] = INF;
            if (kc[v] < kb[v] + nk[v] && a.keys[v][kc[v]] == kmin) {
                const uint32_t ki = kc[v] - kb[v];
                lc[v] = mb[v] + (ki == 0 ? nk[v] : (uint32_t)a.k2t[v][mb[v] + ki - 1]);
                le[v] = mb[v] + (uint32_t)a.k2t[v][mb[v] + ki];
                lh[v] = lc[v] < le[v] ? a.txns[v][tb[v] + (uint32_t)a.k2t[v][lc[v]]] : INF;
                ++kc[v];
            }
        }
        uint32_t x = 0;
        while (true) {
            uint32_t mn = INF;
#pragma unroll
            for (int v = 0; v < NV; ++v) mn = lh[v] < mn ? lh[v] : mn;
            if (mn == INF) break;
            while (out[x] < mn) ++x;
            a.o_k2t[ep++] = (int32_t)x;
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (lh[v] == mn) { ++lc[v]; lh[v] = lc[v] < le[v] ? a.txns[v][tb[v] + (uint32_t)a.k2t[v][lc[v]]] : INF; }
        }
        a.o_keys[okb + j] = kmin;
        a.o_k2t[omb + j] = (int32_t)(ep - omb);
        ++j;
    }
    okc = mk; oent = ep - omb - mk; otc = mu;
}

// Register merge of small replies (NV <= 4); false when the merged keys exceed MC_K (then nothing was written).
template <int NV>
__device__ inline bool merge_cap_small(const MergeCapArgs& a, const uint32_t* kb, const uint32_t* nk, const uint32_t* mb,
                                       const uint32_t* ms, const uint32_t* tb, const uint32_t* tc, uint32_t okb, uint32_t omb,
                                       uint32_t otb, uint32_t& okc, uint32_t& oent, uint32_t& otc) {
    constexpr uint32_t INF = 0xFFFFFFFFu;
    uint32_t T[NV][MC_T];
    uint64_t K[NV][MC_K];
    int32_t S[NV][MC_S];
    // every load unconditional, at an index clamped into the reply's own list (a conditional load merged with a
    // constant at a branch join makes the compiler wait for each load before the next: one latency per slot); a reply
    // without deps reads element 0 (every buffer holds at least 256 bytes)
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const bool h = tc[v] != 0;
#pragma unroll
        for (int s = 0; s < MC_T; ++s) {
            const uint32_t x = a.txns[v][h ? tb[v] + min((uint32_t)s, tc[v] - 1) : 0u];
            T[v][s] = (uint32_t)s < tc[v] ? x : INF;
        }
#pragma unroll
        for (int i = 0; i < MC_K; ++i) {
            const uint64_t x = a.keys[v][h ? kb[v] + min((uint32_t)i, nk[v] - 1) : 0u];
            K[v][i] = (uint32_t)i < nk[v] ? x : 0ull;
        }
#pragma unroll
        for (int s = 0; s < MC_S; ++s) {
            const int32_t x = a.k2t[v][h ? mb[v] + min((uint32_t)s, ms[v] - 1) : 0u];
            S[v][s] = (uint32_t)s < ms[v] ? x : 0;
        }
    }
    // keys: ownership (first view listing the key) and merged positions
    uint32_t kown[NV], nkm = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        kown[v] = 0;
#pragma unroll
        for (int i = 0; i < MC_K; ++i) {
            bool o = (uint32_t)i < nk[v];
#pragma unroll
            for (int w = 0; w < v; ++w)
#pragma unroll
                for (int i2 = 0; i2 < MC_K; ++i2) o = o && !((uint32_t)i2 < nk[w] && K[w][i2] == K[v][i]);
            kown[v] |= (o ? 1u : 0u) << i;
        }
        nkm += (uint32_t)__popc(kown[v]);
    }
    if (nkm > (uint32_t)MC_K) return false;
    // per view: its per-key index lists as masks, key i in bits [8i, 8i + 8) (entry slots s >= nk: key = #ends <= s)
    uint32_t m[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        m[v] = 0;
#pragma unroll
        for (int s = 0; s < MC_S; ++s) {
            if ((uint32_t)s >= nk[v] && (uint32_t)s < ms[v]) {
                uint32_t ki = 0;
#pragma unroll
                for (int j = 0; j < MC_K; ++j) ki += ((uint32_t)j < nk[v] && S[v][j] <= s) ? 1u : 0u;
                m[v] |= 1u << (8 * ki + (uint32_t)S[v][s]);
            }
        }
    }
    // TxnIds: ownership, merged positions, the owned ids written at their positions
    uint32_t own[NV], nu = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        own[v] = 0;
#pragma unroll
        for (int s = 0; s < MC_T; ++s) {
            bool o = (uint32_t)s < tc[v];
#pragma unroll
            for (int w = 0; w < v; ++w)
#pragma unroll
                for (int s2 = 0; s2 < MC_T; ++s2) o = o && T[w][s2] != T[v][s];
            own[v] |= (o ? 1u : 0u) << s;
        }
        nu += (uint32_t)__popc(own[v]);
    }
    uint32_t R[NV][MC_T];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int s = 0; s < MC_T; ++s) {
            uint32_t r = 0;
#pragma unroll
            for (int w = 0; w < NV; ++w)
#pragma unroll
                for (int s2 = 0; s2 < MC_T; ++s2) r += ((own[w] >> s2 & 1u) && T[w][s2] < T[v][s]) ? 1u : 0u;
            R[v][s] = r;
            if (own[v] >> s & 1u) a.o_txns[otb + r] = T[v][s];
        }
    // per merged key: the mask of merged TxnId positions
    uint32_t M[MC_K];
#pragma unroll
    for (int j = 0; j < MC_K; ++j) M[j] = 0;
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int i = 0; i < MC_K; ++i) {
            if ((uint32_t)i >= nk[v]) continue;
            uint32_t kr = 0;
#pragma unroll
            for (int w = 0; w < NV; ++w)
#pragma unroll
                for (int i2 = 0; i2 < MC_K; ++i2) kr += ((kown[w] >> i2 & 1u) && K[w][i2] < K[v][i]) ? 1u : 0u;
            uint32_t B = 0;
#pragma unroll
            for (int e = 0; e < MC_T; ++e) B |= ((m[v] >> (8 * i + e)) & 1u) << R[v][e];
#pragma unroll
            for (int j = 0; j < MC_K; ++j) M[j] |= kr == (uint32_t)j ? B : 0u;
            if (kown[v] >> i & 1u) a.o_keys[okb + kr] = K[v][i];
        }
    uint32_t run = nkm;
#pragma unroll
    for (int j = 0; j < MC_K; ++j) {
        if ((uint32_t)j >= nkm) break;
        uint32_t x = M[j];
        while (x) { a.o_k2t[omb + run++] = __ffs(x) - 1; x &= x - 1; }
        a.o_k2t[omb + j] = (int32_t)run;
    }
    okc = nkm; oent = run - nkm; otc = nu;
    return true;
}

// Block sum of one value per thread (256 threads) -> out (thread 0)
__device__ inline void merge_cap_block_sum(uint32_t v, uint32_t* out) {
    __shared__ uint32_t sh[256 / WAVE];
#pragma unroll
    for (int d = WAVE / 2; d > 0; d >>= 1) v += __shfl_xor(v, d);
    if (__lane_id() == 0) sh[threadIdx.x / WAVE] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < 256 / WAVE; ++w) s += sh[w];
        *out = s;
    }
}

// (at most 128 VGPRs — 4 waves per SIMD for the compare pass; the rare inline merge may spill)
template <int NV>
static __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_merge_ref(MergeCapArgs a) {
    constexpr uint32_t INF = 0xFFFFFFFFu;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t ent = 0;
    bool defer = false;
    if (t < a.n) {
        uint32_t kb[NV], nk[NV], mb[NV], ms[NV], tb[NV], tc[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            kb[v] = a.key_off[v][t]; nk[v] = a.key_off[v][t + 1] - kb[v];
            mb[v] = a.k2t_off[v][t]; ms[v] = a.k2t_off[v][t + 1] - mb[v];
            tb[v] = a.ent_off[v][t]; tc[v] = a.tcnt[v][t];
        }
        uint32_t any = 0;
#pragma unroll
        for (int v = 0; v < NV; ++v) any |= tc[v];
        uint8_t src = MC_EMPTY;
        if (any) {
            // the first reply with deps (f); every other reply with deps must have its shape (and fit the registers)
            uint32_t fkb = 0, fnk = 0, fmb = 0, fms = 0, ftb = 0, ftc = 0;
            int fi = NV;
#pragma unroll
            for (int v = NV - 1; v >= 0; --v)
                if (tc[v]) { fkb = kb[v]; fnk = nk[v]; fmb = mb[v]; fms = ms[v]; ftb = tb[v]; ftc = tc[v]; fi = v; }
            bool same = ftc <= (uint32_t)MC_T && fnk <= (uint32_t)MC_K && fms <= (uint32_t)MC_S;
#pragma unroll
            for (int v = 0; v < NV; ++v) same = same && (tc[v] == 0 || (tc[v] == ftc && nk[v] == fnk && ms[v] == fms));
            if (same) {
                const uint32_t* ft = a.txns[0];
                const uint64_t* fk = a.keys[0];
                const int32_t* fm = a.k2t[0];
#pragma unroll
                for (int v = 1; v < NV; ++v) if (fi == v) { ft = a.txns[v]; fk = a.keys[v]; fm = a.k2t[v]; }
                // every load unconditional, at an index clamped into the list (f has deps: ftc, fnk >= 1, fms >= 2); the
                // differences OR-ed under masks — arithmetic, not short-circuit tests: a branch around a compare sinks its
                // load into it, one memory latency per slot
                uint32_t T[MC_T];
                uint64_t K[MC_K];
                uint32_t S[MC_S];
#pragma unroll
                for (int s = 0; s < MC_T; ++s) T[s] = ft[ftb + min((uint32_t)s, ftc - 1)];
#pragma unroll
                for (int i = 0; i < MC_K; ++i) K[i] = fk[fkb + min((uint32_t)i, fnk - 1)];
#pragma unroll
                for (int s = 0; s < MC_S; ++s) S[s] = (uint32_t)fm[fmb + min((uint32_t)s, fms - 1)];
                uint32_t diff = 0;
                uint64_t diffk = 0;
#pragma unroll
                for (int v = 1; v < NV; ++v) {                   // views after f (those before it have no deps)
                    const bool h = tc[v] != 0 && v > fi;
                    const uint32_t hm = h ? ~0u : 0u;
#pragma unroll
                    for (int s = 0; s < MC_T; ++s) {
                        const uint32_t x = a.txns[v][h ? tb[v] + min((uint32_t)s, ftc - 1) : 0u];
                        diff |= (x ^ T[s]) & ((uint32_t)s < ftc ? hm : 0u);
                    }
#pragma unroll
                    for (int i = 0; i < MC_K; ++i) {
                        const uint64_t x = a.keys[v][h ? kb[v] + min((uint32_t)i, fnk - 1) : 0u];
                        diffk |= (x ^ K[i]) & ((uint32_t)i < fnk && h ? ~0ull : 0ull);
                    }
#pragma unroll
                    for (int s = 0; s < MC_S; ++s) {
                        const uint32_t x = (uint32_t)a.k2t[v][h ? mb[v] + min((uint32_t)s, fms - 1) : 0u];
                        diff |= (x ^ S[s]) & ((uint32_t)s < fms ? hm : 0u);
                    }
                }
                same = diff == 0 && diffk == 0;
                (void)INF;
            }
            if (same) { src = (uint8_t)fi; ent = fms - fnk; }
            else { src = MC_LIST; defer = true; }
        }
        a.src[t] = src;
    }
    // txns whose replies differ (C2: ~12 of 1M) are merged right here: a listed txn's wave claims the region space of
    // its listed lanes (the replies' sizes summed) with one atomic per counter, then each such lane merges its txn
    if (__ballot(defer)) {
        const size_t tt = defer ? t : 0;
        uint32_t kb[NV], nk[NV], mb[NV], ms[NV], tb[NV], tc[NV];
        bool small = NV <= 4;
        uint32_t ck = 0, cm = 0, ct = 0;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            kb[v] = a.key_off[v][tt]; nk[v] = a.key_off[v][tt + 1] - kb[v];
            mb[v] = a.k2t_off[v][tt]; ms[v] = a.k2t_off[v][tt + 1] - mb[v];
            tb[v] = a.ent_off[v][tt]; tc[v] = a.tcnt[v][tt];
            if (!defer) { nk[v] = ms[v] = tc[v] = 0; }
            ck += nk[v]; cm += ms[v]; ct += tc[v];
            small = small && tc[v] <= (uint32_t)MC_T && nk[v] <= (uint32_t)MC_K && ms[v] <= (uint32_t)MC_S;
        }
        uint32_t sk = ck, sm = cm, st = ct;
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
            const uint32_t yk = __shfl_up(sk, d), ym = __shfl_up(sm, d), yt = __shfl_up(st, d);
            if ((int)__lane_id() >= d) { sk += yk; sm += ym; st += yt; }
        }
        const uint64_t lm = __ballot(defer);
        uint32_t bk = 0, bm = 0, bt = 0, bl = 0;
        if (__lane_id() == WAVE - 1) {
            bk = atomicAdd(a.cnt + 1, sk); bm = atomicAdd(a.cnt + 2, sm); bt = atomicAdd(a.cnt + 3, st);
            bl = atomicAdd(a.cnt, (uint32_t)__popcll(lm));
        }
        bk = __shfl(bk, WAVE - 1); bm = __shfl(bm, WAVE - 1); bt = __shfl(bt, WAVE - 1); bl = __shfl(bl, WAVE - 1);
        if (defer) {
            const uint32_t x = bl + (uint32_t)__popcll(lm & ((1ull << __lane_id()) - 1ull));
            const uint32_t okb = bk + sk - ck, omb = bm + sm - cm, otb = bt + st - ct;
            uint32_t okc = 0, oent = 0, otc = 0;
            bool done = false;
            if constexpr (NV <= 4) {
                if (small) done = merge_cap_small<NV>(a, kb, nk, mb, ms, tb, tc, okb, omb, otb, okc, oent, otc);
            }
            if (!done) merge_cap_serial<NV>(a, kb, nk, mb, tb, tc, okb, omb, otb, okc, oent, otc);
            a.l_koff[x] = okb; a.l_moff[x] = omb; a.l_toff[x] = otb;
            a.l_kcnt[x] = okc; a.l_ment[x] = oent; a.l_tcnt[x] = otc;
            a.lidx[t] = x;
            ent = oent;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 4) a.cnt_next[threadIdx.x] = 0u;    // the next call's counters
    merge_cap_block_sum(ent, a.part + blockIdx.x);
}

// merged_ready: per txn the merged row's counts (from the reply it references, or its merged row), then (after an
// exclusive scan, MultiOffsetsOp) the copy into the exact CSR — outside the pipeline.
template <int NV>
static __global__ __launch_bounds__(256) void k_merge_ready_counts(MergeCapArgs a, uint32_t* kcnt, uint32_t* ment, uint32_t* tcnt) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint8_t s = a.src[t];
    uint32_t k = 0, m = 0, c = 0;
    if (s == MC_LIST) {
        const uint32_t x = a.lidx[t];
        k = a.l_kcnt[x]; m = a.l_ment[x]; c = a.l_tcnt[x];
    } else if (s != MC_EMPTY) {
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (v == s) {
                k = a.key_off[v][t + 1] - a.key_off[v][t];
                m = a.k2t_off[v][t + 1] - a.k2t_off[v][t] - k;
                c = a.tcnt[v][t];
            }
    }
    kcnt[t] = k; ment[t] = m; tcnt[t] = c;
}
template <int NV>
static __global__ __launch_bounds__(256) void k_merge_ready_copy(MergeCapArgs a, const uint32_t* __restrict__ xkoff,
                                                                  const uint32_t* __restrict__ xmoff, const uint32_t* __restrict__ xtoff,
                                                                  const uint32_t* __restrict__ kcnt, const uint32_t* __restrict__ ment,
                                                                  const uint32_t* __restrict__ tcnt, uint64_t* __restrict__ xkeys,
                                                                  int32_t* __restrict__ xk2t, uint32_t* __restrict__ xtxns) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint8_t s = a.src[t];
    if (s == MC_EMPTY) return;
    const uint64_t* keys = a.o_keys;
    const int32_t* k2t = a.o_k2t;
    const uint32_t* txns = a.o_txns;
    uint32_t kb = 0, mb = 0, tb = 0;
    if (s == MC_LIST) {
        const uint32_t x = a.lidx[t];
        kb = a.l_koff[x]; mb = a.l_moff[x]; tb = a.l_toff[x];
    } else {
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (v == s) { keys = a.keys[v]; k2t = a.k2t[v]; txns = a.txns[v]; kb = a.key_off[v][t]; mb = a.k2t_off[v][t]; tb = a.ent_off[v][t]; }
    }
    const uint32_t nk = kcnt[t], nm = nk + ment[t], nt = tcnt[t];
    for (uint32_t i = 0; i < nk; ++i) xkeys[xkoff[t] + i] = keys[kb + i];
    for (uint32_t i = 0; i < nm; ++i) xk2t[xmoff[t] + i] = k2t[mb + i];
    for (uint32_t i = 0; i < nt; ++i) xtxns[xtoff[t] + i] = txns[tb + i];
}

inline void merge_launch(const MergeArgs& a, int nv, bool write, int kw, hipStream_t st) {
    switch (nv) {
        case 1: merge_launch_nv<1>(a, write, kw, st); break;
        case 2: merge_launch_nv<2>(a, write, kw, st); break;
        case 3: merge_launch_nv<3>(a, write, kw, st); break;
        case 4: merge_launch_nv<4>(a, write, kw, st); break;
        case 5: merge_launch_nv<5>(a, write, kw, st); break;
        case 6: merge_launch_nv<6>(a, write, kw, st); break;
        case 7: merge_launch_nv<7>(a, write, kw, st); break;
        default: merge_launch_nv<8>(a, write, kw, st); break;
    }
}

}  // namespace ad
