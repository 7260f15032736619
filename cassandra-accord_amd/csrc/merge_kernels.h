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
};

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
__global__ __launch_bounds__(256) void k_merge(MergeArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
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
__global__ __launch_bounds__(256) void k_tcnt_from_off(size_t n, const uint32_t* __restrict__ off, uint32_t* __restrict__ tcnt) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) tcnt[t] = off[t + 1] - off[t];
}

template <int NV>
inline void merge_launch_nv(const MergeArgs& a, bool write, int kw, hipStream_t st) {
    const int g = ceil_div((long)a.n, 256);
    KScope ks(write ? K_MERGE_WRITE : K_MERGE_COUNT, a.n);
    if (kw == 2) {
        if (write) k_merge<NV, true, 2><<<g, 256, 0, st>>>(a);
        else k_merge<NV, false, 2><<<g, 256, 0, st>>>(a);
    } else {
        if (write) k_merge<NV, true, 1><<<g, 256, 0, st>>>(a);
        else k_merge<NV, false, 1><<<g, 256, 0, st>>>(a);
    }
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
