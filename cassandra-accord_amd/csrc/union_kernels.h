// union_kernels.h — virtual query items of large txns, and the per-txn TxnId union in LDS (gfx950).
//
// Large txns are range-domain txns (InMemorySafeStore.mapReduceActive visits every CommandsForKey key
// inside each range: commandsForKey.subMap(start, false, end, true), impl/InMemoryCommandStore.java:272-307)
// and key txns with more than KMAX keys.  Each (txn, distinct key) they query is a "virtual item":
// (txn i, key, segment start, insert position of TxnId i in the key's (key, TxnId)-sorted segment).
// Items of one txn are contiguous and in key order, so the KeyDeps layout is an in-order pass.
//
// k_union_lds is RelationMultiMap.AbstractBuilder.build's global value sort + index mapping
// (utils/RelationMultiMap.java:208-257) for one txn's CSR: a bitonic sort of the txn's dependency
// ranks in LDS, a compaction to the sorted unique TxnId list, and a binary-search remap of each
// keysToTxnIds entry to its index.  Used for large txns' key CSRs and every RangeDeps CSR.
#pragma once
#include "deps_kernels.h"

namespace ad {

__device__ inline uint32_t lb_u64(const uint64_t* a, uint32_t lo, uint32_t hi, uint64_t v) {   // first a[x] >= v
    while (lo < hi) {
        uint32_t m = (lo + hi) >> 1;
        if (a[m] < v) lo = m + 1; else hi = m;
    }
    return lo;
}
__device__ inline uint32_t ub_u64(const uint64_t* a, uint32_t lo, uint32_t hi, uint64_t v) {   // first a[x] > v
    while (lo < hi) {
        uint32_t m = (lo + hi) >> 1;
        if (a[m] <= v) lo = m + 1; else hi = m;
    }
    return lo;
}
__device__ inline uint32_t lb_u32(const uint32_t* a, uint32_t lo, uint32_t hi, uint32_t v) {   // first a[x] >= v
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (a[m] < v) lo = m + 1; else hi = m; }
    return lo;
}
__device__ inline uint32_t ub_u32(const uint32_t* a, uint32_t lo, uint32_t hi, uint32_t v) {   // first a[x] > v
    while (lo < hi) {
        uint32_t m = (lo + hi) >> 1;
        if (a[m] <= v) lo = m + 1; else hi = m;
    }
    return lo;
}

struct VItemArgs {
    size_t n;
    const uint8_t* meta;
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint32_t* range_off;
    const uint64_t* rs;
    const uint64_t* re;
    const uint32_t* e_txn;
    const uint64_t* ukey;        // [U] distinct keys
    const uint32_t* useg;        // [U+1]
    const Params* prm;           // n_keys_u
    uint32_t* vn;                // [n] items per txn (count pass)
    const uint32_t* voff;        // [n+1] (fill pass)
    uint32_t* vi_txn;
    uint32_t* vi_pos;
    uint32_t* vi_u;              // item -> distinct-key index (segment useg[u], key ukey[u])
    const uint32_t* qpos;        // executeAt-bound queries: per txn the bound's arrival position (nullable)
};

// CFK keys inside (s, e]  (EndInclusive: start excluded, end included)
__device__ inline void keys_in_range(const VItemArgs& a, uint32_t U, uint64_t s, uint64_t e, uint32_t& lo, uint32_t& hi) {
    lo = ub_u64(a.ukey, 0, U, s);
    hi = ub_u64(a.ukey, lo, U, e);
}

template <bool FILL>
static __global__ __launch_bounds__(256) void k_vitems(VItemArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t m = a.meta[t];
    if (!(m & META_LARGE)) {
        if (!FILL) a.vn[t] = 0;
        return;
    }
    const uint32_t U = a.prm->n_keys_u;
    if (meta_domain(m) == AD_DOMAIN_KEY) {
        const uint32_t b = a.key_off[t], e = a.key_off[t + 1];
        if (!FILL) { a.vn[t] = e - b; return; }
        uint32_t x = a.voff[t];
        for (uint32_t p = b; p < e; ++p, ++x) {
            // the pair's own sorted entry: its key's segment, then TxnId t inside it (byId order)
            const uint64_t k = a.keys[p];
            const uint32_t u = lb_u64(a.ukey, 0, U, k);
            const uint32_t s0 = a.useg[u], s1 = a.useg[u + 1];
            // PreAccept: the pair itself, walk [seg0, s); Accept: walk up to the bound's position (the txn's own
            // entry inside is skipped by the walk)
            const uint32_t s = a.qpos ? lb_u32(a.e_txn, s0, s1, a.qpos[t]) : ub_u32(a.e_txn, s0, s1, (uint32_t)t) - 1;
            a.vi_txn[x] = (uint32_t)t;
            a.vi_pos[x] = s;
            a.vi_u[x] = u;
        }
        return;
    }
    const uint32_t rb = a.range_off[t], rend = a.range_off[t + 1];
    uint32_t c = 0;
    uint32_t x = FILL ? a.voff[t] : 0u;
    for (uint32_t q = rb; q < rend; ++q) {
        uint32_t lo, hi;
        keys_in_range(a, U, a.rs[q], a.re[q], lo, hi);
        if (!FILL) { c += hi - lo; continue; }
        for (uint32_t u = lo; u < hi; ++u, ++x) {
            const uint32_t s0 = a.useg[u], s1 = a.useg[u + 1];
            a.vi_txn[x] = (uint32_t)t;
            // insertPos(bound): first entry with txn > t (PreAccept) / at or past the bound's position (Accept)
            a.vi_pos[x] = a.qpos ? lb_u32(a.e_txn, s0, s1, a.qpos[t]) : ub_u32(a.e_txn, s0, s1, (uint32_t)t);
            a.vi_u[x] = u;
        }
    }
    if (!FILL) a.vn[t] = c;
}

// Fill pass, one wave per large txn: the lanes stride over its items (a range txn's ~10^3-10^4 CFK keys were one
// thread's serial chain of binary searches: C4's fill pass was 130 ms of tail latency)
static __global__ __launch_bounds__(256) void k_vitems_fill(VItemArgs a) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n) return;
    const uint32_t m = a.meta[t];
    if (!(m & META_LARGE)) return;
    const uint32_t lane = (uint32_t)__lane_id();
    const uint32_t U = a.prm->n_keys_u;
    const uint32_t x0 = a.voff[t];
    if (meta_domain(m) == AD_DOMAIN_KEY) {
        const uint32_t b = a.key_off[t], e = a.key_off[t + 1];
        for (uint32_t p = b + lane; p < e; p += WAVE) {
            const uint64_t k = a.keys[p];
            const uint32_t u = lb_u64(a.ukey, 0, U, k);
            const uint32_t s0 = a.useg[u], s1 = a.useg[u + 1];
            const uint32_t s = a.qpos ? lb_u32(a.e_txn, s0, s1, a.qpos[t]) : ub_u32(a.e_txn, s0, s1, (uint32_t)t) - 1;
            const uint32_t x = x0 + (p - b);
            a.vi_txn[x] = (uint32_t)t;
            a.vi_pos[x] = s;
            a.vi_u[x] = u;
        }
        return;
    }
    uint32_t x = x0;
    for (uint32_t q = a.range_off[t]; q < a.range_off[t + 1]; ++q) {
        uint32_t lo, hi;
        keys_in_range(a, U, a.rs[q], a.re[q], lo, hi);
        for (uint32_t u = lo + lane; u < hi; u += WAVE) {
            const uint32_t s0 = a.useg[u], s1 = a.useg[u + 1];
            const uint32_t y = x + (u - lo);
            a.vi_txn[y] = (uint32_t)t;
            a.vi_pos[y] = a.qpos ? lb_u32(a.e_txn, s0, s1, a.qpos[t]) : ub_u32(a.e_txn, s0, s1, (uint32_t)t);
            a.vi_u[y] = u;
        }
        x += hi - lo;
    }
}

// ---------------------------------------------------------------------------------------------------
// Block-level helpers (256 threads)
// ---------------------------------------------------------------------------------------------------
constexpr int UB = 256;

// exclusive scan of one u32 per thread over an NT-thread block; returns the exclusive prefix, *total = sum
template <int NT = UB>
__device__ inline uint32_t block_scan_u32(uint32_t v, uint32_t* lds_w /* [NT/WAVE] */, uint32_t* total) {
    const int lane = __lane_id(), w = threadIdx.x / WAVE;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == WAVE - 1) lds_w[w] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NT / WAVE; ++k) {
        uint32_t s = lds_w[k];
        if (k < w) base += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// bitonic sort of n2 (a power of two) u32 in buf — LDS, or global memory owned by this block (same CU:
// the barrier orders the block's global accesses as it does its LDS ones)
template <int NT>
__device__ inline void bitonic_sort_block(uint32_t* buf, uint32_t n2) {
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t x = threadIdx.x; x < n2; x += NT) {
                const uint32_t y = x ^ j;
                if (y > x) {
                    const uint32_t a = buf[x], b = buf[y];
                    const bool up = (x & k) == 0;
                    if ((a > b) == up) { buf[x] = b; buf[y] = a; }
                }
            }
            __syncthreads();
        }
    }
}

constexpr int UNION_CAP = 8192;        // dependency entries of one txn's CSR sorted in LDS (32 KiB)
constexpr int UNION_CAP_BIG = 32768;   // overflow pass: 1024 threads, 128 KiB of LDS (gfx950: 160 KiB per CU)
constexpr int UB_BIG = 1024;

constexpr int UNION_CSRS = NVC_MAX + MAXV;   // key classes of every view, then RangeDeps of every view
struct LdsUnionArgs {
    size_t n;
    int ncsr;
    int csr_base;                      // this launch's CSRs are csr_base + k * csr_step, k < ncsr, of the tables
    int csr_step;                      //   (2: keyDeps classes only, the batch has no directKeyDeps)
    int only_large;
    const uint32_t* rows;              // only_large: the large txns' rows (grid x = their count), or null
    const uint32_t* rows_total;        //   their device-side count (guard)
    const uint8_t* meta;
    const uint32_t* key_off[UNION_CSRS];
    const uint32_t* k2t_off[UNION_CSRS];
    const uint32_t* ent_off[UNION_CSRS];
    int32_t* k2t[UNION_CSRS];
    uint32_t* txns[UNION_CSRS];
    uint32_t* tcnt[UNION_CSRS];
    Params* prm;
    // overflow: (txn, csr) pairs with more than UNION_CAP entries, for the big pass
    uint32_t* ovf_count;
    uint2* ovf;                        // {txn, csr}
    uint32_t ovf_cap;
    // small/medium split (RangeDeps launch): items above UNION_SMALL entries queued for the 256-thread pass
    uint32_t* med_count;
    uint2* med;                        // {txn, csr}
    // big pass
    const uint2* items;                // overflow items
    uint32_t* gbuf;                    // global sort space for items above UNION_CAP_BIG
    const uint64_t* gbuf_off;          // [item] offset into gbuf (u32 elements)
};

// Union of one (txn, CSR): sort the txn's per-key TxnId ranks in buf (n2 >= ne), unique them into the
// CSR's TxnId table, then remap every entry to its index (RelationMultiMap.java:201-260).
template <int NT>
__device__ inline uint32_t union_body(uint32_t* buf, uint32_t* wsum, int32_t* body, uint32_t ne, uint32_t* out, uint32_t* tcnt) {
    uint32_t n2 = 1;
    while (n2 < ne) n2 <<= 1;
    for (uint32_t x = threadIdx.x; x < n2; x += NT) buf[x] = x < ne ? (uint32_t)body[x] : 0xFFFFFFFFu;
    __syncthreads();
    bitonic_sort_block<NT>(buf, n2);
    // unique compaction: each thread owns a contiguous chunk
    const uint32_t per = (ne + NT - 1) / NT;
    const uint32_t b0 = min(ne, threadIdx.x * per), b1 = min(ne, b0 + per);
    uint32_t cnt = 0;
    for (uint32_t x = b0; x < b1; ++x) cnt += (x == 0 || buf[x] != buf[x - 1]) ? 1u : 0u;
    uint32_t total;
    uint32_t o = block_scan_u32<NT>(cnt, wsum, &total);
    for (uint32_t x = b0; x < b1; ++x)
        if (x == 0 || buf[x] != buf[x - 1]) out[o++] = buf[x];
    __syncthreads();
    // unique list back into buf, then remap every entry to its index
    for (uint32_t x = threadIdx.x; x < total; x += NT) buf[x] = out[x];
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < ne; x += NT) {
        const uint32_t v = (uint32_t)body[x];
        uint32_t lo = 0, hi = total;
        while (lo < hi) {
            uint32_t m = (lo + hi) >> 1;
            if (buf[m] < v) lo = m + 1; else hi = m;
        }
        body[x] = (int32_t)lo;
    }
    if (threadIdx.x == 0) *tcnt = total;
    return total;
}

// The union of one txn's CSR in several replica views (csr[v], v < nvw) at once.  The views' per-key lists differ
// only where a view dropped an in-flight dependency (rare for a given txn), and identical bodies have identical
// unions and remaps: the first view whose list fits `cap` is sorted, every view with an equal body (a streaming
// compare) receives a copy of its unique TxnId list (still in buf) and remapped body, the rest are sorted on
// their own.  Lists above cap go to too_big(v, csr).  Returns after a final barrier.
template <int NT, class TooBig>
__device__ inline void union_views(const LdsUnionArgs& a, uint32_t t, const int* csr, int nvw, uint32_t* buf, uint32_t* wsum,
                                   uint32_t cap, TooBig&& too_big) {
    uint32_t ne[MAXV], mb[MAXV], nk[MAXV];
    int r = -1;
    for (int v = 0; v < nvw; ++v) {
        const int c = csr[v];
        nk[v] = a.key_off[c][t + 1] - a.key_off[c][t];
        mb[v] = a.k2t_off[c][t];
        ne[v] = nk[v] ? a.k2t_off[c][t + 1] - mb[v] - nk[v] : 0u;
        if (nk[v] == 0) { if (threadIdx.x == 0) a.tcnt[c][t] = 0; continue; }
        if (ne[v] > cap) { if (threadIdx.x == 0) too_big(v, c); continue; }
        if (r < 0) r = v;
    }
    if (r < 0) return;
    const int cr = csr[r];
    int32_t* body_r = a.k2t[cr] + mb[r] + nk[r];
    uint32_t same = 0;
    for (int v = r + 1; v < nvw; ++v) {
        if (nk[v] == 0 || ne[v] > cap || ne[v] != ne[r]) continue;
        const int32_t* body_v = a.k2t[csr[v]] + mb[v] + nk[v];
        bool diff = false;
        for (uint32_t x = threadIdx.x; x < ne[r] && !diff; x += NT) diff = body_v[x] != body_r[x];
        if (!__syncthreads_or(diff ? 1 : 0)) same |= 1u << v;
    }
    const uint32_t tot = union_body<NT>(buf, wsum, body_r, ne[r], a.txns[cr] + a.ent_off[cr][t], &a.tcnt[cr][t]);
    // the copies first (buf still holds the reference's unique list), then the views that differ
    for (int v = r + 1; v < nvw; ++v) {
        if (!(same >> v & 1u)) continue;
        const int c = csr[v];
        int32_t* body_v = a.k2t[c] + mb[v] + nk[v];
        uint32_t* out = a.txns[c] + a.ent_off[c][t];
        for (uint32_t x = threadIdx.x; x < tot; x += NT) out[x] = buf[x];
        for (uint32_t x = threadIdx.x; x < ne[v]; x += NT) body_v[x] = body_r[x];   // this thread's own remaps
        if (threadIdx.x == 0) a.tcnt[c][t] = tot;
    }
    for (int v = r + 1; v < nvw; ++v) {
        const int c = csr[v];
        if (nk[v] == 0 || ne[v] > cap || (same >> v & 1u)) continue;
        __syncthreads();
        union_body<NT>(buf, wsum, a.k2t[c] + mb[v] + nk[v], ne[v], a.txns[c] + a.ent_off[c][t], &a.tcnt[c][t]);
    }
    __syncthreads();
}

// the rows of the large txns (the key-CSR launch only has work there: C4's 4M-row grid x 6 CSRs launched
// 24M mostly empty workgroups for ~4*10^5 range txns)
struct LargeRowsOp {
    using S = uint32_t;
    const uint8_t* meta;
    uint32_t* out;
    uint32_t* total;
    size_t n;
    __device__ S load(size_t i) const { return (meta[i] & META_LARGE) ? 1u : 0u; }
    __device__ S identity() const { return 0u; }
    __device__ S combine(S a, S b) const { return a + b; }
    __device__ void store(size_t i, S ex, S inc, S el) const {
        if (el) out[ex] = (uint32_t)i;
        if (i + 1 == n) *total = inc;
    }
};

// grid (n or #large rows, ncsr): one workgroup per (txn, CSR); CSRs above UNION_CAP entries are queued for k_union_big
static __global__ __launch_bounds__(UB) void k_union_lds(LdsUnionArgs a) {
    if (a.rows && blockIdx.x >= *a.rows_total) return;
    const size_t t = a.rows ? (size_t)a.rows[blockIdx.x] : (size_t)blockIdx.x;
    const int c = a.csr_base + (int)blockIdx.y * a.csr_step;
    if (t >= a.n) return;
    if (a.only_large && !(a.meta[t] & META_LARGE)) return;
    __shared__ uint32_t buf[UNION_CAP];
    __shared__ uint32_t wsum[UB / WAVE];
    const uint32_t nk = a.key_off[c][t + 1] - a.key_off[c][t];
    if (nk == 0) {
        if (threadIdx.x == 0) a.tcnt[c][t] = 0;
        return;
    }
    const uint32_t mb = a.k2t_off[c][t];
    const uint32_t ne = a.k2t_off[c][t + 1] - mb - nk;
    if (ne > (uint32_t)UNION_CAP) {
        if (threadIdx.x == 0) {
            const uint32_t k = atomicAdd(a.ovf_count, 1u);
            if (k < a.ovf_cap) a.ovf[k] = make_uint2((uint32_t)t, (uint32_t)c);
            else atomicOr(&a.prm->err, ERR_CAP);
            a.tcnt[c][t] = 0;
        }
        return;
    }
    union_body<UB>(buf, wsum, a.k2t[c] + mb + nk, ne, a.txns[c] + a.ent_off[c][t], &a.tcnt[c][t]);
}

// grid (#large rows, classes per view): one workgroup per (large txn, class) unions every view's CSR of the class
// (csr = 2v + class), sharing the sort between identical views
static __global__ __launch_bounds__(UB) void k_union_lds_views(LdsUnionArgs a, int nvw) {
    if (blockIdx.x >= *a.rows_total) return;
    const uint32_t t = a.rows[blockIdx.x];
    __shared__ uint32_t buf[UNION_CAP];
    __shared__ uint32_t wsum[UB / WAVE];
    int cs[MAXV];
    for (int v = 0; v < nvw; ++v) cs[v] = 2 * v + (int)blockIdx.y;
    union_views<UB>(a, t, cs, nvw, buf, wsum, (uint32_t)UNION_CAP, [&](int, int c) {
        const uint32_t k = atomicAdd(a.ovf_count, 1u);
        if (k < a.ovf_cap) a.ovf[k] = make_uint2(t, (uint32_t)c);
        else atomicOr(&a.prm->err, ERR_CAP);
        a.tcnt[c][t] = 0;
    });
}

// RangeDeps of every txn (C4: ~10^7 (txn, view) lists of a few hundred entries): one 64-thread workgroup with a
// 2 KiB LDS buffer per (txn, CSR).  The 256-thread kernel's 32 KiB buffer held a CU to 5 workgroups, i.e. 5
// unions in flight per CU, each a chain of ~40 barrier-separated bitonic stages; single-wave workgroups fit 32
// per CU and their barriers are cheap.  Lists above UNION_SMALL go to the medium queue (k_union_lds_list).
constexpr int UNION_SMALL = 512, US_T = 64;
// One workgroup per txn unions every view's RangeDeps CSR (union_views: identical views share one sort); the views
// whose lists exceed UNION_SMALL are queued together as (txn, view mask) for k_union_lds_list.
static __global__ __launch_bounds__(US_T) void k_union_lds_small(LdsUnionArgs a) {
    const size_t t = blockIdx.x;
    if (t >= a.n) return;
    __shared__ uint32_t buf[UNION_SMALL];
    __shared__ uint32_t wsum[1];
    int cs[MAXV];
    for (int v = 0; v < a.ncsr; ++v) cs[v] = a.csr_base + v;
    uint32_t big = 0;
    union_views<US_T>(a, (uint32_t)t, cs, a.ncsr, buf, wsum, (uint32_t)UNION_SMALL, [&](int v, int) { big |= 1u << v; });
    if (threadIdx.x == 0 && big) a.med[atomicAdd(a.med_count, 1u)] = make_uint2((uint32_t)t, big);
}
// the medium queue: grid-stride over the device-side count, one 256-thread workgroup per (txn, view mask) (LDS up
// to UNION_CAP; above it the overflow queue as in k_union_lds)
static __global__ __launch_bounds__(UB) void k_union_lds_list(LdsUnionArgs a) {
    __shared__ uint32_t buf[UNION_CAP];
    __shared__ uint32_t wsum[UB / WAVE];
    const uint32_t count = *a.med_count;
    for (uint32_t it = blockIdx.x; it < count; it += gridDim.x) {
        const uint32_t t = a.med[it].x, mask = a.med[it].y;
        int cs[MAXV], nvw = 0;
        for (int v = 0; v < a.ncsr; ++v) if (mask >> v & 1u) cs[nvw++] = a.csr_base + v;
        union_views<UB>(a, t, cs, nvw, buf, wsum, (uint32_t)UNION_CAP, [&](int, int c) {
            const uint32_t k = atomicAdd(a.ovf_count, 1u);
            if (k < a.ovf_cap) a.ovf[k] = make_uint2(t, (uint32_t)c);
            else atomicOr(&a.prm->err, ERR_CAP);
            a.tcnt[c][t] = 0;
        });
    }
}

// overflow pass, one 1024-thread workgroup per queued (txn, CSR): LDS up to UNION_CAP_BIG entries, beyond
// that a bitonic sort in this item's slice of global memory
static __global__ __launch_bounds__(UB_BIG) void k_union_big(LdsUnionArgs a, uint32_t count) {
    const uint32_t it = blockIdx.x;
    if (it >= count) return;
    __shared__ uint32_t buf[UNION_CAP_BIG];
    __shared__ uint32_t wsum[UB_BIG / WAVE];
    const uint32_t t = a.items[it].x, c = a.items[it].y;
    const uint32_t nk = a.key_off[c][t + 1] - a.key_off[c][t];
    const uint32_t mb = a.k2t_off[c][t];
    const uint32_t ne = a.k2t_off[c][t + 1] - mb - nk;
    uint32_t* space = ne > (uint32_t)UNION_CAP_BIG ? a.gbuf + a.gbuf_off[it] : buf;
    union_body<UB_BIG>(space, wsum, a.k2t[c] + mb + nk, ne, a.txns[c] + a.ent_off[c][t], &a.tcnt[c][t]);
}

}  // namespace ad
