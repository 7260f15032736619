// shard_kernels.h — key-range sharding across GPUs (BASELINE C5).
//
// One CommandStore per GPU owns a contiguous key range (ShardDistributor.EvenSplit,
// local/ShardDistributor.java:32-80).  Each store resolves, for every txn touching its range, the part of
// the PreAccept deps that its keys produce (its local batch: the txns, with their keys sliced to the range,
// in global TxnId order; row -> global arrival rank through `gid`).  PreAccept.reduce across stores
// (messages/PreAccept.java:141-156: Deps.with of the per-store PartialDeps) becomes:
//   export    each store packs, per destination store, the per-(view, class) CSR rows of the local txns
//             homed there (home = the store of the txn's first key) that have any deps, TxnIds rewritten
//             to global ranks: one blob per destination, concatenated in destination order;
//   exchange  all-to-all of the blobs (RCCL grouped send/recv over xGMI, or host staging over gloo):
//             every store receives only the fragments of its own home txns;
//   merge     each store's home txns merge the fragments of every store, per view (k_merge with
//             per-source row indirection), then Deps.merge across the replica views.
// Execution levels: each store runs the chain fixpoint over its own keys on a replicated global level
// array; stores exchange it with an all-reduce(max) until no store raises a level.
#pragma once
#include "level_kernels.h"

namespace ad {

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

// ---- export: rows with deps, partitioned by destination store ----------------------------------------
constexpr int MAX_STORES = 8;
// CSRs per exported row: per view key + direct (2R), and with range txns RangeDeps per view (R more)
constexpr int NVX_MAX = 3 * MAXV;
struct DestOp {                       // per row: rank among the kept rows of its destination
    struct S { uint32_t c[MAX_STORES]; };
    const uint8_t* dest;
    const uint32_t* tcnt[NVX_MAX];    // per (view, class): per-row unique TxnId counts
    int nvc;
    uint32_t* rank;                   // [n] rank within destination, or ~0u (no deps: not exported)
    uint32_t* totals;                 // [MAX_STORES]
    size_t n;
    __device__ S identity() const { S s; for (int k = 0; k < MAX_STORES; ++k) s.c[k] = 0; return s; }
    __device__ bool keep(size_t r) const {
        uint32_t any = 0;
        for (int vc = 0; vc < nvc; ++vc) any |= tcnt[vc][r];
        return any != 0;
    }
    __device__ S load(size_t r) const {
        S s = identity();
        if (keep(r)) s.c[dest[r]] = 1;
        return s;
    }
    __device__ S combine(const S& a, const S& b) const { S s; for (int k = 0; k < MAX_STORES; ++k) s.c[k] = a.c[k] + b.c[k]; return s; }
    __device__ void store(size_t r, const S& ex, const S& inc, const S& el) const {
        const uint32_t d = dest[r];
        rank[r] = el.c[d] ? ex.c[d] : ~0u;
        if (r + 1 == n) for (int k = 0; k < MAX_STORES; ++k) totals[k] = inc.c[k];
    }
};
// list[base[d] + rank] = r  (base = exclusive prefix of the destination totals, computed in-kernel)
static __global__ __launch_bounds__(256) void k_export_list(size_t n, const uint8_t* __restrict__ dest, const uint32_t* __restrict__ rank,
                                                     const uint32_t* __restrict__ totals, uint32_t* __restrict__ list) {
    const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n || rank[r] == ~0u) return;
    uint32_t base = 0;
    for (uint32_t d = 0; d < dest[r]; ++d) base += totals[d];
    list[base + rank[r]] = (uint32_t)r;
}
// global (over the export list) offsets of keys / keysToTxnIds / TxnIds per (view, class)
template <int NVC>
struct ExportOffsetsOp {
    struct S { uint32_t k[NVC], m[NVC], t[NVC]; };
    static constexpr int nvc = NVC;
    const uint32_t* list;
    const uint32_t* key_off[NVC];     // source CSRs (capacity form)
    const uint32_t* k2t_off[NVC];
    const uint32_t* tcnt[NVC];
    uint32_t* ok[NVC];                // [K+1] each
    uint32_t* om[NVC];
    uint32_t* ot[NVC];
    size_t n;                         // K
    __device__ S identity() const { S s; for (int c = 0; c < NVC; ++c) { s.k[c] = s.m[c] = s.t[c] = 0; } return s; }
    __device__ S load(size_t j) const {
        S s = identity();
        const uint32_t r = list[j];
#pragma unroll
        for (int c = 0; c < NVC; ++c) {
            s.k[c] = key_off[c][r + 1] - key_off[c][r];
            s.m[c] = k2t_off[c][r + 1] - k2t_off[c][r];
            s.t[c] = tcnt[c][r];
        }
        return s;
    }
    __device__ S combine(const S& a, const S& b) const {
        S s;
#pragma unroll
        for (int c = 0; c < NVC; ++c) { s.k[c] = a.k[c] + b.k[c]; s.m[c] = a.m[c] + b.m[c]; s.t[c] = a.t[c] + b.t[c]; }
        return s;
    }
    __device__ void store(size_t j, const S& ex, const S& inc, const S&) const {
#pragma unroll
        for (int c = 0; c < NVC; ++c) {
            ok[c][j] = ex.k[c]; om[c][j] = ex.m[c]; ot[c][j] = ex.t[c];
            if (j + 1 == n) { ok[c][n] = inc.k[c]; om[c][n] = inc.m[c]; ot[c][n] = inc.t[c]; }
        }
    }
};
// the global offsets at every destination boundary: out[(d * nvc + c) * 3 + {0,1,2}], d = 0..world
struct ExportOffs { uint32_t* ok[NVX_MAX]; uint32_t* om[NVX_MAX]; uint32_t* ot[NVX_MAX]; };
static __global__ void k_export_bounds(int world, int nvc, const uint32_t* __restrict__ totals, ExportOffs o, uint32_t* __restrict__ out) {
    const int i = threadIdx.x;
    if (i >= (world + 1) * nvc) return;
    const int d = i / nvc, c = i % nvc;
    uint32_t base = 0;
    for (int x = 0; x < d; ++x) base += totals[x];
    out[i * 3 + 0] = o.ok[c][base];
    out[i * 3 + 1] = o.om[c][base];
    out[i * 3 + 2] = o.ot[c][base];
}
// Destination blob sections (byte offsets from the send buffer base), per destination:
// [0] gid, then per vc: [1+7c] key_off [2+7c] k2t_off [3+7c] ent_off [4+7c] tcnt [5+7c] keys [6+7c] k2t [7+7c] txns
// (vc < 2R: key / direct class of view vc/2, keys 8 B; vc >= 2R: RangeDeps of view vc-2R, ranges 16 B)
constexpr int SEC_PER_DEST = 1 + 7 * NVX_MAX;
struct ExportFillArgs {
    size_t K;
    int nvc;
    const uint32_t* list;
    const uint8_t* dest;
    const uint32_t* totals;           // rows per destination
    const uint32_t* gid;
    const uint32_t* bnd;              // k_export_bounds output
    const uint64_t* sec;              // [MAX_STORES * SEC_PER_DEST]
    uint8_t* send;
    const uint32_t* key_off[NVX_MAX];
    const uint64_t* keys[NVX_MAX];
    const uint32_t* k2t_off[NVX_MAX];
    const int32_t* k2t[NVX_MAX];
    const uint32_t* ent_off[NVX_MAX];
    const uint32_t* tcnt[NVX_MAX];
    const uint32_t* txns[NVX_MAX];
    int kw[NVX_MAX];                  // u64 words per key (2: a range)
    ExportOffs o;
};
// one thread per exported row: its gid, rebased offsets, and its keys / keysToTxnIds / TxnIds (as global
// ranks) copied into its destination's blob; the destination's last row writes the closing offsets
static __global__ __launch_bounds__(256) void k_export_fill(ExportFillArgs a) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.K) return;
    const uint32_t r = a.list[j];
    const uint32_t d = a.dest[r];
    uint32_t base = 0;
    for (uint32_t x = 0; x < d; ++x) base += a.totals[x];
    const uint32_t i = (uint32_t)j - base;
    const bool last = i + 1 == a.totals[d];
    const uint64_t* sec = a.sec + (size_t)d * SEC_PER_DEST;
    reinterpret_cast<uint32_t*>(a.send + sec[0])[i] = a.gid[r];
    for (int c = 0; c < a.nvc; ++c) {
        const uint32_t* b0 = a.bnd + ((size_t)d * a.nvc + c) * 3;         // this destination's first row
        const uint32_t kb = a.o.ok[c][j] - b0[0], mb = a.o.om[c][j] - b0[1], tb = a.o.ot[c][j] - b0[2];
        uint32_t* key_off = reinterpret_cast<uint32_t*>(a.send + sec[1 + 7 * c]);
        uint32_t* k2t_off = reinterpret_cast<uint32_t*>(a.send + sec[2 + 7 * c]);
        uint32_t* ent_off = reinterpret_cast<uint32_t*>(a.send + sec[3 + 7 * c]);
        uint32_t* tcnt = reinterpret_cast<uint32_t*>(a.send + sec[4 + 7 * c]);
        uint64_t* keys = reinterpret_cast<uint64_t*>(a.send + sec[5 + 7 * c]);
        int32_t* k2t = reinterpret_cast<int32_t*>(a.send + sec[6 + 7 * c]);
        uint32_t* txns = reinterpret_cast<uint32_t*>(a.send + sec[7 + 7 * c]);
        const uint32_t sk = a.key_off[c][r], nk = a.key_off[c][r + 1] - sk;
        const uint32_t sm = a.k2t_off[c][r], nm = a.k2t_off[c][r + 1] - sm;
        const uint32_t st = a.ent_off[c][r], nt = a.tcnt[c][r];
        key_off[i] = kb; k2t_off[i] = mb; ent_off[i] = tb; tcnt[i] = nt;
        if (last) { key_off[i + 1] = kb + nk; k2t_off[i + 1] = mb + nm; ent_off[i + 1] = tb + nt; }
        const uint32_t w = (uint32_t)a.kw[c];
        for (uint32_t x = 0; x < nk * w; ++x) keys[(size_t)kb * w + x] = a.keys[c][(size_t)sk * w + x];
        for (uint32_t x = 0; x < nm; ++x) k2t[mb + x] = a.k2t[c][sm + x];
        for (uint32_t x = 0; x < nt; ++x) txns[tb + x] = a.gid[a.txns[c][st + x]];
    }
}

// home txns: global ids
static __global__ __launch_bounds__(256) void k_home_gid(size_t H, const uint32_t* __restrict__ rows, const uint32_t* __restrict__ gid,
                                                  uint32_t* __restrict__ hg) {
    const size_t h = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (h < H) hg[h] = gid[rows[h]];
}

// row of each home txn in source s (binary search over the source's ascending global ids; -1 = absent)
static __global__ __launch_bounds__(256) void k_source_rows(size_t H, const uint32_t* __restrict__ hg, const uint32_t* __restrict__ sgid,
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
static __global__ __launch_bounds__(256) void k_levels_gather(size_t n, const uint32_t* __restrict__ gid, const uint32_t* __restrict__ G,
                                                       uint32_t* __restrict__ L) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) L[i] = G[gid[i]];
}
static __global__ __launch_bounds__(256) void k_levels_scatter(size_t n, const uint32_t* __restrict__ gid, uint32_t* __restrict__ G,
                                                        const uint32_t* __restrict__ L, uint32_t* __restrict__ changed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool up = false;
    if (i < n) {
        const uint32_t g = gid[i], l = L[i];
        if (l > G[g]) { G[g] = l; up = true; }
    }
    wave_set_flag(up, changed);
}

// Delta level exchange: a store's chains hold only the txns that touch its keys, so the only
// levels another store needs are those of the txns both hold.  Per round, every level this store raised is
// folded into its own G and, for a txn other stores hold too (holders[r]: bitmask of the stores holding row
// r), appended as (gid << 32 | level) to each of those stores' regions of `out` (region d starts at base[d]
// and holds at most the rows shared with d: no overflow).  Order inside a region is free: the receiver folds
// with max.  *sent: some pair was appended.
static __global__ __launch_bounds__(256) void k_level_deltas(size_t n, const uint32_t* __restrict__ gid, const uint8_t* __restrict__ holders,
                                                      uint32_t others, uint32_t* __restrict__ G, const uint32_t* __restrict__ L,
                                                      const uint32_t* __restrict__ base, uint32_t* __restrict__ cnt,
                                                      uint64_t* __restrict__ out, uint32_t* __restrict__ sent) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t m = 0;
    uint64_t pair = 0;
    if (i < n) {
        const uint32_t g = gid[i], l = L[i];
        if (l > G[g]) {
            G[g] = l;
            m = holders[i] & others;
            pair = ((uint64_t)g << 32) | l;
        }
    }
    const int lane = (int)__lane_id();
#pragma unroll
    for (int d = 0; d < MAX_STORES; ++d) {
        const bool want = (m >> d) & 1u;
        const uint64_t b = __ballot(want);
        if (!b) continue;
        const int leader = __ffsll((unsigned long long)b) - 1;
        uint32_t at = 0;
        if (lane == leader) at = atomicAdd(cnt + d, (uint32_t)__popcll(b));
        at = __builtin_amdgcn_readlane(at, leader);
        if (want) out[base[d] + at + (uint32_t)__popcll(b & ((1ull << lane) - 1ull))] = pair;
    }
    wave_set_flag(m != 0, sent);
}

// Received (gid << 32 | level) pairs folded into G (several stores may raise one txn: max).
static __global__ __launch_bounds__(256) void k_level_apply(size_t m, const uint64_t* __restrict__ pairs, uint32_t* __restrict__ G) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) {
        const uint64_t p = pairs[i];
        atomicMax(G + (uint32_t)(p >> 32), (uint32_t)p);
    }
}

}  // namespace ad
