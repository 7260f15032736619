// deps_kernels.h — PreAccept conflict-dependency kernels for key footprints (gfx950).
//
// Data flow for one batch (all device resident, P = (txn,key) pairs, sorted order = (key, TxnId rank)):
//   k_minmax / k_pack   batch statistics, TxnId/executeAt -> packed ts64, per-txn meta byte, pair owner,
//                       footprint validation (keys ascending per txn, ranges sorted and disjoint)
//   radix sort          (key - key_min, pair) pairs, stable => each key segment is CFK.byId order
//   k_gather_entries    sorted entry SoA: txn rank, meta, executeAt+1 (one 16-byte record per entry)
//   ElideOp scan        per entry: segment start, distinct-key index, prefix max executeAt of committed
//                       writes (maxCommittedWriteBefore), prefix max executeAt of elidable entries, last
//                       "always emitted" entry — CommandsForKey.mapReduceActive's state
//                       (CommandsForKey.java:925-983) as one segmented scan
//   walk<count>         per query item (txn i, key segment, insert position) and replica view: the
//                       dependencies mapReduceActive emits (CommandsForKey.java:945-965), counted per (pair,
//                       class) in one byte, the first WALK_INL ids kept inline
//   OffsetsOp scan      per-txn CSR offsets of every class
//   k_txn_finish        small txns (key txns with <= 4 keys whose pairs kept every id inline): KeyDeps layout,
//                       per-key lists and TxnId union in registers; the rest (deferred) get their layout here
//                       and their lists from walk<fill> + k_txn_union (<= KMAX keys)
//   large txns (range-domain txns querying every CFK key inside their ranges, and key txns with more
//   than KMAX keys) go through "virtual items" (vitem_kernels in engine.hip) and union_kernels.h.
#pragma once
#include "scan.h"

namespace ad {

constexpr int MAXV = 8;       // replica views
constexpr int KMAX = 16;      // keys per key-domain txn handled by the per-txn register kernels
constexpr int NVC_MAX = MAXV * 2;
constexpr uint32_t META_LARGE = 0x80u;   // meta bit 7: txn takes the large (virtual item) path
constexpr uint32_t PREC_EXEQ = 0x100u;   // PairRec.meta bit 8: executeAt == TxnId (the PreAccept bound is executeAt + 1)
// The count walk keeps the first WALK_INL dependencies of every (pair, class) inline, so a txn whose pairs stay
// within it gets its KeyDeps lists and TxnId union written by the offsets scan's store: no fill walk and no union
// pass over it.  Counts are one byte per (pair, class), NCB bytes per pair (one dword for NC <= 4).
constexpr int WALK_INL = 4;
constexpr int ncb_of(int nc) { return (nc + 3) & ~3; }
__device__ inline uint32_t pair_count(const uint8_t* __restrict__ cnt8, const uint32_t* __restrict__ cntx, int ncb, int nc,
                                      size_t x, int c) {
    const uint32_t b = cnt8[x * ncb + c];
    return b == 255u ? cntx[x * nc + c] : b;
}
// all NC counts of pair x (dword loads: NCB is a multiple of 4)
template <int NC>
__device__ inline void pair_counts(const uint8_t* __restrict__ cnt8, const uint32_t* __restrict__ cntx, size_t x, uint32_t* v) {
    constexpr int NCB = ncb_of(NC);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(cnt8 + x * NCB);
    uint32_t d[NCB / 4];
#pragma unroll
    for (int q = 0; q < NCB / 4; ++q) d[q] = w[q];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint32_t b = (d[c >> 2] >> (8 * (c & 3))) & 0xFFu;
        v[c] = b == 255u ? cntx[x * NC + c] : b;
    }
}

struct alignas(16) PairRec {  // per (txn, key) pair, in pair order: what the sorted entries gather
    uint64_t ex1;             // the txn's executeAt + 1 (packed)
    uint32_t txn;             // batch rank
    uint32_t meta;            // meta byte
};

struct Params {                // device-side batch statistics (filled by k_minmax / k_pack)
    unsigned long long msb_min, msb_max, hlc_min, hlc_max;
    unsigned long long key_min, key_max;
    unsigned long long rs_min, re_max, rw_max;   // range starts min, ends max, max width (end - start)
    unsigned int node_min_b, node_max_b;         // node + 2^31
    unsigned int max_keys, err;                  // err bits below
    unsigned int n_large, n_keys_u;              // large txns; distinct keys (after sort)
    unsigned long long n_vitems;                 // virtual items
    unsigned int n_special;                      // key-domain txns that are not Read/Write (sync points,
                                                 // ephemeral reads, local-only): unmanaged execution
    unsigned int range_kinds;                    // bit k: the batch holds a range-domain txn of kind k
    unsigned int n_multi;                        // key segments with more than one entry (k_seg_fuse batches)
};
enum : unsigned { ERR_UNSORTED = 1, ERR_KEYS = 2, ERR_DUPKEY = 4, ERR_KEYORDER = 8, ERR_RANGEORDER = 16,
                  ERR_RANGEBITS = 32, ERR_CAP = 64, ERR_EXECBELOW = 128 };

__device__ inline unsigned long long wmin64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { unsigned long long u = __shfl_xor(v, o); v = u < v ? u : v; }
    return v;
}
__device__ inline unsigned long long wmax64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { unsigned long long u = __shfl_xor(v, o); v = u > v ? u : v; }
    return v;
}

// Batch statistics: per-thread accumulation, wave shuffles, one LDS combine per block, one atomic per
// block and field (per-wave atomics on one address serialise: the first version spent 0.44 ms here).
static __global__ __launch_bounds__(256) void k_minmax(size_t n, const uint64_t* __restrict__ tm, const uint64_t* __restrict__ tl,
                                                const int32_t* __restrict__ tn, const uint64_t* __restrict__ em,
                                                const uint64_t* __restrict__ el, const int32_t* __restrict__ en,
                                                const uint32_t* __restrict__ key_off, const uint64_t* __restrict__ keys,
                                                size_t P, const uint64_t* __restrict__ rs, const uint64_t* __restrict__ re,
                                                size_t Q, unsigned long long* __restrict__ partial) {
    constexpr int NF = 15, NSUM = 12, NOR = 14;
    // fields: 0 msb_min 1 msb_max 2 hlc_min 3 hlc_max 4 node_min 5 node_max 6 key_min 7 key_max 8 max_keys
    //         9 rs_min 10 re_max 11 rw_max ; *_min are stored complemented so every field is a max
    //         12 large txns, 13 special key-domain txns (sums, fields NSUM .. NOR-1)
    //         14 kinds of the range-domain txns (a bit mask: OR, fields >= NOR)
    unsigned long long f[NF] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const size_t stride = (size_t)gridDim.x * blockDim.x;
#pragma unroll 2
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        unsigned long long a = tm[i], b = em[i], ha = tl[i] >> 16, hb = el[i] >> 16;
        unsigned long long na = (unsigned)tn[i] ^ 0x80000000u, nb = (unsigned)en[i] ^ 0x80000000u;
        f[0] = max(f[0], ~min(a, b)); f[1] = max(f[1], max(a, b));
        f[2] = max(f[2], ~min(ha, hb)); f[3] = max(f[3], max(ha, hb));
        f[4] = max(f[4], ~min(na, nb)); f[5] = max(f[5], max(na, nb));
        const unsigned kc = key_off[i + 1] - key_off[i];
        f[8] = max(f[8], (unsigned long long)kc);
        f[12] += ((tl[i] & 1) == AD_DOMAIN_RANGE || kc > (unsigned)KMAX) ? 1ull : 0ull;
        const unsigned kind = (unsigned)((tl[i] >> 1) & 7);
        f[13] += ((tl[i] & 1) == AD_DOMAIN_KEY && kind != AD_KIND_READ && kind != AD_KIND_WRITE) ? 1ull : 0ull;
        f[14] |= (tl[i] & 1) == AD_DOMAIN_RANGE ? 1ull << kind : 0ull;
    }
    // keys as 16-byte pairs (the buffer is a device allocation: 16-byte aligned), four pairs in flight per thread
    const size_t P2 = P >> 1;
    const ulonglong2* __restrict__ kp = reinterpret_cast<const ulonglong2*>(keys);
#pragma unroll 4
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < P2; i += stride) {
        const ulonglong2 k = kp[i];
        f[6] = max(f[6], ~min(k.x, k.y)); f[7] = max(f[7], max(k.x, k.y));
    }
    if ((P & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long k = keys[P - 1];
        f[6] = max(f[6], ~k); f[7] = max(f[7], k);
    }
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < Q; i += stride) {
        unsigned long long s = rs[i], e = re[i];
        f[9] = max(f[9], ~s); f[10] = max(f[10], e); f[11] = max(f[11], e > s ? e - s : 0ull);
    }
    __shared__ unsigned long long red[4][NF];
    const int w = threadIdx.x / WAVE;
#pragma unroll
    for (int k = 0; k < NSUM; ++k) {
        unsigned long long v = wmax64(f[k]);
        if (__lane_id() == 0) red[w][k] = v;
    }
#pragma unroll
    for (int k = NSUM; k < NF; ++k) {
        unsigned long long v = f[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) { const unsigned long long u = __shfl_xor(v, o); v = k >= NOR ? (v | u) : v + u; }
        if (__lane_id() == 0) red[w][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < NF) {
        const int k = threadIdx.x;
        unsigned long long v = k >= NOR ? (red[0][k] | red[1][k] | red[2][k] | red[3][k])
                             : k >= NSUM ? red[0][k] + red[1][k] + red[2][k] + red[3][k]
                                         : max(max(red[0][k], red[1][k]), max(red[2][k], red[3][k]));
        partial[(size_t)blockIdx.x * NF + k] = v;
    }
}

// second level of k_minmax: one block folds the per-block partials into Params (no contended atomics)
// pub_flag != null: also publishes the Params to the host-mapped words (pub_prm) and releases seq into *pub_flag, as
// k_publish would in a launch of its own (engine.hip publish_totals)
constexpr int MM_FINAL_T = 256;   // the fold is latency-bound: 1024 threads measured 16.0 us, 256 threads 10.6 us over 1024 partials
static __global__ __launch_bounds__(MM_FINAL_T) void k_minmax_final(int nblk, const unsigned long long* __restrict__ partial, Params* out,
                                                       uint32_t* pub_flag = nullptr, uint32_t* pub_prm = nullptr, uint32_t seq = 0) {
    constexpr int NF = 15, NSUM = 12, NOR = 14, NW = MM_FINAL_T / WAVE;
    __shared__ unsigned long long red[NW][NF];
    unsigned long long f[NF] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = threadIdx.x; b < nblk; b += blockDim.x)
        for (int k = 0; k < NF; ++k) {
            const unsigned long long v = partial[(size_t)b * NF + k];
            f[k] = k >= NOR ? (f[k] | v) : k >= NSUM ? f[k] + v : max(f[k], v);
        }
    const int w = threadIdx.x / WAVE;
    for (int k = 0; k < NF; ++k) {
        unsigned long long v = f[k];
        if (k >= NOR) {
            for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
        } else if (k >= NSUM) {
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        } else {
            v = wmax64(v);
        }
        if (__lane_id() == 0) red[w][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < NF) {
        const int k = threadIdx.x;
        unsigned long long v = red[0][k];
        for (int x = 1; x < NW; ++x) v = k >= NOR ? (v | red[x][k]) : k >= NSUM ? v + red[x][k] : max(v, red[x][k]);
        // the only writer of these fields (no separate initialisation launch)
        switch (k) {
            case 0: out->msb_min = ~v; break;
            case 1: out->msb_max = v; break;
            case 2: out->hlc_min = ~v; break;
            case 3: out->hlc_max = v; break;
            case 4: out->node_min_b = (unsigned)~v; break;
            case 5: out->node_max_b = (unsigned)v; break;
            case 6: out->key_min = ~v; break;
            case 7: out->key_max = v; break;
            case 8: out->max_keys = (unsigned)v; break;
            case 9: out->rs_min = ~v; break;
            case 10: out->re_max = v; break;
            case 11: out->rw_max = v; break;
            case 12: out->n_large = (unsigned)v; break;
            case 13: out->n_special = (unsigned)v; break;
            case 14: out->range_kinds = (unsigned)v; break;
        }
    }
    if (threadIdx.x == 0) { out->err = 0; out->n_keys_u = 0; out->n_vitems = 0; out->n_multi = 0; }
    if (pub_flag) {
        __syncthreads();
        const uint32_t* pw = reinterpret_cast<const uint32_t*>(out);
        for (int x = threadIdx.x; x < (int)(sizeof(Params) / 4); x += blockDim.x) pub_prm[x] = pw[x];
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(pub_flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Packs timestamps, builds per-txn meta, the sort input and validates footprints.  A wave owns 64 consecutive txns:
// one lane per txn for the per-txn arrays, then the wave's pairs one lane per pair (the owning txn found by a 6-step
// shuffle search over the lanes' key offsets), so the per-pair stores (record, sort key / value, the deps stage's
// count words) are coalesced runs.  One thread writing its own txn's 4 pairs left each store instruction a 64-byte
// stride across the wave: 2.2x the written bytes at the memory side and ~70 % of the wave cycles issue-stalled.
// Device-side plan (PackPlan.dprm != null): the packing parameters, the key base and the count words per pair from
// the Params k_minmax_final wrote, as stage_prepare derives them on the host -- so k_pack is enqueued right behind the
// reduce and the host reads the Params while it runs (the host's wait no longer sits between the two kernels).
struct PackPlan {
    const Params* dprm;                        // null: pk / key_min / ncw as given
    int nv_small, nv_large;                    // views when the batch has no / some large txns (the union view)
    int has_keys;
    uint32_t* clr[4];                          // small counters the deps stage needs zeroed (block 0 clears them:
    int clr_words[4];                          // no fill launch between the sort and k_seg_fuse)
    uint2* succ;                               // per pair: the pull pass's predecessor words, zeroed (k_seg_fuse builds
                                               // the chains in ad_run_pipeline: LevelInputs.chains_prebuilt)
};
__device__ inline int dbits_of(uint64_t x) { return x == 0 ? 0 : 64 - __clzll((long long)x); }
static __global__ __launch_bounds__(256) void k_pack(size_t n, TsPack pk, uint64_t key_min,
                                              const uint64_t* __restrict__ tm, const uint64_t* __restrict__ tl,
                                              const int32_t* __restrict__ tn, const uint64_t* __restrict__ em,
                                              const uint64_t* __restrict__ el, const int32_t* __restrict__ en,
                                              const uint8_t* __restrict__ status, const uint32_t* __restrict__ key_off,
                                              const uint64_t* __restrict__ keys, const uint32_t* __restrict__ range_off,
                                              const uint64_t* __restrict__ rs, const uint64_t* __restrict__ re,
                                              uint64_t* __restrict__ tx_ts, uint64_t* __restrict__ ex1,
                                              uint8_t* __restrict__ meta, PairRec* __restrict__ prec,
                                              uint32_t* __restrict__ skey, uint32_t* __restrict__ sval, Params* prm,
                                              uint32_t* __restrict__ cnt_words, int ncw, uint8_t* __restrict__ dfr,
                                              PackPlan plan = PackPlan{}) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = __lane_id();
    if (blockIdx.x == 0)
        for (int c = 0; c < 4; ++c)
            for (int x = threadIdx.x; x < plan.clr_words[c]; x += blockDim.x) plan.clr[c][x] = 0u;
    if (plan.dprm) {
        const Params& p = *plan.dprm;
        const int MB = dbits_of(p.msb_max - p.msb_min), HB = dbits_of(p.hlc_max - p.hlc_min);
        const int NB = dbits_of((uint64_t)(p.node_max_b - p.node_min_b));
        pk.msb_min = p.msb_min;
        pk.hlc_min = p.hlc_min;
        pk.node_min = (int64_t)(int32_t)(p.node_min_b ^ 0x80000000u);
        pk.sh_flags = (uint32_t)NB;
        pk.sh_hlc = (uint32_t)(NB + 4);
        pk.sh_msb = (uint32_t)(NB + 4 + HB);
        pk.total_bits = (uint32_t)(NB + 4 + HB + MB);   // > 63: the host refuses the batch after its read
        key_min = plan.has_keys ? p.key_min : 0ull;
        const int nv = p.n_large == 0 ? plan.nv_small : plan.nv_large;
        ncw = ncb_of(p.n_special > 0 ? 2 * nv : nv) / 4;
    }
    const size_t t0 = i - (size_t)lane;                 // the wave's first txn
    if (t0 >= n) return;                                // whole wave past the batch (waves stay converged below)
    const bool live = i < n;
    unsigned err = 0;
    uint64_t x1 = 0;
    uint32_t mi = 0, kb = 0xFFFFFFFFu;
    if (live) {
        dfr[i] = 0;
        const uint64_t lsb = tl[i];
        const uint64_t t = ts_pack(pk, tm[i], lsb, tn[i]);
        tx_ts[i] = t;
        const uint64_t e1 = ts_pack(pk, em[i], el[i], en[i]) + 1;
        ex1[i] = e1;
        kb = key_off[i];
        const uint32_t ke = key_off[i + 1];
        const uint32_t rb = range_off ? range_off[i] : 0u, rend = range_off ? range_off[i + 1] : 0u;
        const uint32_t domain = (uint32_t)(lsb & 1);
        if (domain == AD_DOMAIN_RANGE && ke != kb) err |= ERR_KEYORDER;        // a range txn's footprint is its ranges
        if (domain == AD_DOMAIN_KEY && rend != rb) err |= ERR_RANGEORDER;
        const bool large = domain == AD_DOMAIN_RANGE || (ke - kb) > (uint32_t)KMAX;
        const uint8_t m8 = (uint8_t)(((lsb >> 1) & 7) | ((lsb & 1) << 3) | ((uint32_t)(status[i] & 7) << 4) | (large ? META_LARGE : 0u));
        meta[i] = m8;
        mi = (uint32_t)m8 | (e1 - 1 == t ? PREC_EXEQ : 0u);
        x1 = e1;
        if (i > 0 && ts_pack(pk, tm[i - 1], tl[i - 1], tn[i - 1]) >= t) err |= ERR_UNSORTED;
        uint64_t pe = 0;
        for (uint32_t q = rb; q < rend; ++q) {                             // Ranges: sorted, disjoint, start < end
            const uint64_t s = rs[q], e = re[q];
            if (s >= e || (q > rb && s < pe)) err |= ERR_RANGEORDER;
            pe = e;
        }
    }
    // the wave's pairs [P0, P1)
    const size_t tl_last = (n - t0 < (size_t)WAVE) ? n - 1 : t0 + WAVE - 1;
    const uint32_t P0 = __shfl(kb, 0);
    const uint32_t P1 = key_off[tl_last + 1];
    for (uint32_t base = P0; base < P1; base += WAVE) {
        const uint32_t p = base + (uint32_t)lane;
        // owner: the last lane whose first pair is <= p (lanes past the batch hold kb = ~0)
        int j = 0;
#pragma unroll
        for (int step = WAVE / 2; step > 0; step >>= 1) {
            const uint32_t c = __shfl(kb, j + step);
            if (c <= p) j += step;
        }
        const uint32_t jkb = __shfl(kb, j);
        const uint64_t jx1 = __shfl(x1, j);
        const uint32_t jmi = __shfl(mi, j);
        if (p < P1) {
            const uint64_t k = keys[p];
            if (p > jkb && k <= keys[p - 1]) err |= ERR_KEYORDER;           // Keys: sorted unique
            prec[p] = PairRec{jx1, (uint32_t)(t0 + (size_t)j), jmi};
            skey[p] = (uint32_t)(k - key_min);
            sval[p] = p;
            for (int w = 0; w < ncw; ++w) cnt_words[(size_t)p * ncw + w] = 0u;     // the deps stage's count bytes
            if (plan.succ) plan.succ[p] = make_uint2(0u, 0u);
        }
    }
    if (err) atomicOr(&prm->err, err);
}

// Sorted entry SoA: one random 16-byte record read per entry (the pair's txn, meta and executeAt were
// packed per pair by k_pack in pair order, i.e. coalesced), instead of three dependent random loads.
// SKIP (batches of small key txns, 32-bit key spread, PreAccept bound): an entry alone in its key segment has no
// entry before or after it, so no query of this batch reads it (the walks and the pull levels only visit
// multi-entry segments); it gets a placeholder without the random read (C2: ~80% of entries), and
// k_complete_singletons fills it in before anything that reads every entry (complete_entries).
__device__ inline bool lone_entry(size_t s, size_t P, const uint32_t* __restrict__ skey) {
    const uint32_t k = skey[s];
    return (s == 0 || skey[s - 1] != k) && (s + 1 == P || skey[s + 1] != k);
}
template <bool SKIP>
static __global__ __launch_bounds__(256) void k_gather_entries(size_t P, const uint32_t* __restrict__ sval,
                                                        const PairRec* __restrict__ prec, const uint32_t* __restrict__ skey,
                                                        uint32_t* __restrict__ e_txn, uint8_t* __restrict__ e_meta,
                                                        uint64_t* __restrict__ e_exec1) {
    size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P) return;
    if (SKIP && lone_entry(s, P, skey)) {
        e_txn[s] = 0; e_meta[s] = 0; e_exec1[s] = 0;
        return;
    }
    const PairRec r = prec[sval[s]];
    e_txn[s] = r.txn;
    e_meta[s] = (uint8_t)r.meta;
    e_exec1[s] = r.ex1;
}
// The lone entries k_gather_entries<true> skipped: their record, and the elision scan's state at them (a segment
// head with nothing before it: ElideOp::load of the entry itself; seg_start is already theirs).
static __global__ __launch_bounds__(256) void k_complete_singletons(size_t P, const uint32_t* __restrict__ sval,
                                                             const PairRec* __restrict__ prec, const uint32_t* __restrict__ skey,
                                                             uint32_t* __restrict__ e_txn, uint8_t* __restrict__ e_meta,
                                                             uint64_t* __restrict__ e_exec1, int32_t* __restrict__ ud_prev,
                                                             uint64_t* __restrict__ pm_w, uint64_t* __restrict__ pm_c) {
    size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P || !lone_entry(s, P, skey)) return;
    const PairRec r = prec[sval[s]];
    e_txn[s] = r.txn;
    e_meta[s] = (uint8_t)r.meta;
    e_exec1[s] = r.ex1;
    const uint32_t cat = category(r.meta);
    ud_prev[s] = cat == CAT_ALWAYS ? (int32_t)s : -1;
    pm_c[s] = cat == CAT_ELIDABLE ? r.ex1 : 0ull;
    pm_w[s] = (cat == CAT_ELIDABLE && meta_kind(r.meta) == AD_KIND_WRITE) ? r.ex1 : 0ull;
}

// Segmented prefix state of CommandsForKey.mapReduceActive over the (key, TxnId)-sorted entries.
// Wide key spreads: the sort key of pass `shift` (0: low 32 bits, 32: high bits) of the pairs in their current
// order (val = pair index), for an LSD sort of the full 64-bit (key - key_min) by 32-bit halves.
static __global__ __launch_bounds__(256) void k_pair_key_half(size_t P, const uint64_t* __restrict__ keys, const uint32_t* __restrict__ val,
                                                       uint64_t key_min, int shift, uint32_t* __restrict__ out) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < P) out[x] = (uint32_t)((keys[val[x]] - key_min) >> shift);
}

struct ElideOp {
    struct S {
        uint32_t head;
        int32_t ss;          // segment start (max of head indices)
        int32_t ud;          // last CAT_ALWAYS entry index
        uint32_t hc;         // heads so far (distinct-key index + 1)
        uint64_t pw;         // prefix max executeAt+1 of committed writes (0 = none)
        uint64_t pc;         // prefix max executeAt+1 of elidable entries (0 = none)
    };
    const uint32_t* skey;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    int32_t* seg_start;
    int32_t* ud_prev;
    uint64_t* pm_w;
    uint64_t* pm_c;
    uint32_t* nh;            // non-head entries (entries with an earlier entry of their key), in order
    uint64_t* ukey;          // [U] distinct keys (raw u64)
    uint32_t* useg;          // [U+1] segment starts
    uint64_t key_min;
    size_t n;
    Params* prm;
    const uint64_t* keys64;  // wide key spreads (> 32 bits): raw keys through sval (skey holds only low bits)
    const uint32_t* sval;

    __device__ uint64_t key_at(size_t i) const { return keys64 ? keys64[sval[i]] : (uint64_t)skey[i] + key_min; }
    __device__ S load(size_t i) const {
        S s;
        if (keys64) s.head = (i == 0 || keys64[sval[i]] != keys64[sval[i - 1]]) ? 1u : 0u;
        else s.head = (i == 0 || skey[i] != skey[i - 1]) ? 1u : 0u;
        s.ss = s.head ? (int32_t)i : -1;
        uint32_t m = e_meta[i];
        uint32_t cat = category(m);
        s.ud = cat == CAT_ALWAYS ? (int32_t)i : -1;
        s.hc = s.head;
        uint64_t e = e_exec1[i];
        s.pc = cat == CAT_ELIDABLE ? e : 0;
        s.pw = (cat == CAT_ELIDABLE && meta_kind(m) == AD_KIND_WRITE) ? e : 0;
        return s;
    }
    __device__ S identity() const { return S{0u, -1, -1, 0u, 0ull, 0ull}; }
    __device__ S combine(const S& a, const S& b) const {
        S r;
        r.head = a.head | b.head;
        r.ss = max(a.ss, b.ss);
        r.ud = max(a.ud, b.ud);
        r.hc = a.hc + b.hc;
        r.pw = b.head ? b.pw : (a.pw > b.pw ? a.pw : b.pw);
        r.pc = b.head ? b.pc : (a.pc > b.pc ? a.pc : b.pc);
        return r;
    }
    __device__ void store(size_t i, const S&, const S& inc, const S& el) const {
        seg_start[i] = inc.ss;
        ud_prev[i] = inc.ud;
        pm_w[i] = inc.pw;
        pm_c[i] = inc.pc;
        const uint32_t u = inc.hc - 1;
        if (el.head) {
            ukey[u] = key_at(i);
            useg[u] = (uint32_t)i;
        } else {
            nh[i - inc.hc] = (uint32_t)i;     // (i + 1 - hc) non-heads so far, this one included
        }
        if (i + 1 == n) {
            useg[inc.hc] = (uint32_t)n;
            prm->n_keys_u = inc.hc;
        }
    }
};

struct WalkArgs {
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const int32_t* seg_start;
    const int32_t* ud_prev;
    const uint64_t* pm_w;
    const uint64_t* pm_c;
    const uint64_t* tx_ts;
    const uint8_t* meta;      // per txn
    const uint32_t* gid;      // sharded batches: local row -> global arrival rank (nullable = identity)
    size_t P;
    const uint32_t* nh;       // non-head entries (ElideOp), P - n_keys_u of them: the only ones with deps
    const Params* prm;
    uint32_t window;
    uint32_t thresh;
    uint64_t seed;
    int union_last;           // view NV - 1 is the union of the others (deps.hip stage_deps: the merged Deps)
    const uint32_t* sval;     // sorted position -> pair index p
    uint8_t* cnt8;            // real pairs, AoS by pair: [p * NCB + k] count of class k, 255 = see cntx
    uint32_t* cntx;           // [p * NC + k] exact count where cnt8 saturated (>= 255)
    uint32_t* inl;            // [(p * NC + k) * WALK_INL + q]: the first WALK_INL ids the walk emits (descending)
    uint8_t* dfr;             // [txn] 1: the txn has more than 4 keys with entries (fill walk + k_txn_union; the
                              // offsets scan writes it)
    const uint32_t* key_off;  // per txn (a txn with more than 4 keys: every pair with entries goes to the fill walk)
    uint32_t* posof;          // [pair] sorted position, written for the pairs that overflowed their inline ids
    uint32_t* items_out;      // count walk: the sorted positions the fill walk visits, *items_count of them
    uint32_t* items_count;
    const uint32_t* items;    // fill walk: that list, nitems long
    size_t nitems;
    const uint32_t* dst;      // real pairs, AoS by pair: absolute k2t slot of the last entry (fill)
    int32_t* k2t[NVC_MAX];    // per-vc keysToTxnIds (fill)
    // virtual items (large txns): item x queries key segment u = vi_u[x] ([useg[u], ...)) before position vi_pos[x]
    size_t V;
    const uint32_t* vi_txn;
    const uint32_t* vi_pos;
    const uint32_t* vi_u;     // distinct-key index of the item
    const uint32_t* useg;     // [U+1] segment starts
    uint32_t* vcnt;           // [x * nvc + vc]
    const uint32_t* vdst;     // [x * nvc + vc] (the same buffer: k_large_layout rewrites counts into slots)
    // executeAt-bound queries (Accept / GetDeps; nullable = PreAccept, bound TxnId): per txn the arrival position
    // of its bound, q = #{j : TxnId_j < executeAt_i}; ex1 = executeAt + 1
    const uint32_t* qpos;
    const uint32_t* gqpos;    // sharded stores: the bound's GLOBAL arrival position per local row (window placement;
                              // qpos stays the local position for the segment search); nullable = qpos
    const uint64_t* ex1;
    int bound_max;            // GetEphemeralReadDeps: bound Timestamp.MAX (qpos = n; no executeAt bound)
    __device__ uint64_t bound1(uint32_t i) const { return bound_max ? ~0ull : ex1[i]; }
};

// Next emitted "elidable" (committed Read/Write) entry at or before q, or seg0-1.
__device__ inline int next_elidable(const WalkArgs& a, int q, int seg0, uint64_t M1, uint32_t qk) {
    for (; q >= seg0; --q) {
        if (M1 != 0 && a.pm_c[q] < M1) return seg0 - 1;      // no earlier entry reaches maxCommittedWriteBefore
        uint32_t m = a.e_meta[q];
        if (category(m) == CAT_ELIDABLE && witnesses(qk, meta_kind(m)) && (M1 == 0 || a.e_exec1[q] >= M1)) return q;
    }
    return seg0 - 1;
}

// CommandsForKey.mapReduceActive(startedBefore) for one key segment, over the entries [seg0, s) (all with
// TxnId below the bound), every replica view at once.  emit(v, direct, j) in descending order.  gq: the arrival
// position the query is answered at (PreAccept: i's own; Accept: its executeAt's), which places the in-flight
// window; b1 = bound + 1.  The txn's own entry is never emitted (PreAccept.calculatePartialDeps :258-260).
template <int NV, class Emit>
__device__ inline void walk_query(const WalkArgs& a, uint32_t i, uint32_t gq, uint64_t b1, uint32_t qk, int s, int seg0,
                                  Emit&& emit) {
    // window and drop decisions use global arrival ranks (shard-invariant); emitted ids stay local rows
    const uint32_t gi = a.gid ? a.gid[i] : i;
    const uint32_t lo = a.window == 0 ? gq : (gq > a.window ? gq - a.window : 0u);
    // 1. in-flight window: txns j in [q - W, q) are PREACCEPTED from i's viewpoint; replica view v has
    //    not witnessed j with probability drop_p (ad_drop_hash).
    int q = s - 1;
    for (; q >= seg0; --q) {
        const uint32_t j = a.e_txn[q];
        const uint32_t gj = a.gid ? a.gid[j] : j;
        if (gj < lo) break;
        if (j == i) continue;
        const uint32_t mj = a.e_meta[q];
        if (!manages(mj) || !witnesses(qk, meta_kind(mj))) continue;
        const bool direct = !manages_execution(mj);
        if (a.union_last) {
            // the union view: j is in the merged Deps iff some reply kept it
            bool kept = false;
#pragma unroll
            for (int v = 0; v + 1 < NV; ++v)
                if (!(a.thresh && drop_hash(a.seed, (uint32_t)v, gi, gj) < a.thresh)) { emit(v, direct, j); kept = true; }
            if (kept) emit(NV - 1, direct, j);
        } else {
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (!(a.thresh && drop_hash(a.seed, (uint32_t)v, gi, gj) < a.thresh)) emit(v, direct, j);
        }
    }
    // 2. the committed prefix [seg0, p]: mapReduceActive with transitive-dependency elision.
    const int p = q;
    if (p < seg0) return;
    uint64_t M1 = a.pm_w[p];
    bool exact = M1 >= b1;   // a bumped executeAt beyond the bound: exact maxCommittedWriteBefore
    if (!exact && a.qpos && M1 != 0) {
        // bound-position queries (Accept, GetEphemeralReadDeps) keep the txn's own entry inside [seg0, p]: it
        // must not set maxCommittedWriteBefore (the oracle leaves the querying txn out, oracle.cpp map_reduce_active)
        int l = seg0, r = p + 1;
        while (l < r) { const int m = (l + r) >> 1; if (a.e_txn[m] < i) l = m + 1; else r = m; }
        exact = l <= p && a.e_txn[l] == i && a.e_exec1[l] == M1;
    }
    if (exact) {
        M1 = 0;
        for (int x = p; x >= seg0; --x) {
            uint32_t m = a.e_meta[x];
            uint64_t e = a.e_exec1[x];
            if (category(m) == CAT_ELIDABLE && meta_kind(m) == AD_KIND_WRITE && e < b1 && e > M1 && a.e_txn[x] != i) M1 = e;
        }
    }
    int qe = next_elidable(a, p, seg0, M1, qk);
    int qa = a.ud_prev[p];
    if (qa < seg0) qa = -1;
    while (qe >= seg0 || qa >= 0) {
        if (qa > qe) {
            const uint32_t mj = a.e_meta[qa];
            const uint32_t j = a.e_txn[qa];
            if (witnesses(qk, meta_kind(mj)) && j != i) {
                const bool direct = !manages_execution(mj);
#pragma unroll
                for (int v = 0; v < NV; ++v) emit(v, direct, j);
            }
            const int nx = qa - 1;
            qa = nx >= seg0 ? a.ud_prev[nx] : -1;
            if (qa < seg0) qa = -1;
        } else {
            const uint32_t j = a.e_txn[qe];
            if (j != i) {
                const bool direct = !manages_execution(a.e_meta[qe]);
#pragma unroll
                for (int v = 0; v < NV; ++v) emit(v, direct, j);
            }
            qe = next_elidable(a, qe - 1, seg0, M1, qk);
        }
    }
}

// Real pairs of small key txns, one thread per sorted entry (neighbouring threads walk one segment).
// One thread per non-head entry (a key segment's first entry has nothing before it: no deps, and its
// counts stay at the zeros the caller cleared).  The list is dense, so the active threads fill whole
// waves (a grid over all P entries left ~5 of 6 lanes idle in every wave of this latency-bound walk).
// Executeat-bound queries (a.qpos): one thread per entry (a segment head can have deps that arrived after it),
// walking from the first entry of the segment whose TxnId reaches the bound.
// DIRECT: the batch holds key-domain sync points (n_special > 0), so entries split into keyDeps and
// directKeyDeps (class vc = 2 view + direct); otherwise every emitted entry is a keyDeps entry (vc = view) and
// the per-pair count / slot words are R instead of 2R.
template <int NV, bool DIRECT>
__device__ inline int walk_class(int v, bool direct) { return DIRECT ? 2 * v + (direct ? 1 : 0) : v; }

// The query of the key entry at sorted position s (txn i, meta mi): CommandsForKey.mapReduceActive over its key's
// entries below the bound, every replica view (walk_query).  Small key-domain query txns only (large ones are
// virtual items; the other kinds query nothing).
// b1 (PreAccept queries): TxnId + 1 when the caller has it at hand (k_seg_fuse: from the gathered record when
// executeAt == TxnId), else 0 and it is read from tx_ts
template <int NV, class Emit>
__device__ inline void walk_entry(const WalkArgs& a, size_t s, uint32_t i, uint32_t mi, Emit&& emit, uint64_t b1 = 0) {
    const uint32_t qk = meta_kind(mi);
    if (!(meta_domain(mi) == AD_DOMAIN_KEY && qk <= AD_KIND_EXCLUSIVE_SYNC_POINT && !(mi & META_LARGE))) return;
    const int seg0 = a.seg_start[s];
    if (a.qpos) {
        // first entry of the segment at or past the bound: ranks ascend inside a segment
        const uint32_t qi = a.qpos[i];
        size_t lo = s + 1, hi = a.P;
        while (lo < hi) {
            const size_t m = (lo + hi) >> 1;
            if (a.seg_start[m] == seg0 && a.e_txn[m] < qi) lo = m + 1; else hi = m;
        }
        walk_query<NV>(a, i, a.gqpos ? a.gqpos[i] : qi, a.bound1(i), qk, (int)lo, seg0, emit);
    } else {
        const uint32_t gi = a.gid ? a.gid[i] : i;
        walk_query<NV>(a, i, gi, b1 ? b1 : a.tx_ts[i] + 1, qk, (int)s, seg0, emit);
    }
}

template <int NV, bool FILL, bool DIRECT>
__device__ inline bool walk_pair_entry(const WalkArgs& a, size_t s, uint64_t b1 = 0);

template <int NV, bool FILL, bool DIRECT>
static __global__ __launch_bounds__(256) void k_deps_walk(WalkArgs a) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= (FILL ? a.nitems : (a.qpos ? a.P : a.P - a.prm->n_keys_u))) return;
    const size_t s = FILL ? (size_t)a.items[x] : (a.qpos ? x : (size_t)a.nh[x]);
    walk_pair_entry<NV, FILL, DIRECT>(a, s);
}

// One sorted entry's query (count: counts, inline ids, overflow position, fill items; fill: the entries into their
// slots).  The entry state arrays of `a` may point into LDS (k_seg_fuse: shifted so that [s] lands in the tile).
// Count mode returns whether a later kernel re-walks this entry from the global entry state (an overflowed list,
// k_txn_finish_ovf; a wide txn's pair, the fill walk).
template <int NV, bool FILL, bool DIRECT>
__device__ inline bool walk_pair_entry(const WalkArgs& a, size_t s, uint64_t b1) {
    constexpr int NC = DIRECT ? 2 * NV : NV;
    const uint32_t i = a.e_txn[s];
    const uint32_t mi = a.e_meta[s];
    // the pair's counts / slots live AoS by pair index (the per-txn kernels read them contiguously)
    const size_t p = a.sval[s];
    const size_t pb = p * NC;
    uint32_t c[NC];            // count mode: counts; fill mode: next write slot (descending)
#pragma unroll
    for (int k = 0; k < NC; ++k) c[k] = FILL ? a.dst[pb + k] : 0u;
    uint32_t* inl = a.inl + pb * WALK_INL;
    auto emit = [&](int v, bool direct, uint32_t j) {
        const int k = walk_class<NV, DIRECT>(v, direct);
        if (FILL) {
            a.k2t[k][c[k]--] = (int32_t)j;
        } else {
            if (c[k] < (uint32_t)WALK_INL) inl[k * WALK_INL + c[k]] = j;
            c[k]++;
        }
    };
    walk_entry<NV>(a, s, i, mi, emit, b1);
    if (!FILL) {
        constexpr int NCB = ncb_of(NC);
        uint32_t w[NCB / 4];
#pragma unroll
        for (int q = 0; q < NCB / 4; ++q) w[q] = 0;
        bool over = false;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            w[k >> 2] |= (c[k] < 255u ? c[k] : 255u) << (8 * (k & 3));
            if (c[k] >= 255u) a.cntx[pb + k] = c[k];
            over |= c[k] > (uint32_t)WALK_INL;
        }
        uint32_t* d = reinterpret_cast<uint32_t*>(a.cnt8 + p * NCB);
#pragma unroll
        for (int q = 0; q < NCB / 4; ++q) d[q] = w[q];
        bool any = false;
#pragma unroll
        for (int k = 0; k < NC; ++k) any |= c[k] > 0;
        const bool wide = a.key_off[i + 1] - a.key_off[i] > 4u;
        // a pair of a <= 4-key txn that overflowed its inline ids: k_txn_finish re-walks it from here
        if (over && !wide) a.posof[p] = (uint32_t)s;
        // the fill walk's items: every pair with entries of a txn with more than 4 keys (deferred to walk<fill>
        // + k_txn_union; k_txn_finish lays them out)
        wave_append(wide && any, (uint32_t)s, a.items_out, a.items_count);
        return (over && !wide) || (wide && any);
    }
    return false;
}

// Virtual items (large txns), one thread per item; counts/slots AoS [x * NC + vc].
template <int NV, bool FILL, bool DIRECT>
static __global__ __launch_bounds__(256) void k_vitem_walk(WalkArgs a) {
    constexpr int NC = DIRECT ? 2 * NV : NV;
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= a.V) return;
    const uint32_t i = a.vi_txn[x];
    const uint32_t mi = a.meta[i];
    const uint32_t qk = meta_kind(mi);
    uint32_t c[NC];
#pragma unroll
    for (int vc = 0; vc < NC; ++vc)
        c[vc] = FILL ? a.vdst[x * NC + vc] : 0u;
    auto emit = [&](int v, bool direct, uint32_t j) {
        const int vc = walk_class<NV, DIRECT>(v, direct);
        if (FILL) a.k2t[vc][c[vc]--] = (int32_t)j;
        else c[vc]++;
    };
    if (qk <= AD_KIND_EXCLUSIVE_SYNC_POINT) {
        const uint32_t gq = a.qpos ? (a.gqpos ? a.gqpos[i] : a.qpos[i]) : (a.gid ? a.gid[i] : i);
        walk_query<NV>(a, i, gq, a.qpos ? a.bound1(i) : a.tx_ts[i] + 1, qk, (int)a.vi_pos[x], (int)a.useg[a.vi_u[x]], emit);
    }
    if (!FILL) {
#pragma unroll
        for (int vc = 0; vc < NC; ++vc) a.vcnt[x * NC + vc] = c[vc];
    }
}

struct TxnArgs {
    size_t n, P;
    int nvc;
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint8_t* meta;
    const uint8_t* cnt8;          // AoS by pair [p * ncb + vc] (pair_count)
    const uint32_t* cntx;
    uint32_t* nk;                 // [vc * n + t]
    uint32_t* ne;                 // [vc * n + t]
    const uint32_t* out_key_off[NVC_MAX];
    const uint32_t* out_k2t_off[NVC_MAX];
    const uint32_t* out_ent_off[NVC_MAX];
    uint64_t* out_keys[NVC_MAX];
    int32_t* out_k2t[NVC_MAX];
    uint32_t* out_txns[NVC_MAX];
    uint32_t* out_tcnt[NVC_MAX];
    const uint32_t* inl;          // the count walk's inline ids [(p * nvc + vc) * WALK_INL + q], descending
    const uint8_t* dfr;           // [txn] deferred to the fill walk + k_txn_union
    size_t nrows;                 // k_txn_finish: txns
    const uint32_t* spec_bad;     // k_txn_finish launched before the sizes reached the host: exit when set
    WalkArgs w;                   // k_txn_finish re-walks the pairs that overflowed their inline ids (w.posof)
    uint32_t* dst;                // AoS by pair [p * nvc + vc]
    Params* prm;
    // large txns (virtual items, in (txn, key) order): items [voff[t], voff[t+1])
    const uint32_t* voff;
    const uint32_t* vcnt;         // [x * nvc + vc]
    uint32_t* vdst;               // [x * nvc + vc] (aliases vcnt: each slot is read, then rewritten, once)
    const uint32_t* vi_u;         // item -> distinct-key index (its key = ukey[u])
    const uint64_t* ukey;
    unsigned long long* dbg;      // AD_OVF_TIMERS=1: k_txn_finish_ovf's rows, clocks (sum, max), walked pairs, emitted
    uint8_t* ovf_cm;              // ... and their overflowed classes
    uint32_t* ovf_rows;           // k_txn_finish -> k_txn_finish_ovf: txns with a class whose lists overflowed
    uint32_t* ovf_count;          //   their inline ids (zeroed before the finish)
};

// Large txns (virtual items: range-domain txns, >16-key txns), one wave per txn: per-CSR key and entry
// totals (k_large_sums, read by OffsetsOp's load) and the layout (k_large_layout, after the CSRs are
// allocated): the items with deps become the txn's keys in item order, the k2t header gets the running
// entry end, and each item its last k2t slot (the fill walk emits descending).  A C4 range txn has
// ~3*10^3 items: one lane per item instead of one thread walking them all.
__device__ inline uint32_t wave_incl_sum(uint32_t v) {
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_up(v, d);
        if ((int)__lane_id() >= d) v += y;
    }
    return v;
}
template <int NVC>
static __global__ __launch_bounds__(256) void k_large_sums(TxnArgs a) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n || !(a.meta[t] & META_LARGE)) return;
    const uint32_t b = a.voff[t], e = a.voff[t + 1];
    uint32_t k[NVC], en[NVC];
#pragma unroll
    for (int c = 0; c < NVC; ++c) { k[c] = 0; en[c] = 0; }
    for (uint32_t x = b + __lane_id(); x < e; x += WAVE) {
#pragma unroll
        for (int c = 0; c < NVC; ++c) {
            const uint32_t v = a.vcnt[(size_t)x * NVC + c];
            k[c] += v > 0 ? 1u : 0u;
            en[c] += v;
        }
    }
#pragma unroll
    for (int c = 0; c < NVC; ++c) {
        const uint32_t ks = wave_incl_sum(k[c]), es = wave_incl_sum(en[c]);
        if (__lane_id() == WAVE - 1) { a.nk[(size_t)c * a.n + t] = ks; a.ne[(size_t)c * a.n + t] = es; }
    }
}
template <int NVC>
static __global__ __launch_bounds__(256) void k_large_layout(TxnArgs a) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n || !(a.meta[t] & META_LARGE)) return;
    const uint32_t b = a.voff[t], e = a.voff[t + 1];
    const uint64_t below = (1ull << __lane_id()) - 1ull;
    // every class in one pass over the items: the item's key is loaded once, its NVC counts are adjacent
    uint32_t kb[NVC], mb[NVC], run[NVC], kk[NVC];
#pragma unroll
    for (int c = 0; c < NVC; ++c) {
        kb[c] = a.out_key_off[c][t];
        run[c] = a.out_key_off[c][t + 1] - kb[c];            // the header: entries start after the keys
        mb[c] = a.out_k2t_off[c][t];
        kk[c] = 0;
    }
    for (uint32_t x0 = b; x0 < e; x0 += WAVE) {
        const uint32_t x = x0 + __lane_id();
        uint32_t v[NVC];
        bool any = false;
#pragma unroll
        for (int c = 0; c < NVC; ++c) { v[c] = x < e ? a.vcnt[(size_t)x * NVC + c] : 0u; any |= v[c] > 0; }
        const uint64_t key = any ? a.ukey[a.vi_u[x]] : 0ull;
#pragma unroll
        for (int c = 0; c < NVC; ++c) {
            const uint32_t incl = wave_incl_sum(v[c]);
            const uint64_t nz = __ballot(v[c] > 0);
            if (v[c] > 0) {
                const uint32_t r = kk[c] + (uint32_t)__popcll(nz & below);
                const uint32_t before = run[c] + incl - v[c];
                a.out_keys[c][kb[c] + r] = key;
                a.vdst[(size_t)x * NVC + c] = mb[c] + before + v[c] - 1;
                a.out_k2t[c][mb[c] + r] = (int32_t)(before + v[c]);
            }
            run[c] += __builtin_amdgcn_readlane(incl, WAVE - 1);
            kk[c] += (uint32_t)__popcll(nz);
        }
    }
}

// Per-txn (keys, entries) of every (view, class) key CSR, counted from the pairs' AoS counts inside the
// scan's load, and the exclusive offsets key_off / ent_off / k2t_off of all of them in one scan (replaces
// 2NV separate count reductions and 3 * 2NV scans).
// Deps.merge sends txns whose replies total more than this many TxnIds + keys to k_merge_heavy
// (merge_kernels.h: MERGE_HEAVY); the offsets scan flags batches that may have any, so batches without
// (C2) skip the heavy launches.  Entries bound TxnIds from above, so the hint is conservative.
constexpr uint32_t MERGE_HEAVY_HINT = 256;
template <int NVC>
struct OffsetsOp {
    // k / e: keys and entries per class; d: deferred txns and o: overflowed (txn, class) rows, whose exclusive prefixes
    // are the txns' slots in the dtx / ovf_rows lists (an atomic append per wave was ~5x10^4 same-address atomics on
    // C3, whose hot keys overflow ~10^5 rows: 0.55 ms of the scan); ob: the element's overflowed classes (its own
    // value only: combine's sum of it is not used)
    struct S { uint32_t k[NVC], e[NVC], d, o, ob; };
    size_t n;
    const uint8_t* meta;
    const uint32_t* key_off;
    const uint8_t* cnt8;          // AoS by pair, one byte per class (pair_counts)
    const uint32_t* cntx;
    uint32_t* o_key_off[NVC];
    uint32_t* o_ent_off[NVC];
    uint32_t* o_k2t_off[NVC];
    uint8_t* dfr;                 // [txn] deferred to the fill walk + union (set by the walk, or here)
    uint32_t* dtx;                // the deferred txns (k_txn_union's list), *dtx_count of them
    uint32_t* dtx_count;
    const uint32_t* lsum_k;       // [c * n + t] large txns' per-CSR key / entry totals (k_large_sums)
    const uint32_t* lsum_e;
    uint32_t* heavy;              // set when some txn's CSRs total more than MERGE_HEAVY keys + entries
    uint32_t* ovf_rows;           // txns k_txn_finish_ovf lays out (a pair's list overflowed the walk's inline ids) and
    uint8_t* ovf_cm;              //   their overflowed classes: listed here so that kernel can run beside k_txn_finish
    uint32_t* ovf_count;

    __device__ S identity() const {
        S s;
#pragma unroll
        for (int c = 0; c < NVC; ++c) { s.k[c] = 0; s.e[c] = 0; }
        s.d = s.o = s.ob = 0;
        return s;
    }
    __device__ S load(size_t t) const {
        S s = identity();
        const bool large = meta[t] & META_LARGE;
        if (large) {              // summed by k_large_sums (one wave per txn: range txns have ~10^3 items)
#pragma unroll
            for (int c = 0; c < NVC; ++c) { s.k[c] = lsum_k[(size_t)c * n + t]; s.e[c] = lsum_e[(size_t)c * n + t]; }
            return s;
        }
        const uint32_t b = key_off[t], e = key_off[t + 1];
        // a pair's NVC counts are contiguous bytes (one dword per pair for NVC <= 4)
        uint32_t ob = 0, ents = 0;
        for (uint32_t x = b; x < e; ++x) {
            uint32_t v[NVC];
            pair_counts<NVC>(cnt8, cntx, x, v);
#pragma unroll
            for (int c = 0; c < NVC; ++c) {
                s.k[c] += v[c] > 0 ? 1u : 0u; s.e[c] += v[c]; ents += v[c];
                ob |= (v[c] > (uint32_t)WALK_INL ? 1u : 0u) << c;
            }
        }
        // small txns k_txn_finish cannot finish from the inline ids: a pair overflowed them (the walk set dfr), or
        // more than 4 keys carry entries (deferred); k_txn_finish's small txns (<= 4 pairs) with a class whose list
        // overflowed the inline ids (overflowed rows)
        s.d = (dfr[t] != 0 || (ents > 0 && e - b > 4)) ? 1u : 0u;
        if (e - b <= 4) { s.ob = ob; s.o = ob ? 1u : 0u; }
        return s;
    }
    __device__ S combine(const S& x, const S& y) const {
        S r;
#pragma unroll
        for (int c = 0; c < NVC; ++c) { r.k[c] = x.k[c] + y.k[c]; r.e[c] = x.e[c] + y.e[c]; }
        r.d = x.d + y.d; r.o = x.o + y.o; r.ob = 0;
        return r;
    }
    __device__ void store(size_t t, const S& ex, const S& inc, const S& el) const {
        uint32_t w = 0, ents = 0;
#pragma unroll
        for (int c = 0; c < NVC; ++c) { w += el.k[c] + el.e[c]; ents += el.e[c]; }
        if (w > MERGE_HEAVY_HINT && *(volatile uint32_t*)heavy == 0u) *(volatile uint32_t*)heavy = 1u;
#pragma unroll
        for (int c = 0; c < NVC; ++c) {
            o_key_off[c][t] = ex.k[c];
            o_ent_off[c][t] = ex.e[c];
            o_k2t_off[c][t] = ex.k[c] + ex.e[c];
            if (t + 1 == n) {
                o_key_off[c][n] = inc.k[c];
                o_ent_off[c][n] = inc.e[c];
                o_k2t_off[c][n] = inc.k[c] + inc.e[c];
            }
        }
        // the deferred txn and the overflowed rows at their prefix slots (ascending txn order)
        if (el.d) {
            if (!dfr[t]) dfr[t] = 1;
            dtx[ex.d] = (uint32_t)t;
        }
        if (el.ob) { ovf_rows[ex.o] = (uint32_t)t; ovf_cm[ex.o] = (uint8_t)el.ob; }
        if (t + 1 == n) { *dtx_count = inc.d; *ovf_count = inc.o; }
    }
};

// Sorts 16 keys ascending in registers (bitonic network, compile-time indices only).
template <class T>
__device__ inline void sort16(T* v) {
#pragma unroll
    for (int k = 2; k <= 16; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int l = i ^ j;
                if (l > i) {
                    const T x = v[i], y = v[l];
                    const bool up = (i & k) == 0;
                    const bool sw = up ? x > y : x < y;
                    v[i] = sw ? y : x;
                    v[l] = sw ? x : y;
                }
            }
        }
    }
}

static_assert(WALK_INL == 4, "k_txn_finish's sorting network holds 4 pairs x 4 ids");

// Union of up to KMAX sorted lists living in k2t[lo[k] .. hi[k]) -> out (unique, ascending); then
// every entry is rewritten as its index in out.  Returns |out|.
template <int KM>
__device__ inline uint32_t union_lists(int32_t* __restrict__ k2t, const uint32_t* lo, const uint32_t* hi, int nl,
                                       uint32_t* __restrict__ out) {
    uint32_t cur[KM], head[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        cur[k] = k < nl ? lo[k] : 0u;
        head[k] = (k < nl && cur[k] < hi[k]) ? (uint32_t)k2t[cur[k]] : 0xFFFFFFFFu;
    }
    uint32_t u = 0;
    while (true) {
        uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < KM; ++k) mn = head[k] < mn ? head[k] : mn;
        if (mn == 0xFFFFFFFFu) break;
        out[u++] = mn;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            if (head[k] == mn) {
                ++cur[k];
                head[k] = cur[k] < hi[k] ? (uint32_t)k2t[cur[k]] : 0xFFFFFFFFu;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        if (k < nl) {
            uint32_t x = 0;
            for (uint32_t q = lo[k]; q < hi[k]; ++q) {
                uint32_t v = (uint32_t)k2t[q];
                while (out[x] < v) ++x;
                k2t[q] = (int32_t)x;
            }
        }
    }
    return u;
}

template <int KM>
__device__ inline uint32_t union_small(int32_t* __restrict__ k2t, uint32_t mb, uint32_t nk, uint32_t* __restrict__ out) {
    uint32_t lo[KM], hi[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        if (k < (int)nk) {
            lo[k] = mb + (k == 0 ? nk : (uint32_t)k2t[mb + k - 1]);
            hi[k] = mb + (uint32_t)k2t[mb + k];
        } else {
            lo[k] = hi[k] = 0;
        }
    }
    return union_lists<KM>(k2t, lo, hi, (int)nk, out);
}

// Per (small txn, class), after the CSRs are sized: the KeyDeps layout (keys in ascending order, keysToTxnIds
// header), the per-key lists and the TxnId union with every entry remapped to its index (RelationMultiMap.
// AbstractBuilder's finishKey/build, utils/RelationMultiMap.java:201-260).  Lists come from the count walk's
// inline ids (emitted descending, laid out ascending); when every list of the class fits them, the union of up to
// 4 pairs x WALK_INL (TxnId, slot) pairs is one register sorting network.  A pair whose class overflowed them is
// re-walked here (walk_entry from the position the count walk left in posof, this class only) and the class's
// lists are then unioned from memory (union_small) -- rare (C2: a few txns per batch), and inside this kernel its
// latency hides behind the other threads instead of forming a serial chain of small launches.  Txns with more
// than 4 keys (deferred: dfr) only get their layout and the fill walk's dst slots; walk<fill> + k_txn_union
// finish them.  Grid (txns, classes): the offsets, counts and keys are loaded before the ids and the first store.
// The speculative k_txn_finish's guard: some CSR total exceeds the capacity of the buffer it was launched into.
struct CapCheck {
    const uint32_t* tot[3 * NVC_MAX];
    uint32_t cap[3 * NVC_MAX];
    int m;
    uint32_t* bad;
};
// What a publish does before it copies the totals (engine.hip k_publish): the speculative finish's capacity guard
// (k_cap_check's rule) and k_seg_fuse's head count (k_seg_heads' sum into n_keys_u) — one launch instead of three
struct PubExtra {
    CapCheck cap;                 // cap.bad == null: none
    const uint32_t* hpart;        // null: none
    int nparts;
    Params* prm;
};
static __global__ __launch_bounds__(64) void k_cap_check(CapCheck a) {
    const int l = threadIdx.x;
    const bool over = l < a.m && *a.tot[l] > a.cap[l];
    const uint64_t m = __ballot(over);
    if (l == 0) *a.bad = m ? 1u : 0u;
}

// WIDE: batches of 2^28 txns or more (the 32-bit sort words hold TxnId << 4)
template <int NV, bool DIRECT, bool WIDE>
static __global__ __launch_bounds__(256) void k_txn_finish(TxnArgs a) {
    constexpr int NVC = DIRECT ? 2 * NV : NV;
    if (a.spec_bad && *a.spec_bad) return;          // speculative launch into too-small buffers: re-run after sizing
    // class-minor lanes: the NVC threads of one txn are neighbours, so their shared per-txn loads (key_off, meta,
    // counts, keys) fall on the same lines within a wave instead of being fetched once per class pass
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= a.nrows * NVC) return;
    const size_t t = x / NVC;
    const int c = (int)(x - t * NVC);
    const uint32_t kb = a.out_key_off[c][t], ke = a.out_key_off[c][t + 1];
    const uint32_t b = a.key_off[t], e = a.key_off[t + 1];
    const uint32_t mb = a.out_k2t_off[c][t], ob = a.out_ent_off[c][t];
    const uint32_t mt = a.meta[t];
    const bool defer = a.dfr[t] != 0;
    if (mt & META_LARGE) return;                    // k_large_layout
    const uint32_t nk = ke - kb;
    if (nk == 0) { if (!defer) a.out_tcnt[c][t] = 0; return; }
    constexpr int NCB = ncb_of(NVC);
    int32_t* k2t = a.out_k2t[c];
    if (e - b > 4) {                                // deferred: every pair with entries is on the fill walk's list
        uint32_t run = nk, kk = 0;
        for (uint32_t y = b; y < e; ++y) {
            const uint32_t cc = pair_count(a.cnt8, a.cntx, NCB, NVC, y, c);
            if (cc == 0) continue;
            a.out_keys[c][kb + kk] = a.keys[y];
            a.dst[(size_t)y * NVC + c] = mb + run + cc - 1;      // the fill walk emits descending from here
            run += cc;
            k2t[mb + kk] = (int32_t)run;
            ++kk;
        }
        return;
    }
    uint32_t cc[4];
    uint64_t kx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) cc[j] = b + j < e ? pair_count(a.cnt8, a.cntx, NCB, NVC, b + j, c) : 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) kx[j] = cc[j] > 0 ? a.keys[b + j] : 0ull;     // only the keys with entries
    bool ovf = false;                               // some list of this class overflowed its inline ids
#pragma unroll
    for (int j = 0; j < 4; ++j) ovf |= cc[j] > (uint32_t)WALK_INL;
    uint32_t id[4][WALK_INL];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t* src = a.inl + ((size_t)(b + j) * NVC + c) * WALK_INL;
#pragma unroll
        for (int q = 0; q < WALK_INL; ++q) id[j][q] = (uint32_t)q < cc[j] && cc[j] <= (uint32_t)WALK_INL ? src[q] : 0u;
    }
    // some list of this class overflowed its inline ids: k_txn_finish_ovf lays the class out from memory (a re-walk
    // of the overflowed pairs; the offsets scan listed the row, and that kernel runs beside this one); kept out of
    // this kernel, whose registers it would raise from 60 to 81 (8 -> 5 waves per SIMD)
    if (ovf) return;
    uint32_t run = nk, kk = 0, rb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        rb[j] = run;
        if (cc[j] == 0) continue;
        a.out_keys[c][kb + kk] = kx[j];
        run += cc[j];
        k2t[mb + kk] = (int32_t)run;
        ++kk;
    }
    uint32_t* tx = a.out_txns[c] + ob;
    if (nk == 1) {                                  // one key: its list is the union, indices 0..cc-1
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (cc[j] == 0) continue;
#pragma unroll
            for (int q = 0; q < WALK_INL; ++q) {
                if ((uint32_t)q < cc[j]) {
                    const uint32_t pos = cc[j] - 1 - (uint32_t)q;
                    tx[pos] = id[j][q];
                    k2t[mb + rb[j] + pos] = (int32_t)pos;
                }
            }
            a.out_tcnt[c][t] = cc[j];
        }
        return;
    }
    // several keys: (TxnId, k2t slot) pairs sorted in registers, equal TxnIds folded into one index.  Batches below
    // 2^28 txns sort 32-bit words (TxnId << 4 | pair * 4 + id): half the registers of (TxnId, slot) u64 pairs
    // (82 -> fewer VGPRs: more waves per SIMD for this latency-bound kernel)
    uint32_t sb[4];                                 // k2t slot of pair j's id 0 (ids run downwards from it)
#pragma unroll
    for (int j = 0; j < 4; ++j) sb[j] = mb + rb[j] + cc[j] - 1;
    if (!WIDE) {
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < WALK_INL; ++q)
                v[j * WALK_INL + q] = (uint32_t)q < cc[j] ? (id[j][q] << 4) | (uint32_t)(j * WALK_INL + q) : ~0u;
        sort16(v);
        uint32_t u = 0, prev = 0xFFFFFFFFu;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (v[r] != ~0u) {
                const uint32_t y = v[r] >> 4, jq = v[r] & 15u, j = jq >> 2;
                const uint32_t base = j == 0 ? sb[0] : j == 1 ? sb[1] : j == 2 ? sb[2] : sb[3];
                if (y != prev) { tx[u++] = y; prev = y; }
                k2t[base - (jq & 3u)] = (int32_t)(u - 1);
            }
        }
        a.out_tcnt[c][t] = u;
        return;
    }
    uint64_t v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < WALK_INL; ++q)
            v[j * WALK_INL + q] = (uint32_t)q < cc[j] ? ((uint64_t)id[j][q] << 32) | (uint64_t)(sb[j] - (uint32_t)q) : ~0ull;
    sort16(v);
    uint32_t u = 0, prev = 0xFFFFFFFFu;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        if (v[r] != ~0ull) {
            const uint32_t y = (uint32_t)(v[r] >> 32);
            if (y != prev) { tx[u++] = y; prev = y; }
            k2t[(uint32_t)v[r]] = (int32_t)(u - 1);
        }
    }
    a.out_tcnt[c][t] = u;
}
// The txns whose lists overflowed k_txn_finish's inline ids (the offsets scan listed them with their overflowed
// classes): per overflowed class the per-key lists in memory (raw TxnIds, ascending) from the inline ids and, for
// the overflowed pairs, ONE re-walk of the pair for all of its overflowed classes (walk_entry from posof; a walk per
// (txn, class) row walked C3's hot pairs ~3 times: 0.8 ms of random line traffic), then each class's union
// (union_small).  C2: a few hundred txns; C3: ~3*10^5 (its hot keys' pairs).  Grid-stride over the device-side count.
template <int NV, bool DIRECT>
static __global__ __launch_bounds__(256) void k_txn_finish_ovf(TxnArgs a) {
    constexpr int NVC = DIRECT ? 2 * NV : NV;
    constexpr int NCB = ncb_of(NVC);
    if (a.spec_bad && *a.spec_bad) return;
    const uint32_t cnt = *(const volatile uint32_t*)a.ovf_count;
    for (size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x; x < cnt; x += (size_t)gridDim.x * blockDim.x) {
        const uint64_t c0 = a.dbg ? clock64() : 0;
        uint32_t dwalk = 0, demit = 0;
        const size_t t = a.ovf_rows[x];
        const uint32_t cm = a.ovf_cm[x];                 // the overflowed classes
        const uint32_t b = a.key_off[t], e = a.key_off[t + 1];
        const uint32_t mt = a.meta[t];
        uint32_t kb[NVC], nk[NVC], mb[NVC], run[NVC], kk[NVC];
#pragma unroll
        for (int c = 0; c < NVC; ++c) {
            const bool on = (cm >> c) & 1u;
            kb[c] = on ? a.out_key_off[c][t] : 0u;
            nk[c] = on ? a.out_key_off[c][t + 1] - kb[c] : 0u;
            mb[c] = on ? a.out_k2t_off[c][t] : 0u;
            run[c] = nk[c]; kk[c] = 0;
        }
        for (uint32_t y = b; y < e; ++y) {                   // <= 4 pairs (k_txn_finish's small txns)
            uint32_t cc[NVC];
            pair_counts<NVC>(a.cnt8, a.cntx, y, cc);
            uint32_t walk = 0, slot[NVC];
#pragma unroll
            for (int c = 0; c < NVC; ++c) {
                slot[c] = 0;
                if (!((cm >> c) & 1u) || cc[c] == 0) continue;
                int32_t* k2t = a.out_k2t[c];
                a.out_keys[c][kb[c] + kk[c]] = a.keys[y];    // the key and its keysToTxnIds end (header)
                k2t[mb[c] + kk[c]] = (int32_t)(run[c] + cc[c]);
                ++kk[c];
                if (cc[c] <= (uint32_t)WALK_INL) {
                    const uint32_t* src = a.inl + ((size_t)y * NVC + c) * WALK_INL;
                    for (uint32_t q = 0; q < cc[c]; ++q) k2t[mb[c] + run[c] + cc[c] - 1 - q] = (int32_t)src[q];
                } else {
                    walk |= 1u << c;
                    slot[c] = mb[c] + run[c] + cc[c] - 1;
                }
                run[c] += cc[c];
            }
            if (walk) {
                ++dwalk;
                walk_entry<NV>(a.w, (size_t)a.w.posof[y], (uint32_t)t, mt, [&](int v, bool direct, uint32_t dj) {
                    ++demit;
                    const int c = walk_class<NV, DIRECT>(v, direct);
#pragma unroll
                    for (int k = 0; k < NVC; ++k)
                        if (k == c && ((walk >> k) & 1u)) a.out_k2t[k][slot[k]--] = (int32_t)dj;
                });
            }
        }
#pragma unroll
        for (int c = 0; c < NVC; ++c)
            if ((cm >> c) & 1u)
                a.out_tcnt[c][t] = union_small<4>(a.out_k2t[c], mb[c], nk[c], a.out_txns[c] + a.out_ent_off[c][t]);
        if (a.dbg) {
            const unsigned long long dc = (unsigned long long)(clock64() - c0);
            atomicAdd(&a.dbg[0], 1ull); atomicAdd(&a.dbg[1], dc); atomicMax(&a.dbg[2], dc);
            atomicAdd(&a.dbg[3], (unsigned long long)dwalk); atomicAdd(&a.dbg[4], (unsigned long long)demit);
        }
    }
}

struct UnionArgs {
    size_t n;
    int nvc;
    const uint8_t* meta;
    const uint32_t* key_off[NVC_MAX];
    const uint32_t* k2t_off[NVC_MAX];
    const uint32_t* ent_off[NVC_MAX];
    int32_t* k2t[NVC_MAX];
    uint32_t* txns[NVC_MAX];
    uint32_t* tcnt[NVC_MAX];
    const uint32_t* rows;         // the deferred txns (OffsetsOp's list), nrows of them
    size_t nrows;
};

// Small txns: register K-way merge of the per-key lists (large txns: k_union_lds).
template <int NVC>
static __global__ __launch_bounds__(256) void k_txn_union(UnionArgs a) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= a.nrows) return;
    const size_t t = a.rows[x];              // the other small txns were finished by k_txn_finish
    // every CSR's key range up front: the loads issue together instead of behind each CSR's stores
    uint32_t kb[NVC], ke[NVC];
#pragma unroll
    for (int vc = 0; vc < NVC; ++vc) { kb[vc] = a.key_off[vc][t]; ke[vc] = a.key_off[vc][t + 1]; }
    uint32_t mbv[NVC], obv[NVC];
#pragma unroll
    for (int vc = 0; vc < NVC; ++vc) {
        const bool any = ke[vc] != kb[vc];
        mbv[vc] = any ? a.k2t_off[vc][t] : 0u;
        obv[vc] = any ? a.ent_off[vc][t] : 0u;
    }
#pragma unroll
    for (int vc = 0; vc < NVC; ++vc) {
        const uint32_t nk = ke[vc] - kb[vc];
        if (nk == 0) { a.tcnt[vc][t] = 0; continue; }
        const uint32_t mb = mbv[vc];
        int32_t* k2t = a.k2t[vc];
        uint32_t* out = a.txns[vc] + obv[vc];
        if (nk == 1) {                 // one key: its list is already sorted and unique
            const uint32_t b = mb + 1, e = mb + (uint32_t)k2t[mb];
            for (uint32_t q = b; q < e; ++q) { out[q - b] = (uint32_t)k2t[q]; k2t[q] = (int32_t)(q - b); }
            a.tcnt[vc][t] = e - b;
            continue;
        }
        // register K-way merge sized to the key count (C2/C3 txns: 4 keys)
        if (nk <= 4) a.tcnt[vc][t] = union_small<4>(k2t, mb, nk, out);
        else if (nk <= 8) a.tcnt[vc][t] = union_small<8>(k2t, mb, nk, out);
        else a.tcnt[vc][t] = union_small<KMAX>(k2t, mb, nk, out);
    }
}

}  // namespace ad
