// deps_kernels.h — PreAccept conflict-dependency kernels (gfx950).
//
// Data flow for one batch (all device resident, P = key pairs, sorted order = (key, TxnId rank)):
//   k_minmax / k_pack   TxnId / executeAt -> packed ts64, per-txn meta byte, pair owner, sort input
//   radix sort          (key - key_min, pair) pairs, stable => each key segment is CFK.byId order
//   k_gather_entries    sorted entry SoA: txn rank, meta, executeAt+1, inverse permutation
//   ElideOp scan        per entry: segment start, prefix max executeAt of committed writes (for
//                       maxCommittedWriteBefore), prefix max executeAt of elidable entries, last
//                       "always emitted" entry — CommandsForKey.mapReduceActive's state
//                       (CommandsForKey.java:925-983) as segmented scans
//   k_deps_walk<count>  per (txn,key) pair and replica view: emitted-dependency counts
//   k_txn_counts / scans / k_txn_layout   per txn: keys that carry deps, KeyDeps header, slots
//   k_deps_walk<fill>   writes dependency ranks straight into each txn's keysToTxnIds
//   k_txn_union         per txn: sorted unique TxnIds + remap entries to indices
//                       (RelationMultiMap.AbstractBuilder.build, RelationMultiMap.java:201-260)
#pragma once
#include "scan.h"

namespace ad {

constexpr int MAXV = 8;       // replica views
constexpr int KMAX = 16;      // keys per key-domain txn handled by the per-txn kernels
constexpr int NVC_MAX = MAXV * 2;

struct Params {                // device-side batch statistics (filled by k_minmax)
    unsigned long long msb_min, msb_max, hlc_min, hlc_max;
    unsigned long long key_min, key_max;
    unsigned int node_min_b, node_max_b;   // node + 2^31
    unsigned int max_keys, err;            // err bits below
};
enum : unsigned { ERR_UNSORTED = 1, ERR_KEYS = 2, ERR_DUPKEY = 4, ERR_RANGE = 8 };

__global__ void k_params_init(Params* p) {
    p->msb_min = ~0ull; p->msb_max = 0; p->hlc_min = ~0ull; p->hlc_max = 0;
    p->key_min = ~0ull; p->key_max = 0; p->node_min_b = ~0u; p->node_max_b = 0; p->max_keys = 0; p->err = 0;
}

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

__global__ __launch_bounds__(256) void k_minmax(size_t n, const uint64_t* __restrict__ tm, const uint64_t* __restrict__ tl,
                                                const int32_t* __restrict__ tn, const uint64_t* __restrict__ em,
                                                const uint64_t* __restrict__ el, const int32_t* __restrict__ en,
                                                const uint32_t* __restrict__ key_off, const uint64_t* __restrict__ keys,
                                                size_t P, const uint32_t* __restrict__ range_off, Params* out) {
    unsigned long long mmin = ~0ull, mmax = 0, hmin = ~0ull, hmax = 0, kmin = ~0ull, kmax = 0, nmin = ~0ull, nmax = 0, kc = 0;
    unsigned rng = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        unsigned long long a = tm[i], b = em[i], ha = tl[i] >> 16, hb = el[i] >> 16;
        unsigned long long na = (unsigned)tn[i] ^ 0x80000000u, nb = (unsigned)en[i] ^ 0x80000000u;
        mmin = min(mmin, min(a, b)); mmax = max(mmax, max(a, b));
        hmin = min(hmin, min(ha, hb)); hmax = max(hmax, max(ha, hb));
        nmin = min(nmin, min(na, nb)); nmax = max(nmax, max(na, nb));
        kc = max(kc, (unsigned long long)(key_off[i + 1] - key_off[i]));
        if (range_off && range_off[i + 1] != range_off[i]) rng = 1;
    }
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += stride) {
        unsigned long long k = keys[i];
        kmin = min(kmin, k); kmax = max(kmax, k);
    }
    mmin = wmin64(mmin); mmax = wmax64(mmax); hmin = wmin64(hmin); hmax = wmax64(hmax);
    nmin = wmin64(nmin); nmax = wmax64(nmax); kmin = wmin64(kmin); kmax = wmax64(kmax); kc = wmax64(kc);
    bool anyr = __any(rng);
    if (__lane_id() == 0) {
        atomicMin(&out->msb_min, mmin); atomicMax(&out->msb_max, mmax);
        atomicMin(&out->hlc_min, hmin); atomicMax(&out->hlc_max, hmax);
        atomicMin(&out->key_min, kmin); atomicMax(&out->key_max, kmax);
        atomicMin(&out->node_min_b, (unsigned)nmin); atomicMax(&out->node_max_b, (unsigned)nmax);
        atomicMax(&out->max_keys, (unsigned)kc);
        if (anyr) atomicOr(&out->err, ERR_RANGE);
    }
}

// Packs timestamps, builds per-txn meta and the sort input.  One thread per txn.
__global__ __launch_bounds__(256) void k_pack(size_t n, TsPack pk, uint64_t key_min,
                                              const uint64_t* __restrict__ tm, const uint64_t* __restrict__ tl,
                                              const int32_t* __restrict__ tn, const uint64_t* __restrict__ em,
                                              const uint64_t* __restrict__ el, const int32_t* __restrict__ en,
                                              const uint8_t* __restrict__ status, const uint32_t* __restrict__ key_off,
                                              const uint64_t* __restrict__ keys, uint64_t* __restrict__ tx_ts,
                                              uint64_t* __restrict__ ex1, uint8_t* __restrict__ meta,
                                              uint32_t* __restrict__ pair_txn, uint32_t* __restrict__ skey,
                                              uint32_t* __restrict__ sval, Params* prm) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t lsb = tl[i];
    uint64_t t = ts_pack(pk, tm[i], lsb, tn[i]);
    tx_ts[i] = t;
    ex1[i] = ts_pack(pk, em[i], el[i], en[i]) + 1;
    meta[i] = (uint8_t)(((lsb >> 1) & 7) | ((lsb & 1) << 3) | ((uint32_t)(status[i] & 7) << 4));
    if (i > 0 && ts_pack(pk, tm[i - 1], tl[i - 1], tn[i - 1]) >= t) atomicOr(&prm->err, ERR_UNSORTED);
    for (uint32_t p = key_off[i]; p < key_off[i + 1]; ++p) {
        pair_txn[p] = (uint32_t)i;
        skey[p] = (uint32_t)(keys[p] - key_min);
        sval[p] = p;
    }
}

// Sorted entry SoA + inverse permutation.
__global__ __launch_bounds__(256) void k_gather_entries(size_t P, const uint32_t* __restrict__ sval,
                                                        const uint32_t* __restrict__ pair_txn,
                                                        const uint8_t* __restrict__ meta, const uint64_t* __restrict__ ex1,
                                                        uint32_t* __restrict__ e_txn, uint8_t* __restrict__ e_meta,
                                                        uint64_t* __restrict__ e_exec1, uint32_t* __restrict__ spos) {
    size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P) return;
    uint32_t p = sval[s];
    uint32_t t = pair_txn[p];
    e_txn[s] = t;
    e_meta[s] = meta[t];
    e_exec1[s] = ex1[t];
    spos[p] = (uint32_t)s;
}

// Segmented prefix state of CommandsForKey.mapReduceActive over the (key, TxnId)-sorted entries.
struct ElideOp {
    struct S {
        uint32_t head;
        int32_t ss;          // segment start (max of head indices)
        int32_t ud;          // last CAT_ALWAYS entry index
        uint32_t pad;
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

    __device__ S load(size_t i) const {
        S s;
        s.head = (i == 0 || skey[i] != skey[i - 1]) ? 1u : 0u;
        s.ss = s.head ? (int32_t)i : -1;
        uint32_t m = e_meta[i];
        uint32_t cat = category(m);
        s.ud = cat == CAT_ALWAYS ? (int32_t)i : -1;
        s.pad = 0;
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
        r.pad = 0;
        r.pw = b.head ? b.pw : (a.pw > b.pw ? a.pw : b.pw);
        r.pc = b.head ? b.pc : (a.pc > b.pc ? a.pc : b.pc);
        return r;
    }
    __device__ void store(size_t i, const S&, const S& inc, const S&) const {
        seg_start[i] = inc.ss;
        ud_prev[i] = inc.ud;
        pm_w[i] = inc.pw;
        pm_c[i] = inc.pc;
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
    size_t P;
    uint32_t window;
    uint32_t thresh;
    uint64_t seed;
    uint32_t* cnt;            // [vc * P + s], vc = view * 2 + class
    const uint32_t* dst;      // [vc * P + s] absolute k2t slot of the first entry (fill)
    int32_t* k2t[NVC_MAX];    // per-vc keysToTxnIds (fill)
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

template <int NV, bool FILL>
__global__ __launch_bounds__(256) void k_deps_walk(WalkArgs a) {
    const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= a.P) return;
    const uint32_t i = a.e_txn[s];
    const uint32_t mi = a.e_meta[s];
    const uint32_t qk = meta_kind(mi);
    uint32_t c0[NV], c1[NV];   // count mode: counts; fill mode: next write slot (descending)
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        if (FILL) {
            c0[v] = a.dst[(size_t)(2 * v) * a.P + s] + a.cnt[(size_t)(2 * v) * a.P + s] - 1;
            c1[v] = a.dst[(size_t)(2 * v + 1) * a.P + s] + a.cnt[(size_t)(2 * v + 1) * a.P + s] - 1;
        } else {
            c0[v] = 0; c1[v] = 0;
        }
    }
    auto emit = [&](int v, bool direct, uint32_t j) {
        if (FILL) {
            if (direct) a.k2t[2 * v + 1][c1[v]--] = (int32_t)j;
            else a.k2t[2 * v][c0[v]--] = (int32_t)j;
        } else {
            if (direct) c1[v]++; else c0[v]++;
        }
    };
    const bool query = meta_domain(mi) == AD_DOMAIN_KEY && qk <= AD_KIND_EXCLUSIVE_SYNC_POINT;
    if (query) {
        const int seg0 = a.seg_start[s];
        const uint32_t lo = a.window == 0 ? i : (i > a.window ? i - a.window : 0u);
        // 1. in-flight window: txns j in [i - W, i) are PREACCEPTED from i's viewpoint; replica
        //    view v has not witnessed j with probability drop_p (ad_drop_hash).
        int q = (int)s - 1;
        for (; q >= seg0; --q) {
            const uint32_t j = a.e_txn[q];
            if (j < lo) break;
            const uint32_t mj = a.e_meta[q];
            if (!manages(mj) || !witnesses(qk, meta_kind(mj))) continue;
            const bool direct = !manages_execution(mj);
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (!(a.thresh && drop_hash(a.seed, (uint32_t)v, i, j) < a.thresh)) emit(v, direct, j);
        }
        // 2. the committed prefix [seg0, p]: mapReduceActive with transitive-dependency elision.
        const int p = q;
        if (p >= seg0) {
            uint64_t M1 = a.pm_w[p];
            const uint64_t b1 = a.tx_ts[i] + 1;
            if (M1 >= b1) {   // a bumped executeAt beyond the bound: exact maxCommittedWriteBefore
                M1 = 0;
                for (int x = p; x >= seg0; --x) {
                    uint32_t m = a.e_meta[x];
                    uint64_t e = a.e_exec1[x];
                    if (category(m) == CAT_ELIDABLE && meta_kind(m) == AD_KIND_WRITE && e < b1 && e > M1) M1 = e;
                }
            }
            int qe = next_elidable(a, p, seg0, M1, qk);
            int qa = a.ud_prev[p];
            if (qa < seg0) qa = -1;
            while (qe >= seg0 || qa >= 0) {
                if (qa > qe) {
                    const uint32_t mj = a.e_meta[qa];
                    if (witnesses(qk, meta_kind(mj))) {
                        const uint32_t j = a.e_txn[qa];
                        const bool direct = !manages_execution(mj);
#pragma unroll
                        for (int v = 0; v < NV; ++v) emit(v, direct, j);
                    }
                    const int nx = qa - 1;
                    qa = nx >= seg0 ? a.ud_prev[nx] : -1;
                    if (qa < seg0) qa = -1;
                } else {
                    const uint32_t j = a.e_txn[qe];
                    const bool direct = !manages_execution(a.e_meta[qe]);
#pragma unroll
                    for (int v = 0; v < NV; ++v) emit(v, direct, j);
                    qe = next_elidable(a, qe - 1, seg0, M1, qk);
                }
            }
        }
    }
    if (!FILL) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            a.cnt[(size_t)(2 * v) * a.P + s] = c0[v];
            a.cnt[(size_t)(2 * v + 1) * a.P + s] = c1[v];
        }
    }
}

struct TxnArgs {
    size_t n, P;
    int nvc;
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint32_t* spos;
    const uint32_t* cnt;          // [vc * P + s]
    uint32_t* nk;                 // [vc * n + t]
    uint32_t* ne;                 // [vc * n + t]
    const uint32_t* out_key_off[NVC_MAX];
    const uint32_t* out_k2t_off[NVC_MAX];
    uint64_t* out_keys[NVC_MAX];
    int32_t* out_k2t[NVC_MAX];
    uint32_t* dst;                // [vc * P + s]
    Params* prm;
};

__global__ __launch_bounds__(256) void k_txn_counts(TxnArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t b = a.key_off[t], e = a.key_off[t + 1];
    if (e - b > KMAX) { atomicOr(&a.prm->err, ERR_KEYS); return; }
    for (int vc = 0; vc < a.nvc; ++vc) {
        uint32_t nk = 0, ne = 0;
        for (uint32_t p = b; p < e; ++p) {
            uint32_t c = a.cnt[(size_t)vc * a.P + a.spos[p]];
            nk += c > 0;
            ne += c;
        }
        a.nk[(size_t)vc * a.n + t] = nk;
        a.ne[(size_t)vc * a.n + t] = ne;
    }
}

// Per txn: keys in ascending order, KeyDeps header offsets, per-pair first-entry slot.
__global__ __launch_bounds__(256) void k_txn_layout(TxnArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t b = a.key_off[t], e = a.key_off[t + 1];
    const int K = (int)(e - b);
    if (K > KMAX || K == 0) return;
    uint64_t ks[KMAX];
    uint32_t ss[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        if (k < K) { ks[k] = a.keys[b + k]; ss[k] = a.spos[b + k]; }
    }
    // insertion sort by key (Keys are a sorted set: KeyDeps keys ascending)
#pragma unroll
    for (int k = 1; k < KMAX; ++k) {
        if (k < K) {
#pragma unroll
            for (int x = k; x > 0; --x) {
                if (ks[x - 1] > ks[x]) {
                    uint64_t tk = ks[x - 1]; ks[x - 1] = ks[x]; ks[x] = tk;
                    uint32_t ts = ss[x - 1]; ss[x - 1] = ss[x]; ss[x] = ts;
                }
            }
        }
    }
#pragma unroll
    for (int k = 1; k < KMAX; ++k)
        if (k < K && ks[k] == ks[k - 1]) atomicOr(&a.prm->err, ERR_DUPKEY);
    for (int vc = 0; vc < a.nvc; ++vc) {
        const uint32_t kb = a.out_key_off[vc][t];
        const uint32_t nk = a.out_key_off[vc][t + 1] - kb;
        if (nk == 0) continue;
        const uint32_t mb = a.out_k2t_off[vc][t];
        uint32_t run = nk, kk = 0;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (k < K) {
                const uint32_t c = a.cnt[(size_t)vc * a.P + ss[k]];
                if (c > 0) {
                    a.out_keys[vc][kb + kk] = ks[k];
                    a.dst[(size_t)vc * a.P + ss[k]] = mb + run;
                    run += c;
                    a.out_k2t[vc][mb + kk] = (int32_t)run;
                    ++kk;
                }
            }
        }
    }
}

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

struct UnionArgs {
    size_t n;
    int nvc;
    const uint32_t* key_off[NVC_MAX];
    const uint32_t* k2t_off[NVC_MAX];
    const uint32_t* ent_off[NVC_MAX];
    int32_t* k2t[NVC_MAX];
    uint32_t* txns[NVC_MAX];
    uint32_t* tcnt[NVC_MAX];
};

__global__ __launch_bounds__(256) void k_txn_union(UnionArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    for (int vc = 0; vc < a.nvc; ++vc) {
        const uint32_t nk = a.key_off[vc][t + 1] - a.key_off[vc][t];
        if (nk == 0) { a.tcnt[vc][t] = 0; continue; }
        const uint32_t mb = a.k2t_off[vc][t];
        int32_t* k2t = a.k2t[vc];
        uint32_t lo[KMAX], hi[KMAX];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
            if (k < (int)nk) {
                lo[k] = mb + (k == 0 ? nk : (uint32_t)k2t[mb + k - 1]);
                hi[k] = mb + (uint32_t)k2t[mb + k];
            }
        }
        a.tcnt[vc][t] = union_lists<KMAX>(k2t, lo, hi, (int)nk, a.txns[vc] + a.ent_off[vc][t]);
    }
}

}  // namespace ad
