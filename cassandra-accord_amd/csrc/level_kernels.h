// level_kernels.h — execution levels (Kahn wavefront index) over the resolved dependency graph.
//
// Semantics (the reference's dynamic release order, local/Commands.java:617-821 and
// local/cfk/CommandsForKey.java:1208-1330): on every key, a Write waits for all earlier-executeAt
// Reads and Writes, a Read for earlier-executeAt Writes; every edge raises executeAt, so
//   level[T] = 1 + max level over T's predecessors (0 if none)
// is a topological wavefront numbering, and `order` = txns sorted by (level, executeAt).
//
// Device algorithm (no per-level launches — C3 chains are ~10^5 deep):
//   1. chain order: the (key, TxnId)-sorted entries are re-sorted by executeAt inside each key
//      segment (in-place fix-up; nearly sorted because only slow-path txns move).
//   2. along one key chain the recurrence is a max-plus affine map on the state (y = max level so far,
//      w = max Write level so far):  Read: y' = max(y, w+1, a), w' = w;  Write: y' = w' = max(y+1, a)
//      where a = the txn's current level from its other keys.  Maps compose associatively, so one
//      segmented scan (scan.h) resolves an entire chain at once, whatever its depth.
//   3. a txn's level is the max over its keys (atomicMax); 2-3 repeat until no level changes.  The
//      iteration count is the number of chain-to-chain hops on the critical path (C2: ~5).
//   4. order: LSD radix sorts by executeAt (64-bit, two 32-bit halves) then stably by level.
#pragma once
#include "radix_sort.h"

namespace ad {

constexpr int NEG = -(1 << 29);
__device__ inline int mp_add(int x, int y) { return (x <= NEG || y <= NEG) ? NEG : x + y; }
__device__ inline int mp_max(int x, int y) { return x > y ? x : y; }

struct ChainOp {
    struct S {
        int m00, m01, m10, m11;   // max-plus matrix
        int c0, c1;               // constant
        int a;                    // element only: the txn's level estimate
        uint32_t flags;           // element only: bit0 head, bit1 participates, bit2 write
    };
    const uint32_t* c_txn;
    const uint8_t* c_meta;
    const int32_t* seg_start;     // key segments (same in (key,TxnId) and (key,executeAt) order)
    uint32_t* L;
    uint32_t* changed;

    __device__ S identity() const { return S{0, NEG, NEG, 0, NEG, NEG, 0, 0u}; }
    __device__ S load(size_t i) const {
        const uint32_t m = c_meta[i];
        const bool head = seg_start[i] == (int32_t)i;
        const bool part = manages_execution(m);
        const bool wr = meta_kind(m) == AD_KIND_WRITE;
        S s = identity();
        s.flags = (head ? 1u : 0u) | (part ? 2u : 0u) | (wr ? 4u : 0u);
        if (!part) {
            if (head) { s.m00 = s.m01 = s.m10 = s.m11 = NEG; s.c0 = -1; s.c1 = -1; }
            return s;
        }
        const int a = (int)L[c_txn[i]];
        s.a = a;
        if (head) {                          // constant map: f(init = (-1,-1))
            s.m00 = s.m01 = s.m10 = s.m11 = NEG;
            s.c0 = a;
            s.c1 = wr ? a : -1;
        } else if (wr) {
            s.m00 = 1; s.m01 = 1; s.m10 = 1; s.m11 = 1; s.c0 = a; s.c1 = a;
        } else {
            s.m00 = 0; s.m01 = 1; s.m10 = NEG; s.m11 = 0; s.c0 = a; s.c1 = NEG;
        }
        return s;
    }
    // later o earlier
    __device__ S combine(const S& f, const S& g) const {
        S h;
        h.m00 = mp_max(mp_add(g.m00, f.m00), mp_add(g.m01, f.m10));
        h.m01 = mp_max(mp_add(g.m00, f.m01), mp_add(g.m01, f.m11));
        h.m10 = mp_max(mp_add(g.m10, f.m00), mp_add(g.m11, f.m10));
        h.m11 = mp_max(mp_add(g.m10, f.m01), mp_add(g.m11, f.m11));
        h.c0 = mp_max(mp_max(mp_add(g.m00, f.c0), mp_add(g.m01, f.c1)), g.c0);
        h.c1 = mp_max(mp_max(mp_add(g.m10, f.c0), mp_add(g.m11, f.c1)), g.c1);
        h.a = 0; h.flags = 0;
        return h;
    }
    __device__ void store(size_t i, const S& ex, const S&, const S& el) const {
        if (!(el.flags & 2u)) return;
        int py, pw;
        if (el.flags & 1u) { py = -1; pw = -1; }
        else {
            py = mp_max(mp_max(mp_add(ex.m00, -1), mp_add(ex.m01, -1)), ex.c0);
            pw = mp_max(mp_max(mp_add(ex.m10, -1), mp_add(ex.m11, -1)), ex.c1);
        }
        const int x = (el.flags & 4u) ? mp_max(py + 1, el.a) : mp_max(pw + 1, el.a);
        if (x > el.a) {
            uint32_t old = atomicMax(&L[c_txn[i]], (uint32_t)x);
            if (old < (uint32_t)x) *changed = 1u;
        }
    }
};

__global__ __launch_bounds__(256) void k_chain_copy(size_t P, const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                                    const uint64_t* __restrict__ e_exec1, uint32_t* __restrict__ c_txn,
                                                    uint8_t* __restrict__ c_meta, uint64_t* __restrict__ c_exec1) {
    const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P) return;
    c_txn[s] = e_txn[s];
    c_meta[s] = e_meta[s];
    c_exec1[s] = e_exec1[s];
}

// Per-segment fix-up: entries of one key ordered by executeAt (insertion sort; one thread per segment).
__global__ __launch_bounds__(256) void k_chain_order(size_t P, const int32_t* __restrict__ seg_start,
                                                     uint32_t* __restrict__ c_txn, uint8_t* __restrict__ c_meta,
                                                     uint64_t* __restrict__ c_exec1) {
    const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P || seg_start[s] != (int32_t)s) return;
    size_t e = s + 1;
    bool sorted = true;
    uint64_t prev = c_exec1[s];
    while (e < P && seg_start[e] == (int32_t)s) {
        uint64_t x = c_exec1[e];
        if (x < prev) sorted = false;
        prev = x;
        ++e;
    }
    if (sorted) return;
    for (size_t x = s + 1; x < e; ++x) {
        uint64_t kx = c_exec1[x];
        uint32_t tx = c_txn[x];
        uint8_t mx = c_meta[x];
        size_t y = x;
        while (y > s && c_exec1[y - 1] > kx) {
            c_exec1[y] = c_exec1[y - 1]; c_txn[y] = c_txn[y - 1]; c_meta[y] = c_meta[y - 1];
            --y;
        }
        c_exec1[y] = kx; c_txn[y] = tx; c_meta[y] = mx;
    }
}

__global__ __launch_bounds__(256) void k_exec_split(size_t n, const uint64_t* __restrict__ ex1, const uint32_t* __restrict__ idx,
                                                    uint32_t* __restrict__ key, int hi) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = idx ? idx[i] : (uint32_t)i;
    const uint64_t e = ex1[t] - 1;
    key[i] = hi ? (uint32_t)(e >> 32) : (uint32_t)e;
}
__global__ __launch_bounds__(256) void k_iota(size_t n, uint32_t* __restrict__ v) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}
__global__ __launch_bounds__(256) void k_gather_u32(size_t n, const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                    uint32_t* __restrict__ dst, uint32_t* __restrict__ maxv) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v = 0;
    if (i < n) { v = src[idx[i]]; dst[i] = v; }
    v = wave_max(v);
    if (maxv && __lane_id() == 0) atomicMax(maxv, v);
}

struct LevelState {
    size_t capP = 0, capN = 0;
    uint32_t* c_txn = nullptr;
    uint8_t* c_meta = nullptr;
    uint64_t* c_exec1 = nullptr;
    uint32_t* flags = nullptr;          // [0] changed, [1] max level
    void* agg = nullptr;
    size_t agg_cap = 0;
    uint32_t *sk0 = nullptr, *sv0 = nullptr, *sk1 = nullptr, *sv1 = nullptr;
    uint32_t* rs = nullptr;              // radix scratch
    size_t rs_cap = 0;
};

inline void free_level_state(LevelState& s) {
    void* ps[] = {s.c_txn, s.c_meta, s.c_exec1, s.flags, s.agg, s.sk0, s.sv0, s.sk1, s.sv1, s.rs};
    for (void* p : ps) if (p) hipFree(p);
    s = LevelState{};
}

inline size_t level_scratch_bytes(size_t, size_t) { return 0; }

struct LevelInputs {
    size_t n, P;
    const uint32_t* skey;
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const int32_t* seg_start;
    const uint8_t* meta;
    const uint64_t* ex1;
    uint32_t* lvl;
    uint32_t* order;
    void* scratch;
    size_t scratch_cap;
    const DevCsr* merged_direct;
    const DevCsr* merged_range;
    uint32_t n_large;
    uint32_t exec_bits;
};

inline int run_levels(LevelState& ls, const LevelInputs& in, bool want_order, hipStream_t st, int* iters,
                      std::string& err) {
    const size_t n = in.n, P = in.P;
    auto grow = [&](void** p, size_t bytes, size_t& cap) -> bool {
        if (cap >= bytes && *p) return true;
        if (*p) { hipStreamSynchronize(st); hipFree(*p); *p = nullptr; }
        if (hipMalloc(p, bytes) != hipSuccess) return false;
        cap = bytes;
        return true;
    };
    if ((in.merged_direct && in.merged_direct->nkeys > 0) || (in.merged_range && in.merged_range->nkeys > 0) || in.n_large > 0) {
        err = "exec levels: direct-key / range dependencies and range txns are not supported by this build's device path";
        return AD_ERR_UNSUPPORTED;
    }
    if (ls.capP < P || !ls.c_txn) {
        size_t c = std::max<size_t>(P, 1);
        size_t dummy;
        dummy = 0; if (!grow((void**)&ls.c_txn, c * 4, dummy)) goto oom;
        dummy = 0; if (!grow((void**)&ls.c_meta, c, dummy)) goto oom;
        dummy = 0; if (!grow((void**)&ls.c_exec1, c * 8, dummy)) goto oom;
        ls.capP = c;
    }
    if (ls.capN < n || !ls.sk0) {
        size_t c = std::max<size_t>(n, 1);
        size_t dummy;
        dummy = 0; if (!grow((void**)&ls.sk0, c * 4, dummy)) goto oom;
        dummy = 0; if (!grow((void**)&ls.sv0, c * 4, dummy)) goto oom;
        dummy = 0; if (!grow((void**)&ls.sk1, c * 4, dummy)) goto oom;
        dummy = 0; if (!grow((void**)&ls.sv1, c * 4, dummy)) goto oom;
        ls.capN = c;
    }
    if (!ls.flags) { size_t d = 0; if (!grow((void**)&ls.flags, 256, d)) goto oom; }
    if (!grow(&ls.agg, device_scan_scratch<ChainOp>(std::max<size_t>(P, 1)) + 256, ls.agg_cap)) goto oom;
    if (!grow((void**)&ls.rs, (3 * (radix_hist_len(std::max<size_t>(n, 1)) + 128) + 64 * 1024) * 4, ls.rs_cap)) goto oom;

    hipMemsetAsync(in.lvl, 0, std::max<size_t>(n, 1) * 4, st);
    *iters = 0;
    if (P > 0) {
        {
            KScope ks(K_CHAIN_PREP);
            k_chain_copy<<<ceil_div((long)P, 256), 256, 0, st>>>(P, in.e_txn, in.e_meta, in.e_exec1, ls.c_txn, ls.c_meta, ls.c_exec1);
            k_chain_order<<<ceil_div((long)P, 256), 256, 0, st>>>(P, in.seg_start, ls.c_txn, ls.c_meta, ls.c_exec1);
        }
        ChainOp op{ls.c_txn, ls.c_meta, in.seg_start, in.lvl, ls.flags};
        for (int it = 0; it < (1 << 22); ++it) {
            hipMemsetAsync(ls.flags, 0, 4, st);
            { KScope ks(K_SCAN_CHAIN); device_scan(op, P, (ChainOp::S*)ls.agg, st); }
            uint32_t changed = 0;
            if (hipMemcpyAsync(&changed, ls.flags, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                err = "exec levels: device error";
                return AD_ERR_DEVICE;
            }
            *iters = it + 1;
            if (!changed) break;
        }
    }
    if (want_order && n > 0) {
        RadixScratch rs;
        const size_t hl = radix_hist_len(n);
        rs.hist = ls.rs;
        rs.offs = rs.hist + hl + 64;
        rs.agg = rs.offs + hl + 64;
        const int g = ceil_div((long)n, 256);
        const int eb = (int)in.exec_bits;
        // executeAt order: low 32 bits then high bits (stable LSD)
        k_exec_split<<<g, 256, 0, st>>>(n, in.ex1, nullptr, ls.sk0, 0);
        k_iota<<<g, 256, 0, st>>>(n, ls.sv0);
        uint32_t *k = ls.sk0, *v = ls.sv0, *ko = ls.sk1, *vo = ls.sv1;
        if (radix_sort_pairs(k, v, ko, vo, n, eb < 32 ? eb : 32, rs, st)) { std::swap(k, ko); std::swap(v, vo); }
        if (eb > 32) {
            k_exec_split<<<g, 256, 0, st>>>(n, in.ex1, v, k, 1);
            if (radix_sort_pairs(k, v, ko, vo, n, eb - 32, rs, st)) { std::swap(k, ko); std::swap(v, vo); }
        }
        // then stably by level
        hipMemsetAsync(ls.flags + 1, 0, 4, st);
        k_gather_u32<<<g, 256, 0, st>>>(n, in.lvl, v, k, ls.flags + 1);
        uint32_t maxl = 0;
        hipMemcpyAsync(&maxl, ls.flags + 1, 4, hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
        int lb = maxl == 0 ? 0 : 32 - __builtin_clz(maxl);
        if (radix_sort_pairs(k, v, ko, vo, n, lb, rs, st)) { std::swap(k, ko); std::swap(v, vo); }
        hipMemcpyAsync(in.order, v, n * 4, hipMemcpyDeviceToDevice, st);
    }
    return AD_OK;
oom:
    err = "exec levels: out of device memory";
    return AD_ERR_NOMEM;
}

}  // namespace ad
