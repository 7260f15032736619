// scan.h — generic device-wide (segmented) scans for gfx950.
//
// A scan is described by an Op with:
//   using S = ...;                          // the scanned state
//   __device__ S load(size_t i) const;      // element i (i < n)
//   __device__ S identity() const;
//   __device__ S combine(S earlier, S later) const;   // associative
//   __device__ void store(size_t i, S exclusive, S inclusive, S element) const;
// Three launches: per-tile aggregate, single-workgroup scan of the aggregates, per-tile apply.
// Tiles are BLOCK threads x ITEMS consecutive elements (thread-blocked, so loads of ITEMS
// consecutive elements per lane).  Used for CSR offsets (sum), segmented prefix maxima of the
// CFK elision state, and the max-plus execution-level chain scan.
#pragma once
#include "common.h"

namespace ad {

// Cross-lane moves of an arbitrary 4-byte-multiple state, dword by dword, through DPP (VALU-rate lane
// moves; ds_bpermute-based __shfl costs an LDS-crossbar round trip per dword, which made the 32-40 B
// scan states of the elision and chain scans shuffle-bound).  Lanes whose DPP source is outside the
// pattern (or whose row is masked off) receive `old`.
template <int CTRL, int ROW_MASK, class S>
__device__ inline S dpp_state(const S& v, const S& old) {
    static_assert(sizeof(S) % 4 == 0, "scan state must be a multiple of 4 bytes");
    constexpr int W = sizeof(S) / 4;
    S r;
    const int* a = reinterpret_cast<const int*>(&v);
    const int* o = reinterpret_cast<const int*>(&old);
    int* d = reinterpret_cast<int*>(&r);
#pragma unroll
    for (int k = 0; k < W; ++k) d[k] = __builtin_amdgcn_update_dpp(o[k], a[k], CTRL, ROW_MASK, 0xf, false);
    return r;
}
template <class S>
__device__ inline S readlane_state(const S& v, int lane) {
    constexpr int W = sizeof(S) / 4;
    S r;
    const int* a = reinterpret_cast<const int*>(&v);
    int* d = reinterpret_cast<int*>(&r);
#pragma unroll
    for (int k = 0; k < W; ++k) d[k] = __builtin_amdgcn_readlane(a[k], lane);
    return r;
}
// DPP controls (GFX9 family, wave64): row_shr:n = 0x110+n, row_bcast:15 = 0x142, row_bcast:31 = 0x143,
// wave_shr:1 = 0x138
// Inclusive ordered scan of one state per lane across the 64-lane wave: 4 row_shr steps inside each
// 16-lane row, then row 0/2's last lane into rows 1/3 and lane 31 into rows 2/3.
template <class Op>
__device__ inline typename Op::S wave_incl_scan(const Op& op, typename Op::S x) {
    using S = typename Op::S;
    const S id = op.identity();
    x = op.combine(dpp_state<0x111, 0xf>(x, id), x);
    x = op.combine(dpp_state<0x112, 0xf>(x, id), x);
    x = op.combine(dpp_state<0x114, 0xf>(x, id), x);
    x = op.combine(dpp_state<0x118, 0xf>(x, id), x);
    x = op.combine(dpp_state<0x142, 0xa>(x, id), x);
    x = op.combine(dpp_state<0x143, 0xc>(x, id), x);
    return x;
}
// the previous lane's value (lane 0: identity)
template <class Op>
__device__ inline typename Op::S wave_shift_up1(const Op& op, const typename Op::S& x) {
    return dpp_state<0x138, 0xf>(x, op.identity());
}

// Block-wide exclusive scan: 64-lane shuffle scan per wave (no LDS round trips), then one LDS slot per
// wave for the wave totals.  Returns the thread's exclusive prefix; *total = block aggregate.
template <class Op, int BLOCK>
__device__ inline typename Op::S block_exclusive_scan(const Op& op, typename Op::S v, typename Op::S* lds,
                                                      typename Op::S* total) {
    using S = typename Op::S;
    constexpr int NW = BLOCK / WAVE;
    const int lane = __lane_id();
    const int w = threadIdx.x / WAVE;
    const S x = wave_incl_scan(op, v);
    S ex_w = wave_shift_up1(op, x);
    if (lane == WAVE - 1) lds[w] = x;
    __syncthreads();
    S pre = op.identity();
    for (int k = 0; k < w; ++k) pre = op.combine(pre, lds[k]);
    if (total) {
        S tot = pre;
        for (int k = w; k < NW; ++k) tot = op.combine(tot, lds[k]);
        *total = tot;
    }
    __syncthreads();
    return op.combine(pre, ex_w);
}

// Wave-striped tiles: wave w of a block owns 64 * ITEMS consecutive elements; in round k lane l holds
// element wbase + 64k + l, so every load/store instruction of a wave touches 64 consecutive elements
// (coalesced).  Order is preserved: each round is an ordered 64-lane scan, rounds are folded in order,
// waves in wave order (the ops are associative, not commutative).
template <class Op, int BLOCK, int ITEMS>
static __global__ __launch_bounds__(BLOCK) void k_scan_reduce(Op op, size_t n, typename Op::S* agg) {
    using S = typename Op::S;
    constexpr int NW = BLOCK / WAVE;
    __shared__ S lds[NW];
    const int lane = __lane_id(), w = threadIdx.x / WAVE;
    const size_t wbase = (size_t)blockIdx.x * BLOCK * ITEMS + (size_t)w * WAVE * ITEMS;
    S acc = op.identity();
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const size_t i = wbase + (size_t)k * WAVE + lane;
        S x = wave_incl_scan(op, i < n ? op.load(i) : op.identity());
        acc = op.combine(acc, readlane_state(x, WAVE - 1));
    }
    if (lane == 0) lds[w] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        S t = lds[0];
        for (int k = 1; k < NW; ++k) t = op.combine(t, lds[k]);
        agg[blockIdx.x] = t;
    }
}

// Exclusive scan of nblk aggregates in place by one workgroup: chunks of BLOCK x AI, each thread folding
// AI consecutive aggregates serially before one block scan (4096 aggregates = one chunk: the 4M-entry
// elision scan spent 19 us here with one aggregate per thread and four chunk rounds).
template <class Op, int BLOCK, int AI = 4>
static __global__ __launch_bounds__(BLOCK) void k_scan_aggregates(Op op, int nblk, typename Op::S* agg) {
    using S = typename Op::S;
    __shared__ S lds[BLOCK / WAVE];
    S carry = op.identity();
    for (int c0 = 0; c0 < nblk; c0 += BLOCK * AI) {
        const int b = c0 + (int)threadIdx.x * AI;
        S v[AI];
        S t = op.identity();
#pragma unroll
        for (int k = 0; k < AI; ++k) {
            v[k] = b + k < nblk ? agg[b + k] : op.identity();
            t = op.combine(t, v[k]);
        }
        S total;
        S ex = op.combine(carry, block_exclusive_scan<Op, BLOCK>(op, t, lds, &total));
#pragma unroll
        for (int k = 0; k < AI; ++k) {
            if (b + k < nblk) agg[b + k] = ex;
            ex = op.combine(ex, v[k]);
        }
        carry = op.combine(carry, total);
        __syncthreads();
    }
}

template <class Op, int BLOCK, int ITEMS>
static __global__ __launch_bounds__(BLOCK) void k_scan_apply(Op op, size_t n, const typename Op::S* agg) {
    using S = typename Op::S;
    constexpr int NW = BLOCK / WAVE;
    __shared__ S lds[NW];
    const int lane = __lane_id(), w = threadIdx.x / WAVE;
    const size_t wbase = (size_t)blockIdx.x * BLOCK * ITEMS + (size_t)w * WAVE * ITEMS;
    S el[ITEMS], x[ITEMS];
    S acc = op.identity();
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const size_t i = wbase + (size_t)k * WAVE + lane;
        el[k] = i < n ? op.load(i) : op.identity();
        x[k] = wave_incl_scan(op, el[k]);
        acc = op.combine(acc, readlane_state(x[k], WAVE - 1));
    }
    if (lane == 0) lds[w] = acc;
    __syncthreads();
    S carry = agg[blockIdx.x];
    for (int k = 0; k < w; ++k) carry = op.combine(carry, lds[k]);
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const size_t i = wbase + (size_t)k * WAVE + lane;
        const S ex = op.combine(carry, wave_shift_up1(op, x[k]));
        const S inc = op.combine(carry, x[k]);
        if (i < n) op.store(i, ex, inc, el[k]);
        carry = op.combine(carry, readlane_state(x[k], WAVE - 1));
    }
}

template <class Op, int BLOCK = 256, int ITEMS = 4>
inline void device_scan(const Op& op, size_t n, typename Op::S* agg_scratch, hipStream_t st) {
    if (n == 0) return;
    const int nblk = ceil_div((long)n, (long)BLOCK * ITEMS);
    k_scan_reduce<Op, BLOCK, ITEMS><<<nblk, BLOCK, 0, st>>>(op, n, agg_scratch);
    k_scan_aggregates<Op, 1024><<<1, 1024, 0, st>>>(op, nblk, agg_scratch);
    k_scan_apply<Op, BLOCK, ITEMS><<<nblk, BLOCK, 0, st>>>(op, n, agg_scratch);
}
template <class Op, int BLOCK = 256, int ITEMS = 4>
inline size_t device_scan_scratch(size_t n) {
    return (size_t)ceil_div((long)n, (long)BLOCK * ITEMS) * sizeof(typename Op::S) + 64;
}

// ---- exclusive prefix sum producing offsets[0..n] (offsets[n] = total) ------------------------
template <class T>
struct SumOp {
    using S = T;
    const T* in;
    T* out;
    size_t n;
    __device__ S load(size_t i) const { return in[i]; }
    __device__ S identity() const { return 0; }
    __device__ S combine(S a, S b) const { return a + b; }
    __device__ void store(size_t i, S ex, S inc, S) const {
        out[i] = ex;
        if (i + 1 == n) out[n] = inc;
    }
};

// sum of a strided sequence: in[i] = a[i] + b[i]  (k2t sizes = keys + entries)
template <class T>
struct Sum2Op {
    using S = T;
    const T* a;
    const T* b;
    T* out;
    size_t n;
    __device__ S load(size_t i) const { return a[i] + b[i]; }
    __device__ S identity() const { return 0; }
    __device__ S combine(S x, S y) const { return x + y; }
    __device__ void store(size_t i, S ex, S inc, S) const {
        out[i] = ex;
        if (i + 1 == n) out[n] = inc;
    }
};

}  // namespace ad
