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

template <class Op, int BLOCK>
__device__ inline typename Op::S block_exclusive_scan(const Op& op, typename Op::S v, typename Op::S* lds,
                                                      typename Op::S* total) {
    using S = typename Op::S;
    const int t = threadIdx.x;
    lds[t] = v;
    __syncthreads();
    // Hillis-Steele inclusive scan over the BLOCK thread aggregates
    for (int off = 1; off < BLOCK; off <<= 1) {
        S x = lds[t];
        S y = t >= off ? op.combine(lds[t - off], x) : x;
        __syncthreads();
        lds[t] = y;
        __syncthreads();
    }
    S incl = lds[t];
    S excl = t == 0 ? op.identity() : lds[t - 1];
    if (total) *total = lds[BLOCK - 1];
    __syncthreads();
    (void)incl;
    return excl;
}

template <class Op, int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_scan_reduce(Op op, size_t n, typename Op::S* agg) {
    using S = typename Op::S;
    __shared__ S lds[BLOCK];
    const size_t base = (size_t)blockIdx.x * BLOCK * ITEMS + (size_t)threadIdx.x * ITEMS;
    S acc = op.identity();
#pragma unroll
    for (int k = 0; k < ITEMS; ++k)
        if (base + k < n) acc = op.combine(acc, op.load(base + k));
    S total;
    block_exclusive_scan<Op, BLOCK>(op, acc, lds, &total);
    if (threadIdx.x == 0) agg[blockIdx.x] = total;
}

// Exclusive scan of nblk aggregates in place by one workgroup (chunks of BLOCK with a carry).
template <class Op, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_scan_aggregates(Op op, int nblk, typename Op::S* agg) {
    using S = typename Op::S;
    __shared__ S lds[BLOCK];
    S carry = op.identity();
    for (int c0 = 0; c0 < nblk; c0 += BLOCK) {
        int i = c0 + threadIdx.x;
        S v = i < nblk ? agg[i] : op.identity();
        S total;
        S ex = block_exclusive_scan<Op, BLOCK>(op, v, lds, &total);
        if (i < nblk) agg[i] = op.combine(carry, ex);
        carry = op.combine(carry, total);
        __syncthreads();
    }
}

template <class Op, int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_scan_apply(Op op, size_t n, const typename Op::S* agg) {
    using S = typename Op::S;
    __shared__ S lds[BLOCK];
    const size_t base = (size_t)blockIdx.x * BLOCK * ITEMS + (size_t)threadIdx.x * ITEMS;
    S el[ITEMS];
    S acc = op.identity();
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        el[k] = base + k < n ? op.load(base + k) : op.identity();
        acc = op.combine(acc, el[k]);
    }
    S ex = block_exclusive_scan<Op, BLOCK>(op, acc, lds, nullptr);
    S run = op.combine(agg[blockIdx.x], ex);
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        if (base + k < n) {
            S inc = op.combine(run, el[k]);
            op.store(base + k, run, inc, el[k]);
            run = inc;
        }
    }
}

template <class Op, int BLOCK = 256, int ITEMS = 8>
inline void device_scan(const Op& op, size_t n, typename Op::S* agg_scratch, hipStream_t st) {
    if (n == 0) return;
    const int nblk = ceil_div((long)n, (long)BLOCK * ITEMS);
    k_scan_reduce<Op, BLOCK, ITEMS><<<nblk, BLOCK, 0, st>>>(op, n, agg_scratch);
    k_scan_aggregates<Op, 1024><<<1, 1024, 0, st>>>(op, nblk, agg_scratch);
    k_scan_apply<Op, BLOCK, ITEMS><<<nblk, BLOCK, 0, st>>>(op, n, agg_scratch);
}
template <class Op, int BLOCK = 256, int ITEMS = 8>
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
