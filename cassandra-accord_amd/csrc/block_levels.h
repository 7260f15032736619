// block_levels.h — execution levels of deep key-chain graphs (C3: Zipf hot keys, ~1.6*10^5 levels) by
// executeAt blocks instead of Kahn wavefronts.
//
// The levels are the reference's release order (level_kernels.h header; oracle.cpp exec_levels), which is a
// sequential DP in executeAt order: level[T] = max over T's keys k of (Write ? y_k + 1 : w_k + 1) (0 if none),
// then y_k = max(y_k, level[T]) and, for a Write, w_k = max(w_k, level[T]) — y_k the greatest level on key k
// so far, w_k the greatest Write level (CommandsForKey.notifyManaged + unappliedCounters,
// local/cfk/CommandsForKey.java:1208-1330).  Every edge goes forward in executeAt, so the DP can be cut
// into consecutive executeAt blocks whose only inputs from the past are the per-key states (y_k, w_k) the
// earlier blocks leave (the "carry").  Inside a block:
//   * the entries are grouped by key (key-major, executeAt-minor: a contiguous run of each key's chain);
//   * along one key the DP step is a max-plus affine map of (y, w) — Read: y' = max(y, w+1, a), w' = w;
//     Write: y' = w' = max(y+1, a), a = the txn's level from its other keys — and maps compose, so ONE
//     block-wide scan resolves every key run of the block at once, whatever its depth;
//   * txns couple key runs (a = max over the txn's entries), so the scan repeats until no txn's level
//     rises (a Jacobi fixpoint inside the block: ~6 rounds for C3's 256-txn blocks, because only the
//     block's few hot keys couple).
// One workgroup walks the blocks in executeAt order (the carry is a sequential dependency); each block's
// state lives in LDS.  Cost = blocks x rounds x one 1024-entry LDS scan, instead of depth x one global
// wavefront (C3: ~2.7*10^4 scans vs ~1.6*10^5 wavefronts).
//
// Preparation (all parallel, once per batch): chain order by (key, executeAt) (k_chain_rank), executeAt rank
// of every txn (order_rows with zero levels), block of every txn from the prefix of its entry counts
// (blocks hold <= BL_CAP entries and <= BL_CAP txns), a stable radix sort of the chain positions by block,
// and one 8-byte record per entry: carry slot (the key's segment head), txn index inside the block, Write /
// first-of-key-in-block / last-of-key-in-block bits.
#pragma once

namespace ad {

constexpr int BL_T = 256;                    // one wave per SIMD
constexpr int BL_EPT = 4;                    // entries per thread
constexpr int BL_CAP = BL_T * BL_EPT;        // entries (and txns) per block
constexpr int BL_NEG = -(1 << 28);
constexpr uint32_t BL_TL = (1u << 11) - 1;     // txn-in-block index bits of a record's high word

// y' = max(y + a00, w + a01, c0), w' = max(y + a10, w + a11, c1)
struct BlMap {
    int a00, a01, a10, a11, c0, c1;
};
__device__ inline int bl_clamp(int x) { return x < BL_NEG ? BL_NEG : x; }
__device__ inline BlMap bl_identity() { return BlMap{0, BL_NEG, BL_NEG, 0, BL_NEG, BL_NEG}; }
// g o f (f earlier, g later); entries clamp at BL_NEG so repeated composition never overflows
__device__ inline BlMap bl_compose(const BlMap& f, const BlMap& g) {
    BlMap h;
    h.a00 = bl_clamp(max(f.a00 + g.a00, f.a10 + g.a01));
    h.a01 = bl_clamp(max(f.a01 + g.a00, f.a11 + g.a01));
    h.a10 = bl_clamp(max(f.a00 + g.a10, f.a10 + g.a11));
    h.a11 = bl_clamp(max(f.a01 + g.a10, f.a11 + g.a11));
    h.c0 = bl_clamp(max(max(f.c0 + g.a00, f.c1 + g.a01), g.c0));
    h.c1 = bl_clamp(max(max(f.c0 + g.a10, f.c1 + g.a11), g.c1));
    return h;
}
struct BlOp {                                 // adaptor for the DPP wave scan (scan.h)
    using S = BlMap;
    __device__ S identity() const { return bl_identity(); }
    __device__ S combine(const S& f, const S& g) const { return bl_compose(f, g); }
};

// executeAt rank of every txn (order[k] = txn at rank k)
static __global__ __launch_bounds__(256) void k_bl_erank(size_t n, const uint32_t* __restrict__ order, uint32_t* __restrict__ erank) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) erank[order[k]] = (uint32_t)k;
}
// exclusive prefix of max(1, keys) in executeAt order (a key-less txn still takes one txn slot of its block)
struct BlCntOp {
    using S = uint32_t;
    const uint32_t* order;
    const uint32_t* key_off;
    uint32_t* epre;
    size_t n;
    __device__ S load(size_t k) const {
        const uint32_t t = order[k];
        const uint32_t c = key_off[t + 1] - key_off[t];
        return c ? c : 1u;
    }
    __device__ S identity() const { return 0u; }
    __device__ S combine(S a, S b) const { return a + b; }
    __device__ void store(size_t k, S ex, S inc, S) const {
        epre[k] = ex;
        if (k + 1 == n) epre[n] = inc;
    }
};
// block of every chain position (blocks cut the entry prefix every bcap; a txn belongs to the block its
// first entry falls in, so a block holds < bcap + max keys per txn entries)
static __global__ __launch_bounds__(256) void k_bl_chain_block(size_t P, const uint32_t* __restrict__ c_txn, const uint32_t* __restrict__ erank,
                                                        const uint32_t* __restrict__ epre, uint32_t bcap, uint32_t* __restrict__ bk,
                                                        uint32_t* __restrict__ bv) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    bk[q] = epre[erank[c_txn[q]]] / bcap;
    bv[q] = (uint32_t)q;
}
// tb[b] = first executeAt rank of block b, boff[b] = first slot of block b (b = 0..B)
static __global__ __launch_bounds__(256) void k_bl_bounds(uint32_t B, size_t n, size_t P, const uint32_t* __restrict__ epre, uint32_t bcap,
                                                   const uint32_t* __restrict__ sk, uint32_t* __restrict__ tb, uint32_t* __restrict__ boff) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > B) return;
    const uint64_t want = (uint64_t)b * bcap;
    size_t lo = 0, hi = n;
    while (lo < hi) { const size_t m = (lo + hi) >> 1; if (epre[m] < want) lo = m + 1; else hi = m; }
    tb[b] = (uint32_t)lo;
    lo = 0; hi = P;
    while (lo < hi) { const size_t m = (lo + hi) >> 1; if (sk[m] < b) lo = m + 1; else hi = m; }
    boff[b] = (uint32_t)lo;
}
// Record of one slot of the block-sorted entries (u64):
//   bits  0-31  carry slot in global memory (the key's segment head position)
//   bits 32-42  txn index inside the block                     bit 43 Write
//   bit  44     first entry of its key in the block (HEAD)      bit 45 last (LAST)
//   bit  46     LAST entry whose key continues >= 3 blocks later: its carry also goes to global memory
//   bits 47-48  HEAD's carry source: 0 none (the key's first entry: (-1, -1)), 1 the LDS ring (the key's
//               previous run ended 1 or 2 blocks earlier), 2 global memory (earlier)
//   bits 49-60  LDS ring index of that previous run's last entry ((block % 3) * BL_CAP + slot in its block)
constexpr int BL_SH_W = 11, BL_SH_HEAD = 12, BL_SH_LAST = 13, BL_SH_G = 14, BL_SH_SRC = 15, BL_SH_RING = 17;
constexpr uint32_t BL_NONE = 0xFFFFFFFFu;
__device__ inline uint32_t bl_block_of(uint32_t q, const uint32_t* c_txn, const uint32_t* erank, const uint32_t* epre, uint32_t bcap) {
    return epre[erank[c_txn[q]]] / bcap;
}
static __global__ __launch_bounds__(256) void k_bl_inverse(size_t P, const uint32_t* __restrict__ sv, uint32_t* __restrict__ inv) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < P) inv[sv[j]] = (uint32_t)j;
}
static __global__ __launch_bounds__(256) void k_bl_records(size_t P, const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                                                    const uint32_t* __restrict__ inv, const uint32_t* __restrict__ c_txn,
                                                    const uint8_t* __restrict__ c_meta, const int32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ erank, const uint32_t* __restrict__ epre, uint32_t bcap,
                                                    const uint32_t* __restrict__ tb, const uint32_t* __restrict__ boff,
                                                    uint64_t* __restrict__ rec, uint32_t* __restrict__ bad) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool b_ = false;
    if (j < P) {
        const uint32_t b = sk[j], q = sv[j];
        const uint32_t key = (uint32_t)seg_start[q];
        const bool head = j == 0 || sk[j - 1] != b || (uint32_t)seg_start[sv[j - 1]] != key;
        const bool last = j + 1 == P || sk[j + 1] != b || (uint32_t)seg_start[sv[j + 1]] != key;
        const uint32_t tl = erank[c_txn[q]] - tb[b];
        b_ = tl > BL_TL || j - boff[b] >= (uint32_t)BL_CAP;
        uint64_t fl = (uint64_t)(tl & BL_TL) | ((uint64_t)(meta_kind(c_meta[q]) == AD_KIND_WRITE) << BL_SH_W) |
                      ((uint64_t)head << BL_SH_HEAD) | ((uint64_t)last << BL_SH_LAST);
        if (last && q + 1 < P && (uint32_t)seg_start[q + 1] == key && bl_block_of(q + 1, c_txn, erank, epre, bcap) >= b + 3)
            fl |= 1ull << BL_SH_G;
        if (head && q != key) {                                   // the key's previous run
            const uint32_t pb = bl_block_of(q - 1, c_txn, erank, epre, bcap);
            if (b - pb <= 2) {
                const uint32_t ps = inv[q - 1] - boff[pb];
                fl |= (1ull << BL_SH_SRC) | ((uint64_t)((pb % 3) * BL_CAP + ps) << BL_SH_RING);
            } else {
                fl |= 2ull << BL_SH_SRC;
            }
        }
        rec[j] = (uint64_t)key | (fl << 32);
    }
    wave_set_flag(b_, bad);
}

// Rounds over the block's multi-entry key runs, compacted (in block order) into mfl / mcar, by ONE wave with
// E entries per lane: no barrier and no cross-wave step per round.  Every txn's singleton entries were
// folded into lv by the prefill, so only these entries can raise a level.  The round body is branch-free
// (absent entries are identity maps whose raises go to per-lane sink slots past BL_CAP).  On return mout[k] holds the
// carry-out of every LAST entry k (state after it, from the final levels).  Returns the rounds.
template <int E>
__device__ inline uint32_t bl_wave_rounds(int nm, const uint32_t* __restrict__ mfl, const int2* __restrict__ mcar, int* lv,
                                          const uint8_t* nl, int2* mout) {
    const int lane = __lane_id();
    uint32_t slot[E];
    bool valid[E], head[E], wr[E], last[E];
    int yc[E], wc[E], py[E], pw[E], a[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int k = lane * E + e;
        valid[e] = k < nm;
        const uint32_t fe = valid[e] ? mfl[k] : 0u;
        const int2 c = valid[e] ? mcar[k] : make_int2(-1, -1);
        slot[e] = valid[e] ? (fe & BL_TL) : (uint32_t)(BL_CAP + lane);     // absent: the lane's own sink
        head[e] = fe & (1u << BL_SH_HEAD);
        wr[e] = fe & (1u << BL_SH_W);
        last[e] = valid[e] && (fe & (1u << BL_SH_LAST));
        yc[e] = c.x; wc[e] = c.y;
        py[e] = pw[e] = -1;
    }
    const BlOp op{};
    uint32_t it = 0;
    while (true) {
#pragma unroll
        for (int e = 0; e < E; ++e) a[e] = lv[slot[e]];
        // the lane's aggregate, field by field (a struct select would go through scratch memory)
        int g00 = 0, g01 = BL_NEG, g10 = BL_NEG, g11 = 0, gc0 = BL_NEG, gc1 = BL_NEG;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            // head -> constant; Write: y' = w' = max(y + 1, a); Read: y' = max(y, w + 1, a), w' = w
            const bool W = wr[e], H = head[e], V = valid[e];
            const int hx = W ? max(yc[e] + 1, a[e]) : max(wc[e] + 1, a[e]);
            const int c0w = max(gc0 + 1, a[e]);
            int n00 = W ? g00 + 1 : max(g00, g10 + 1);
            int n01 = W ? g01 + 1 : max(g01, g11 + 1);
            int n10 = W ? g00 + 1 : g10;
            int n11 = W ? g01 + 1 : g11;
            int nc0 = W ? c0w : max(max(gc0, gc1 + 1), a[e]);
            int nc1 = W ? c0w : gc1;
            n00 = H ? BL_NEG : n00;
            n01 = H ? BL_NEG : n01;
            n10 = H ? BL_NEG : n10;
            n11 = H ? BL_NEG : n11;
            nc0 = H ? max(yc[e], hx) : nc0;
            nc1 = H ? (W ? hx : wc[e]) : nc1;
            g00 = V ? n00 : g00; g01 = V ? n01 : g01; g10 = V ? n10 : g10;
            g11 = V ? n11 : g11; gc0 = V ? nc0 : gc0; gc1 = V ? nc1 : gc1;
        }
        BlMap agg;
        agg.a00 = g00; agg.a01 = g01; agg.a10 = g10; agg.a11 = g11; agg.c0 = gc0; agg.c1 = gc1;
        agg.a00 = bl_clamp(agg.a00); agg.a01 = bl_clamp(agg.a01); agg.a10 = bl_clamp(agg.a10); agg.a11 = bl_clamp(agg.a11);
        const BlMap inc = wave_incl_scan(op, agg);
        const BlMap pre = wave_shift_up1(op, inc);
        int y = max(pre.a00 - 1, max(pre.a01 - 1, pre.c0));
        int w = max(pre.a10 - 1, max(pre.a11 - 1, pre.c1));
        bool up = false;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            y = head[e] ? yc[e] : y;
            w = head[e] ? wc[e] : w;
            py[e] = y; pw[e] = w;
            const int x = wr[e] ? max(y + 1, a[e]) : max(w + 1, a[e]);
            if (x > a[e]) {                              // rare after the first round: the branch is skipped
                atomicMax(&lv[slot[e]], x);
                up |= nl[slot[e]] != 0;
            }
            y = max(y, x);
            w = wr[e] ? x : w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // this round's raises before the next reads
        ++it;
        if (!__ballot(up)) break;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (!last[e]) continue;
        const int x = lv[slot[e]];
        mout[lane * E + e] = make_int2(max(py[e], x), wr[e] ? x : pw[e]);
    }
    return it;
}

struct BlIntSum {
    using S = int;
    __device__ S identity() const { return 0; }
    __device__ S combine(S a, S b) const { return a + b; }
};

// The sequential walk over the blocks (one workgroup; see the file header).  Per block:
//   setup (all waves)  carry-in of the key runs that start here (LDS ring of the last three blocks'
//                      carry-outs, else global memory), prefill of every txn's level with its heads' carry
//                      bounds (a singleton run is then final), compaction of the multi-entry runs in block
//                      order;
//   rounds (wave 0)    bl_wave_rounds until no txn with a non-final entry rises; meanwhile waves 1-3 stage
//                      the NEXT block's records, global carry-ins and order slice into LDS, so no global
//                      load latency sits on the sequential path;
//   out (all waves)    carry-out of every run (ring; global memory for keys whose next run is >= 3 blocks
//                      away) and the levels.
// Global carries are written and read by this one workgroup (one CU): workgroup-scope ordering suffices.  A
// block's global stores are released (fence) at the end of the NEXT block, before that block's own stores,
// and read no earlier than the staging during the block after that.
// stats[0] = greatest level + 1, stats[1] = rounds, stats[2..3] = clock64 in rounds, stats[4..5] = total.
__device__ inline void bl_stage(uint32_t b, uint32_t B, int t, int nthr, const uint32_t* __restrict__ boff,
                                const uint32_t* __restrict__ tb, const uint64_t* __restrict__ rec, const int2* carry,
                                const uint32_t* __restrict__ order, uint64_t* srec, int2* scar, uint32_t* sord, uint32_t* sbnd) {
    if (b >= B) return;
    const uint32_t j0 = boff[b], j1 = boff[b + 1], t0 = tb[b], t1 = tb[b + 1];
    for (int x = t; x < BL_CAP; x += nthr) {
        const uint32_t j = j0 + (uint32_t)x;
        const uint64_t r = j < j1 ? rec[j] : ~0ull;
        int2 c = make_int2(-1, -1);
        if (r != ~0ull && (((uint32_t)(r >> 32) >> BL_SH_SRC) & 3u) == 2u) {
            const int* g = reinterpret_cast<const int*>(&carry[(uint32_t)r]);
            c.x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            c.y = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        srec[x] = r;
        scar[x] = c;
        sord[x] = (uint32_t)x < t1 - t0 ? order[t0 + x] : 0u;
    }
    if (t == 0) { sbnd[0] = j0; sbnd[1] = j1; sbnd[2] = t0; sbnd[3] = t1; }
}

static __global__ __launch_bounds__(BL_T) void k_level_blocks(uint32_t B, const uint32_t* __restrict__ boff, const uint32_t* __restrict__ tb,
                                                       const uint64_t* __restrict__ rec, int2* carry,
                                                       const uint32_t* __restrict__ order, uint32_t* __restrict__ L,
                                                       uint32_t* __restrict__ stats) {
    __shared__ int lvb[2][BL_CAP + WAVE];      // levels of the block's txns (txn-in-block index), by block parity;
                                               // [BL_CAP + lane]: sinks of the rounds' absent entries
    __shared__ uint8_t nlb[2][BL_CAP + WAVE];     // txn has an entry that is not its key's last in the block
    __shared__ int2 ring[3 * BL_CAP];          // carry-out of every slot of the last three blocks
    __shared__ uint32_t mfl[BL_CAP];           // compacted multi-entry runs: record flags
    __shared__ int2 mcar[BL_CAP];              //   carry-in (heads)
    __shared__ int2 mout[BL_CAP];              //   carry-out (LAST entries)
    __shared__ uint64_t srec[BL_CAP];          // staged next block: records, global carry-ins, order slice
    __shared__ int2 scar[BL_CAP];
    __shared__ uint32_t sord[BL_CAP];
    __shared__ uint32_t sbnd[4];
    __shared__ int sred[BL_T / WAVE];
    __shared__ uint32_t srounds;
    const int tid = threadIdx.x, lane = __lane_id();
    const uint64_t tstart = clock64();
    uint64_t tround = 0;
    for (int x = tid; x < BL_CAP + WAVE; x += BL_T) { lvb[0][x] = lvb[1][x] = 0; nlb[0][x] = nlb[1][x] = 0; }
    int maxl = -1;
    uint32_t rounds = 0;
    bl_stage(0, B, tid, BL_T, boff, tb, rec, carry, order, srec, scar, sord, sbnd);
    uint32_t pfl[BL_EPT];
#pragma unroll
    for (int e = 0; e < BL_EPT; ++e) pfl[e] = BL_NONE;
    __syncthreads();
    for (uint32_t b = 0; b < B; ++b) {
        const int pb = b & 1;
        int* lv = lvb[pb];
        uint8_t* nl = nlb[pb];
        const uint32_t nt = sbnd[3] - sbnd[2];
        uint32_t fl[BL_EPT], key[BL_EPT], ord[BL_EPT];
        int yc[BL_EPT], wc[BL_EPT];
#pragma unroll
        for (int e = 0; e < BL_EPT; ++e) {
            const uint64_t r = srec[tid * BL_EPT + e];
            key[e] = (uint32_t)r;
            fl[e] = r == ~0ull ? BL_NONE : (uint32_t)(r >> 32);
            const int2 c = scar[tid * BL_EPT + e];
            yc[e] = c.x; wc[e] = c.y;
            ord[e] = sord[tid + e * BL_T];
        }
        // ---- setup: clear the previous block's slots (other parity), carry-in, prefill, compaction
#pragma unroll
        for (int e = 0; e < BL_EPT; ++e)
            if (pfl[e] != BL_NONE) { lvb[pb ^ 1][pfl[e] & BL_TL] = 0; nlb[pb ^ 1][pfl[e] & BL_TL] = 0; }
        int mcount = 0;
#pragma unroll
        for (int e = 0; e < BL_EPT; ++e) {
            const uint32_t f = fl[e];
            if (f == BL_NONE) continue;
            const bool head = f & (1u << BL_SH_HEAD), last = f & (1u << BL_SH_LAST);
            if (head) {
                const uint32_t src = (f >> BL_SH_SRC) & 3u;
                if (src == 0u) { yc[e] = -1; wc[e] = -1; }
                else if (src == 1u) { const int2 c = ring[f >> BL_SH_RING]; yc[e] = c.x; wc[e] = c.y; }
                const int lb = (f & (1u << BL_SH_W)) ? yc[e] + 1 : wc[e] + 1;
                if (lb > 0) atomicMax(&lv[f & BL_TL], lb);
            }
            if (!last) nl[f & BL_TL] = 1;
            mcount += (head && last) ? 0 : 1;
        }
        int mtotal;
        const int mbase = block_exclusive_scan<BlIntSum, BL_T>(BlIntSum{}, mcount, sred, &mtotal);
        {
            int k = mbase;
#pragma unroll
            for (int e = 0; e < BL_EPT; ++e) {
                const uint32_t f = fl[e];
                if (f == BL_NONE || ((f & (1u << BL_SH_HEAD)) && (f & (1u << BL_SH_LAST)))) continue;
                mfl[k] = f;
                mcar[k] = make_int2(yc[e], wc[e]);
                ++k;
            }
        }
        __syncthreads();
        // ---- rounds (wave 0) | staging of the next block (waves 1-3)
        if (tid < WAVE) {
            if (mtotal > 0) {
                const uint64_t t0 = clock64();
                uint32_t r;
                const int epl = (mtotal + WAVE - 1) / WAVE;        // entries per lane
                if (epl <= 2) r = bl_wave_rounds<2>(mtotal, mfl, mcar, lv, nl, mout);
                else if (epl <= 3) r = bl_wave_rounds<3>(mtotal, mfl, mcar, lv, nl, mout);
                else if (epl <= 4) r = bl_wave_rounds<4>(mtotal, mfl, mcar, lv, nl, mout);
                else if (epl <= 5) r = bl_wave_rounds<5>(mtotal, mfl, mcar, lv, nl, mout);
                else if (epl <= 6) r = bl_wave_rounds<6>(mtotal, mfl, mcar, lv, nl, mout);
                else if (epl <= 8) r = bl_wave_rounds<8>(mtotal, mfl, mcar, lv, nl, mout);
                else if (epl <= 12) r = bl_wave_rounds<12>(mtotal, mfl, mcar, lv, nl, mout);
                else r = bl_wave_rounds<16>(mtotal, mfl, mcar, lv, nl, mout);
                tround += clock64() - t0;
                rounds += r;
            }
        } else {
            bl_stage(b + 1, B, tid - WAVE, BL_T - WAVE, boff, tb, rec, carry, order, srec, scar, sord, sbnd);
        }
        __syncthreads();
        // ---- out: carry-out of every run's LAST entry, levels.  The fence first releases the previous
        // block's global carries (issued a block ago) before this block's are issued.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        const int rb = (int)(b % 3) * BL_CAP;
        {
            int k = mbase;
#pragma unroll
            for (int e = 0; e < BL_EPT; ++e) {
                const uint32_t f = fl[e];
                if (f == BL_NONE) continue;
                const bool head = f & (1u << BL_SH_HEAD), last = f & (1u << BL_SH_LAST);
                const bool multi = !(head && last);
                if (last) {
                    int2 c;
                    if (multi) {
                        c = mout[k];
                    } else {
                        const int x = lv[f & BL_TL];
                        c = make_int2(max(yc[e], x), (f & (1u << BL_SH_W)) ? x : wc[e]);
                    }
                    ring[rb + tid * BL_EPT + e] = c;
                    if (f & (1u << BL_SH_G)) {
                        int* g = reinterpret_cast<int*>(&carry[key[e]]);
                        __hip_atomic_store(g, c.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(g + 1, c.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                if (multi) ++k;
            }
        }
#pragma unroll
        for (int e = 0; e < BL_EPT; ++e) {
            const uint32_t x = (uint32_t)(tid + e * BL_T);
            if (x < nt) {
                const int l = lv[x];
                L[ord[e]] = (uint32_t)l;
                maxl = max(maxl, l);
            }
        }
#pragma unroll
        for (int e = 0; e < BL_EPT; ++e) pfl[e] = fl[e];
        __syncthreads();
    }
    maxl = wave_max(maxl);
    if (lane == 0) atomicMax(&stats[0], (uint32_t)(maxl + 1));
    if (tid == 0) {
        stats[1] = rounds;
        const uint64_t tot = clock64() - tstart;
        stats[2] = (uint32_t)tround; stats[3] = (uint32_t)(tround >> 32);
        stats[4] = (uint32_t)tot; stats[5] = (uint32_t)(tot >> 32);
    }
}

struct BlockBufs {                             // grow-only, owned by LevelState
    uint64_t* rec = nullptr;                   // [P]
    uint32_t *epre = nullptr, *erank = nullptr, *bk = nullptr, *bv = nullptr, *bk2 = nullptr, *bv2 = nullptr;
    uint32_t *tb = nullptr, *boff = nullptr, *stats = nullptr, *rs = nullptr;
    int2* carry = nullptr;
    size_t capP = 0, capN = 0, capB = 0, rs_cap = 0;
    uint32_t nblocks = 0;                      // blocks of the last run
};

inline void free_block_bufs(BlockBufs& b) {
    void* ps[] = {b.rec, b.epre, b.erank, b.bk, b.bv, b.bk2, b.bv2, b.tb, b.boff, b.stats, b.rs, b.carry};
    for (void* p : ps) if (p) hipFree(p);
    b = BlockBufs{};
}

}  // namespace ad
