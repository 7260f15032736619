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
//   * along one key the DP runs in write epochs (a Write and the Reads after it): a Write's level is
//     max(previous Write's level + 1 (+1 more if the epoch had Reads), its own bound a, 1 + the epoch's
//     greatest Read bound), a Read's max(a, previous Write's level + 1) -- a max-plus recurrence that unrolls
//     into two max scans of one packed word per entry (below), so ONE pair of wave scans resolves every key
//     run of the block at once, whatever its depth;
//   * txns couple key runs (a = max over the txn's entries), so the scan repeats until no txn's level
//     rises (a Jacobi fixpoint inside the block: ~6.4 rounds for C3's ~250-txn blocks, because only the
//     block's few hot keys couple).
// One workgroup walks the blocks in executeAt order (the carry is a sequential dependency); each block's
// state lives in LDS.  Cost = blocks x rounds x two one-word wave scans, instead of depth x one global
// wavefront (C3: ~2.7*10^4 rounds vs ~1.6*10^5 wavefronts).  (Round 3 scanned 2x2 max-plus maps of six ints:
// ~2,400 cycles a round, 72 % of the walk.)
//
// Preparation (all parallel, once per batch): chain order by (key, executeAt) (k_chain_rank), executeAt rank
// of every txn (order_rows with zero levels), block of every txn from the prefix of its entry counts
// (blocks hold <= BL_CAP entries and <= BL_CAP txns), a stable radix sort of the chain positions by block,
// one 8-byte record per entry: carry slot (the key's segment head), txn index inside the block, Write /
// first-of-key-in-block / last-of-key-in-block bits; then per block the compacted multi-entry runs with their
// static epoch / run ids and write-step prefix (k_bl_compact).
#pragma once

namespace ad {

constexpr int BL_T = 256;                    // one wave per SIMD
#ifndef AD_BL_EPT
#define AD_BL_EPT 4
#endif
constexpr int BL_EPT = AD_BL_EPT;            // entries per thread
constexpr int BL_CAP = BL_T * BL_EPT;        // entries (and txns) per block
constexpr uint32_t BL_TL = (1u << 11) - 1;     // txn-in-block index bits of a record's high word

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
// (blk: the same block per chain position, kept for k_bl_records past the sort's ping-pong)
static __global__ __launch_bounds__(256) void k_bl_chain_block(size_t P, const uint32_t* __restrict__ c_txn, const uint32_t* __restrict__ erank,
                                                        const uint32_t* __restrict__ epre, uint32_t bcap, uint32_t* __restrict__ bk,
                                                        uint32_t* __restrict__ bv, uint32_t* __restrict__ blk) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const uint32_t b = epre[erank[c_txn[q]]] / bcap;
    bk[q] = b;
    bv[q] = (uint32_t)q;
    blk[q] = b;
}
// The blocks' first executeAt ranks alone (tb of k_bl_bounds, before the block sort): tb[b] = first rank whose entry
// prefix reaches b * bcap, b = 0..B
static __global__ __launch_bounds__(256) void k_bl_tbounds(uint32_t B, size_t n, const uint32_t* __restrict__ epre, uint32_t bcap,
                                                    uint32_t* __restrict__ tb) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b > B) return;
    const uint64_t want = (uint64_t)b * bcap;
    size_t lo = 0, hi = n;
    while (lo < hi) { const size_t m = (lo + hi) >> 1; if (epre[m] < want) lo = m + 1; else hi = m; }
    tb[b] = (uint32_t)lo;
}
// k_bl_chain_block with the block found from the txn's executeAt rank among the blocks' first ranks (tb, in LDS)
// instead of a second random read (epre[rank]), and the txn's index inside its block kept per chain position (tl:
// k_bl_records reads it in chain order instead of gathering erank again).  One random read per entry (erank of its
// txn) where there were three.
constexpr int BL_TB_LDS = 8192;               // blocks + 1 held in LDS (32 KB)
static __global__ __launch_bounds__(256) void k_bl_chain_block_tb(size_t P, uint32_t B, const uint32_t* __restrict__ c_txn,
                                                           const uint32_t* __restrict__ erank, const uint32_t* __restrict__ tb,
                                                           uint32_t* __restrict__ bk, uint32_t* __restrict__ bv,
                                                           uint32_t* __restrict__ blk, uint32_t* __restrict__ tl) {
    __shared__ uint32_t s_tb[BL_TB_LDS];
    for (uint32_t x = threadIdx.x; x <= B; x += blockDim.x) s_tb[x] = tb[x];
    __syncthreads();
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < P; q += stride) {
        const uint32_t r = erank[c_txn[q]];
        uint32_t lo = 0, hi = B;                    // the last block whose first rank is <= r
        while (lo < hi) { const uint32_t m = (lo + hi + 1) >> 1; if (s_tb[m] <= r) lo = m; else hi = m - 1; }
        bk[q] = lo;
        bv[q] = (uint32_t)q;
        blk[q] = lo;
        tl[q] = r - s_tb[lo];
    }
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
//   bits  0-31  HEAD with carry source 2: the block-sorted position of the key's previous run's last entry (its
//               producer stores the carry at its own position: a retiring block's stores stay inside its window)
//   bits 32-42  txn index inside the block                     bit 43 Write
//   bit  44     first entry of its key in the block (HEAD)      bit 45 last (LAST)
//   bit  46     LAST entry whose key continues >= 3 blocks later: its carry also goes to global memory
//   bits 47-48  HEAD's carry source: 0 none (the key's first entry: (-1, -1)), 1 the LDS ring (the key's
//               previous run ended 1 or 2 blocks earlier), 2 global memory (earlier)
//   bits 49-60  LDS ring index of that previous run's last entry ((block % 3) * BL_CAP + slot in its block)
//   bit  61     LAST entry whose key continues 1 or 2 blocks later (its carry goes to the LDS ring only)
constexpr int BL_SH_W = 11, BL_SH_HEAD = 12, BL_SH_LAST = 13, BL_SH_G = 14, BL_SH_SRC = 15, BL_SH_RING = 17,
              BL_SH_R = 29;
constexpr uint32_t BL_NONE = 0xFFFFFFFFu;
static_assert(BL_CAP - 1 <= (int)BL_TL, "txn-in-block index must fit the record's 11-bit field");
static_assert(3 * BL_CAP <= (1 << 12), "LDS ring index ((block % 3) * BL_CAP + slot) must fit 12 bits");
// stats words: [0..15] the walk's (k_level_blocks, below), [16] k_bl_records' layout-violation flag
constexpr int BL_STAT_RECORDS_BAD = 16;
constexpr size_t BL_STATS_BYTES = 4 * (BL_STAT_RECORDS_BAD + 4);
__device__ inline uint32_t bl_block_of(uint32_t q, const uint32_t* c_txn, const uint32_t* erank, const uint32_t* epre, uint32_t bcap) {
    return epre[erank[c_txn[q]]] / bcap;
}
static __global__ __launch_bounds__(256) void k_bl_inverse(size_t P, const uint32_t* __restrict__ sv, uint32_t* __restrict__ inv) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < P) inv[sv[j]] = (uint32_t)j;
}
// One thread per CHAIN position q (coalesced reads of the chain arrays and of q's neighbours), its record stored at
// its block-sorted slot inv[q].  Along a key's chain the blocks never decrease (blocks are executeAt ranges) and the
// block sort is stable, so the entry before q in its block is q - 1 exactly when blk[q - 1] == blk[q] and q is not
// its key's first position (else q heads its key's run in the block); symmetrically for the last entry.  Walking the
// block-sorted slots instead made ~10 dependent random reads per entry (seg_start / c_txn / erank / epre of q and of
// both neighbours): 1.36 GB fetched per C3 launch for 4M entries.
// (tlq != nullptr: the txn-in-block index per chain position from k_bl_chain_block_tb; else erank[c_txn[q]] - tb[b])
static __global__ __launch_bounds__(256) void k_bl_records(size_t P, const uint32_t* __restrict__ blk, const uint32_t* __restrict__ inv,
                                                    const uint32_t* __restrict__ c_txn, const uint8_t* __restrict__ c_meta,
                                                    const int32_t* __restrict__ seg_start, const uint32_t* __restrict__ erank,
                                                    const uint32_t* __restrict__ tb, const uint32_t* __restrict__ boff,
                                                    uint64_t* __restrict__ rec, uint32_t* __restrict__ bad,
                                                    const uint32_t* __restrict__ tlq = nullptr) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool b_ = false;
    if (q < P) {
        const uint32_t b = blk[q];
        const uint32_t key = (uint32_t)seg_start[q];
        const uint32_t j = inv[q];
        const bool first_of_key = q == key;
        const bool next_same_key = q + 1 < P && (uint32_t)seg_start[q + 1] == key;
        const uint32_t bprev = first_of_key ? 0u : blk[q - 1];
        const uint32_t bnext = next_same_key ? blk[q + 1] : 0u;
        const bool head = first_of_key || bprev != b;
        const bool last = !next_same_key || bnext != b;
        const uint32_t tl = tlq ? tlq[q] : erank[c_txn[q]] - tb[b];
        b_ = tl > BL_TL || j - boff[b] >= (uint32_t)BL_CAP;
        uint64_t fl = (uint64_t)(tl & BL_TL) | ((uint64_t)(meta_kind(c_meta[q]) == AD_KIND_WRITE) << BL_SH_W) |
                      ((uint64_t)head << BL_SH_HEAD) | ((uint64_t)last << BL_SH_LAST);
        if (last && next_same_key) fl |= 1ull << (bnext >= b + 3 ? BL_SH_G : BL_SH_R);
        uint32_t lo = 0;
        if (head && !first_of_key) {                                // the key's previous run
            if (b - bprev <= 2) {
                const uint32_t ps = inv[q - 1] - boff[bprev];
                fl |= (1ull << BL_SH_SRC) | ((uint64_t)((bprev % 3) * BL_CAP + ps) << BL_SH_RING);
            } else {
                fl |= 2ull << BL_SH_SRC;
                lo = inv[q - 1];
            }
        }
        rec[j] = (uint64_t)lo | (fl << 32);
    }
    wave_set_flag(b_, bad);
}

// ---- the multi-entry key runs of a block, compacted once per block (all blocks in parallel) ----
// Along one key run the Read/Write rule splits into write epochs: a Write W_{k+1} closes epoch k (W_k and the
// Reads after it), and its level is X_{k+1} = max(X_k + d_k, b_k) with d_k = 1 + [epoch k has Reads] and
// b_k = max(a(W_{k+1}), 1 + the greatest a of epoch k's Reads); a Read of epoch k gets max(a, X_k + 1).  The
// carry (y0, w0) of the run's head is epoch 0 (X_0 = w0, y0 taken as one more Read value of epoch 0).  With D
// the prefix sum of d over the block's Writes this unrolls to X(p) = D(p) + max over the run's epochs so far of
// z, z = b - D(W) (and w0 - D before the head): two max scans of one packed word per entry (segment id in the
// high bits, so a plain unsigned max restarts at every epoch / run) instead of a scan of 2x2 max-plus maps.
// d, D, the epoch and run ids are static per block: k_bl_compact computes them before the walk.
// crec (uint4 per multi-entry run entry, at boff[b] + c for the c-th one of block b, block slot order):
//   x  txn slot in block (11) | Write << 11 | HEAD << 12 | LAST << 13 | G << 14 | SRC << 15 (2) | D << 17 (12)
//      | NLE << 29 (a raise of its txn needs another round)
//   y  epoch id (11) | run id << 11 (11) | block slot << 22 (10)          (ids count from 1 inside the block)
//   z  carry position of the head's source (SRC 2)      w  LDS ring index of the head's carry source (SRC 1)
constexpr int BC_DS = 17, BC_NLE = 29;
struct BlPackSum {                            // rn (11) | ep << 11 (11) | d << 22 (12) | cnt << 34 (11)
    using S = unsigned long long;
    __device__ S identity() const { return 0ull; }
    __device__ S combine(S a, S b) const { return a + b; }
};
struct BlSum32 {
    using S = uint32_t;
    __device__ S identity() const { return 0u; }
    __device__ S combine(S a, S b) const { return a + b; }
};
static __global__ __launch_bounds__(BL_T) void k_bl_compact(uint32_t B, const uint32_t* __restrict__ boff, const uint64_t* __restrict__ rec,
                                                     uint4* __restrict__ crec, uint32_t* __restrict__ mt,
                                                     uint64_t* __restrict__ la, uint32_t* __restrict__ lb,
                                                     uint32_t* __restrict__ lcnt) {
    __shared__ unsigned long long sred[BL_T / WAVE];
    __shared__ uint32_t sred2[BL_T / WAVE];
    __shared__ uint32_t ncnt[BL_CAP];          // per txn of the block: its non-LAST entries
    const uint32_t b = blockIdx.x;
    if (b >= B) return;
    const uint32_t j0 = boff[b], j1 = boff[b + 1];
    const int tid = threadIdx.x;
    for (int x = tid; x < BL_CAP; x += BL_T) ncnt[x] = 0u;
    __syncthreads();
    uint32_t fl[BL_EPT], fa[BL_EPT], lc = 0;
    unsigned long long v[BL_EPT], tot = 0;
#pragma unroll
    for (int e = 0; e < BL_EPT; ++e) {
        const uint32_t j = j0 + (uint32_t)(tid * BL_EPT + e);
        fl[e] = BL_NONE;
        fa[e] = 0u;
        v[e] = 0;
        if (j >= j1) continue;
        const uint32_t f = (uint32_t)(rec[j] >> 32);
        const bool head = f & (1u << BL_SH_HEAD), last = f & (1u << BL_SH_LAST), w = f & (1u << BL_SH_W);
        if (!last) atomicAdd(&ncnt[f & BL_TL], 1u);
        if (head && last) {                                          // a singleton run: not compacted; lists
            fa[e] = (((f >> BL_SH_SRC) & 3u) == 1u ? 1u : 0u) | (((f >> BL_SH_R) & 1u) ? 1u << 16 : 0u);
            lc += fa[e];
            continue;
        }
        fl[e] = f;
        uint32_t d = 0;
        if (w) d = head ? 1u : (((uint32_t)(rec[j - 1] >> 32) & (1u << BL_SH_W)) ? 1u : 2u);
        v[e] = (unsigned long long)(head ? 1u : 0u) | ((unsigned long long)((w || head) ? 1u : 0u) << 11) |
               ((unsigned long long)d << 22) | (1ull << 34);
        tot += v[e];
    }
    unsigned long long total;
    unsigned long long run = block_exclusive_scan<BlPackSum, BL_T>(BlPackSum{}, tot, sred, &total);
    uint32_t ltot;
    uint32_t lpos = block_exclusive_scan<BlSum32, BL_T>(BlSum32{}, lc, sred2, &ltot);   // (its barriers also
                                                                                       // order ncnt)
#pragma unroll
    for (int e = 0; e < BL_EPT; ++e) {
        const uint32_t j = j0 + (uint32_t)(tid * BL_EPT + e);
        if (fa[e]) {                                                 // ring-sourced / ring-continuing singleton
            const uint32_t f = (uint32_t)(rec[j] >> 32), tl = f & BL_TL, w = (f >> BL_SH_W) & 1u, x = j - j0;
            if (fa[e] & 1u)
                la[j0 + (lpos & 0xFFFFu)] =
                    (uint64_t)(((f >> BL_SH_RING) & 0xFFFu) | (w << 12) | (tl << 13)) | ((uint64_t)x << 32);
            if (fa[e] >> 16) lb[j0 + (lpos >> 16)] = x | (tl << 10) | (w << 21);
            lpos += fa[e];
        }
        if (fl[e] == BL_NONE) continue;
        run += v[e];
        const uint32_t rn = (uint32_t)(run & 0x7FFu), ep = (uint32_t)((run >> 11) & 0x7FFu);
        const uint32_t ds = (uint32_t)((run >> 22) & 0xFFFu), c = (uint32_t)(run >> 34) - 1u;
        const uint32_t key = (uint32_t)rec[j];
        // NLE: a raise of this entry's txn needs another round only if the txn has a non-LAST entry other than
        // this one (a run's scan already carries its own entries' levels forward; a LAST entry feeds only the
        // carry-out, taken from the final levels)
        const uint32_t nle = ncnt[fl[e] & BL_TL] > (((fl[e] >> BL_SH_LAST) & 1u) ? 0u : 1u) ? 1u : 0u;
        crec[j0 + c] = make_uint4((fl[e] & 0x1FFFFu) | (ds << BC_DS) | (nle << BC_NLE),
                                  ep | (rn << 11) | ((j - j0) << 22), key, (fl[e] >> BL_SH_RING) & 0xFFFu);
    }
    if (tid == 0) { mt[b] = (uint32_t)(total >> 34); lcnt[b] = ltot; }
}

// w ? a : b on values (a ternary over the members of an int2 held in a register array was compiled into a pointer
// select and a scratch round trip per slot)
__device__ inline int bl_sel(bool w, int a, int b) { return b + ((a - b) & -(int)w); }
// a global carry (y, w) moves as one 8-byte word: one memory transaction per carry instead of two
__device__ inline void bl_carry_store(int2* carry, uint32_t slot, int2 c) {
    const uint64_t v = (uint64_t)(uint32_t)c.x | ((uint64_t)(uint32_t)c.y << 32);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(&carry[slot]), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Phase clocks of the walk (AD_DEBUG_LEVELS prints them) only in AD_BL_TIMERS builds: a clock read waits for the
// wave's outstanding LDS operations, which the timed code would otherwise overlap.
__device__ inline uint64_t bl_clk() {
#ifdef AD_BL_TIMERS
    return clock64();
#else
    return 0;
#endif
}

// Packed scan words: segment id in the high bits, value + BZ_BIAS in the low bits (u32: values < 2^20, i.e.
// batches of <= 2^20 txns; u64 otherwise).  The word 0 is below every real entry's (ids count from 1).
constexpr int BZ_BIAS = 1 << 12;
template <class PK> __device__ constexpr int bz_sh() { return sizeof(PK) == 4 ? 21 : 32; }
template <class PK> __device__ inline PK bz_pack(uint32_t seg, int v) {
    return ((PK)seg << bz_sh<PK>()) | (PK)(uint32_t)(v + BZ_BIAS);
}
template <class PK> __device__ inline int bz_val(PK p) {
    return (int)(uint32_t)(p & (((PK)1 << bz_sh<PK>()) - 1)) - BZ_BIAS;
}
template <class PK> __device__ inline PK bz_max(PK a, PK b) { return a > b ? a : b; }
template <class PK>
struct BzMax {
    using S = PK;
    __device__ S identity() const { return (PK)0; }
    __device__ S combine(S a, S b) const { return a > b ? a : b; }
};

// Jacobi rounds over the block's compacted multi-entry runs by ONE wave, E consecutive entries per lane: per
// round the two packed max scans above give every entry's level candidate x; x > a raises the txn (LDS
// atomicMax).  Until no raise flagged NLE happens.  Absent entries (beyond nm) read and raise the
// lane's sink slot past BL_CAP.  A head whose carry comes from the ring (-2, ring index) reads it first (this
// wave wrote it one or two blocks earlier).  Then the carry-out of every LAST entry -- y' = max(y0, the levels
// of the run's txns), w' = max(w0, the levels of its Writes) -- into the ring.  Returns the rounds.
template <int E, class PK>
__device__ inline uint32_t bl_rounds(int nm, const uint4* __restrict__ cr, const int2* __restrict__ hc, int* lv,
                                     int2* ring, int rb, uint32_t* stuck, uint64_t* tph) {
    const uint64_t tq0 = bl_clk();
    const int lane = __lane_id();
    uint32_t slot[E], ds[E], ep[E], rn[E], bs[E];
    bool wr[E], hd[E], lst[E], nle[E];
    int y0[E], w0[E], a[E];
    int2 h[E];
    // all reads unconditional (k < BL_CAP: inside the arrays; absent entries masked after): a conditional LDS
    // read merged with a constant at a branch join is waited for per entry
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int k = lane * E + e;
        const bool v = k < nm;
        uint4 c = cr[k];
        const int2 hk = hc[k];
        if (!v) c = make_uint4(0u, 0u, 0u, 0u);
        slot[e] = v ? (c.x & BL_TL) : (uint32_t)(BL_CAP + lane);
        bs[e] = c.y >> 22;
        wr[e] = (c.x >> BL_SH_W) & 1u;
        hd[e] = (c.x >> BL_SH_HEAD) & 1u;
        lst[e] = (c.x >> BL_SH_LAST) & 1u;
        ds[e] = (c.x >> BC_DS) & 0xFFFu;
        ep[e] = c.y & 0x7FFu;
        rn[e] = (c.y >> 11) & 0x7FFu;
        h[e] = hd[e] ? hk : make_int2(-1, -1);
        nle[e] = (c.x >> BC_NLE) & 1u;                   // static (k_bl_compact)
    }
    bool fr[E];                                             // carry from the ring
    int2 hr[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        fr[e] = h[e].x == -2;
        hr[e] = ring[fr[e] ? h[e].y : 0];
    }
#pragma unroll
    for (int e = 0; e < E; ++e) h[e] = fr[e] ? hr[e] : h[e];   // used on every path: the reads stay unconditional
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int lb = bl_sel(wr[e], h[e].x, h[e].y) + 1;
        if (fr[e] && lb > 0) atomicMax(&lv[slot[e]], lb);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) { y0[e] = h[e].x; w0[e] = h[e].y; }
    // The per-entry words of the two scans and the level candidate, folded into static constants so that a
    // round costs one add + one max per scan input (all words are unsigned; every real word of epoch / run s
    // is >= s << SH >= 2^SH, every level < 2^SH, so a constant 0 or a bare level never wins over one):
    //   scan 1  rv = max(a + c1, c2)                 Write: c1 = 0, c2 = (ep); Read: c1 = (ep) + BIAS,
    //                                                c2 = head ? (ep) + BIAS + y0 : 0
    //   scan 2  zv = max(a + cA, (prev & M) + cB, cC)  = pack(rn, z) for Writes and heads; a value < 2^SH
    //                                                (below the run's head word, which precedes it) for the
    //                                                other Reads, whose z is unused
    //   level   x  = max((zm & M) + c7, a + ka)      Write: X; Read: max(a, X + 1)
    constexpr int SH = bz_sh<PK>();
    constexpr PK M = ((PK)1 << SH) - 1;
    PK c1[E], c2[E], cA[E], cB[E], cC[E];
    int c7[E], ka[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const PK se = (PK)ep[e] << SH, sr = (PK)rn[e] << SH;
        const int d = (int)ds[e];
        c1[e] = wr[e] ? (PK)0 : se + (PK)BZ_BIAS;
        c2[e] = wr[e] ? se : (hd[e] ? se + (PK)(BZ_BIAS + y0[e]) : (PK)0);
        cA[e] = wr[e] ? sr + (PK)(BZ_BIAS - d) : (PK)0;
        cB[e] = (wr[e] && !hd[e]) ? sr + (PK)(int64_t)(1 - d) : (PK)0;
        cC[e] = !hd[e] ? (PK)0
                       : sr + (PK)(BZ_BIAS + (wr[e] ? max(w0[e] - d + 1, y0[e] + 1 - d) : w0[e] - d));
        c7[e] = d - BZ_BIAS + (wr[e] ? 0 : 1);
        ka[e] = wr[e] ? -(1 << 30) : 0;
    }
    const BzMax<PK> op{};
    uint32_t it = 0;
    const uint64_t tq1 = bl_clk();
    tph[0] += tq1 - tq0;
    while (true) {
#pragma unroll
        for (int e = 0; e < E; ++e) a[e] = lv[slot[e]];
        // scan 1: Read values by epoch (a Write opens its epoch with the bare segment word)
        PK r1 = 0, pre1[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            pre1[e] = r1;
            r1 = bz_max(r1, bz_max((PK)(uint32_t)a[e] + c1[e], c2[e]));
        }
        const PK in1 = wave_shift_up1(op, wave_incl_scan(op, r1));
        // scan 2: z by run
        PK r2 = 0, inc2[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const PK prev = bz_max(in1, pre1[e]);                  // the previous epoch's greatest Read value
            const PK zv = bz_max(bz_max((PK)(uint32_t)a[e] + cA[e], (prev & M) + cB[e]), cC[e]);
            r2 = bz_max(r2, zv);
            inc2[e] = r2;
        }
        const PK in2 = wave_shift_up1(op, wave_incl_scan(op, r2));
        bool up = false;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const PK zm = bz_max(in2, inc2[e]);
            const int x = max((int)(uint32_t)(zm & M) + c7[e], a[e] + ka[e]);
            const bool r = x > a[e];
            atomicMax(&lv[slot[e]], x);                      // unconditional: no exec-mask dance (x <= a: no-op)
            up |= r && nle[e];
        }
        // (no wait for the raises: a wave's LDS operations complete in order, so the next round's reads see them)
        ++it;
        if (!__ballot(up)) break;
        // each round finalises at least the lowest unfinished txn of the block: more rounds than txns + 1 is
        // a broken invariant; stop (the host reports it) instead of spinning
        if (it > (uint32_t)BL_CAP + 1) { *stuck = 1u; break; }
    }
    const uint64_t tq2 = bl_clk();
    // carry-out of the runs
    PK ry = 0, rw = 0, iy[E], iw[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int x = lv[slot[e]];
        const int vy = hd[e] ? max(x, y0[e]) : x;
        const int vw = wr[e] ? (hd[e] ? max(x, w0[e]) : x) : (hd[e] ? w0[e] : -BZ_BIAS);
        const PK py = bz_pack<PK>(rn[e], vy), pw = bz_pack<PK>(rn[e], vw);
        ry = ry > py ? ry : py;
        rw = rw > pw ? rw : pw;
        iy[e] = ry; iw[e] = rw;
    }
    const PK iny = wave_shift_up1(op, wave_incl_scan(op, ry));
    const PK inw = wave_shift_up1(op, wave_incl_scan(op, rw));
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int k = lane * E + e;
        if (k >= nm || !lst[e]) continue;
        const PK my = iny > iy[e] ? iny : iy[e], mw = inw > iw[e] ? inw : iw[e];
        ring[rb + (int)bs[e]] = make_int2(bz_val<PK>(my), bz_val<PK>(mw));
    }
    tph[1] += bl_clk() - tq2;
    return it;
}

// The sequential walk over the blocks (one workgroup; see the file header).  Only wave 0 (W0) is on the
// sequential path, and it touches LDS only; waves 1-3 (the workers) do all global memory traffic one block
// ahead / one block behind.  Per block b, ONE phase R_b:
//   W0       the singleton runs of b whose carry comes from the ring (list la: their key's previous run ended
//            one or two blocks earlier) -> carry-in, txn lower bound; the rounds of b's multi-entry runs and
//            their carry-outs into the ring; the carry-outs of b's singleton runs whose key continues one or two
//            blocks later (list lb) into the ring.
//   workers  issue block b + 1's global carry-ins (its records were loaded one phase earlier) and block b + 2's
//            static loads (records, compacted entries); meanwhile retire block b - 1: its levels into Lr (by
//            executeAt rank: coalesced) and its carry-outs for keys continuing >= 3 blocks later into global
//            memory (the "G" carries, at the producer's own position: inside the block's window); clear the
//            buffers block b + 2 will use; stage block b + 1, prefill its txn levels from every head whose carry
//            is known (a singleton run is then final), count its non-last entries per txn, build its la / lb
//            lists; release their global stores.
// Levels / flags / bounds / list counts live in four buffers by b % 4 (W0's b, the workers' b - 1, b + 1 and the
// cleared b + 2); staged block data in two by b % 2: a worker reads block b - 1's slot x and then overwrites it
// with block b + 1's, and the two use the same slot -> thread mapping, so no barrier is needed between them.
// A G carry stored while block b - 1 is retired (R_b) is read by the staging of block >= b + 2 (R_{b+1} or
// later), after the workers' release fence and the barrier that ends R_b.
// stats[0] = greatest level + 1, stats[1] = rounds, stats[2..3] = clock64 in rounds, stats[4..5] = total,
// stats[6] = a block's rounds did not converge, stats[7] = clock64 / 256 W0 waited for the workers,
// stats[8] = W0's list work, stats[9] = the workers' work (thread WAVE), stats[10..12] = its retire, clear and
// staging parts.
// The walk's workgroup: 256 threads (W0 + 3 worker waves, one per SIMD) or 512 (W0's SIMD partner, wave 4, idles
// so that W0 keeps its SIMD's issue slots; 6 worker waves, two per SIMD, hide each other's latencies).
#ifndef AD_BL_WT
#define AD_BL_WT 512
#endif
constexpr int BL_WT = AD_BL_WT;
constexpr int BL_NW = BL_WT == 512 ? BL_WT - 2 * WAVE : BL_WT - WAVE;   // worker threads
constexpr int BL_SI = (BL_CAP + BL_NW - 1) / BL_NW;                       // slots per worker thread
// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits for the wave's outstanding global stores
// (s_waitcnt vmcnt(0)); the workers release their global stores themselves (end of their phase).
__device__ inline void bl_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct BlStage {                               // one block's staged data in LDS (two of these, by block parity)
    uint64_t rec[BL_CAP];                      // slot records (~0: none)
    int2 car[BL_CAP];                          // singleton runs' carry-in (ring-sourced ones: written by W0)
    uint4 cr[BL_CAP];                          // compacted multi-entry run entries
    int2 hc[BL_CAP];                           // their heads' carry-in ((-2, ring index): W0 reads the ring)
    uint64_t la[BL_CAP];                       // ring-sourced singleton runs: ring | W << 12 | txn << 13 | slot << 32
    uint32_t lb[BL_CAP];                       // ring-continuing singleton runs: slot | txn << 10 | W << 21
};
struct BlBounds { uint32_t j0, j1, t0, t1, m, cnt; };   // cnt: la entries | lb entries << 16

// A block's static inputs in a worker's registers (loaded two blocks ahead: they do not depend on the walk).
struct BlPre {
    uint32_t j0, j1, t0, t1, m, l;
    uint64_t r[BL_SI];                         // slot records (~0: none)
    uint4 q[BL_SI];                            // compacted entries
    uint64_t a[BL_SI];                         // la list entries (k_bl_compact)
    uint32_t b[BL_SI];                         // lb list entries
};
struct BlBnd { uint32_t j0, j1, t0, t1, m, l; };
// A block's bounds, one phase before its static loads need them, by vector loads: a scalar load shares its
// wait counter with LDS operations, so the phase's first LDS wait would stall for it.
__device__ inline BlBnd bl_load_bounds(uint32_t b, const uint32_t* boff, const uint32_t* tb, const uint32_t* mt,
                                     const uint32_t* lcnt) {
    auto ld = [](const uint32_t* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
    return BlBnd{ld(boff + b), ld(boff + b + 1), ld(tb + b), ld(tb + b + 1), ld(mt + b), ld(lcnt + b)};
}
__device__ inline void bl_load_static(const BlBnd& bn, int t, int nthr, const uint64_t* __restrict__ rec,
                                      const uint4* __restrict__ crec, const uint64_t* __restrict__ la,
                                      const uint32_t* __restrict__ lb, BlPre& p) {
    p.j0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bn.j0);
    p.j1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bn.j1);
    p.t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bn.t0);
    p.t1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bn.t1);
    p.m = (uint32_t)__builtin_amdgcn_readfirstlane((int)bn.m);
    p.l = (uint32_t)__builtin_amdgcn_readfirstlane((int)bn.l);
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const uint32_t x = (uint32_t)(t + i * nthr);
        p.r[i] = (x < (uint32_t)BL_CAP && p.j0 + x < p.j1) ? rec[p.j0 + x] : ~0ull;
        p.q[i] = x < p.m ? crec[p.j0 + x] : make_uint4(0u, 0u, 0u, 0u);
        p.a[i] = x < (p.l & 0xFFFFu) ? la[p.j0 + x] : 0ull;
        p.b[i] = x < (p.l >> 16) ? lb[p.j0 + x] : 0u;
    }
}
// The block's carry-ins from global memory (keys whose previous run ended >= 3 blocks earlier; released by the
// retiring workers before an earlier barrier) and the ring references of its compacted heads.
// Every lane loads (position 0 when it has no carry to fetch) and the words are decoded only in bl_stage_write:
// a conditional load merged with a constant at the branch join made the compiler wait for each load before the
// next (one memory latency per slot instead of one for all).
__device__ inline bool bl_wants_c(const BlPre& p, int i) {
    const uint32_t f = (uint32_t)(p.r[i] >> 32);
    return p.r[i] != ~0ull && (f & (1u << BL_SH_HEAD)) && (f & (1u << BL_SH_LAST)) && ((f >> BL_SH_SRC) & 3u) == 2u;
}
__device__ inline bool bl_wants_h(const BlPre& p, int i, uint32_t x) {
    return x < p.m && ((p.q[i].x >> BL_SH_HEAD) & 1u) && ((p.q[i].x >> BL_SH_SRC) & 3u) == 2u;
}
__device__ inline void bl_load_carries(int t, int nthr, const BlPre& p, const int2* carry, uint64_t* vc, uint64_t* vh) {
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const uint32_t x = (uint32_t)(t + i * nthr);
        const uint32_t ac = bl_wants_c(p, i) ? (uint32_t)p.r[i] : 0u, ah = bl_wants_h(p, i, x) ? p.q[i].z : 0u;
        vc[i] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(&carry[ac]), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
        vh[i] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(&carry[ah]), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
__device__ inline int2 bl_unpack(uint64_t v) { return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32)); }
// Stage the block into `s` and prefill its levels (lv: its buffer) from every head whose carry is known now; copy
// its la / lb lists (built by k_bl_compact).
__device__ inline void bl_stage_write(int t, int nthr, const BlPre& p, const uint64_t* vc, const uint64_t* vh,
                                      BlStage& s, BlBounds& bd, int* lv) {
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const uint32_t x = (uint32_t)(t + i * nthr);
        if (x >= (uint32_t)BL_CAP) continue;
        const uint64_t r = p.r[i];
        const uint32_t f = (uint32_t)(r >> 32);
        const int2 c = bl_wants_c(p, i) ? bl_unpack(vc[i]) : make_int2(-1, -1);
        s.rec[x] = r;
        s.car[x] = c;
        // a singleton run whose carry is known now: its txn's lower bound (ring-sourced ones: W0, list la)
        if (r != ~0ull && (f & (1u << BL_SH_HEAD)) && (f & (1u << BL_SH_LAST)) && ((f >> BL_SH_SRC) & 3u) != 1u) {
            const int lb = bl_sel(f & (1u << BL_SH_W), c.x, c.y) + 1;
            if (lb > 0) atomicMax(&lv[f & BL_TL], lb);
        }
        if (x < p.m) {
            const uint4 q = p.q[i];
            const bool h1 = ((q.x >> BL_SH_HEAD) & 1u) && ((q.x >> BL_SH_SRC) & 3u) == 1u;
            const int2 h = bl_wants_h(p, i, x) ? bl_unpack(vh[i]) : (h1 ? make_int2(-2, (int)q.w) : make_int2(-1, -1));
            s.cr[x] = q;
            s.hc[x] = h;
            if (((q.x >> BL_SH_HEAD) & 1u) && !h1) {
                const int lb = bl_sel((q.x >> BL_SH_W) & 1u, h.x, h.y) + 1;
                if (lb > 0) atomicMax(&lv[q.x & BL_TL], lb);
            }
        }
        if (x < (p.l & 0xFFFFu)) s.la[x] = p.a[i];
        if (x < (p.l >> 16)) s.lb[x] = p.b[i];
    }
    if (t == 0) { bd.j0 = p.j0; bd.j1 = p.j1; bd.t0 = p.t0; bd.t1 = p.t1; bd.m = p.m; bd.cnt = p.l; }
}

// Retire block b (workers, the same slot -> thread mapping as bl_stage_write): its levels into Lr (by executeAt
// rank; k_bl_scatter moves them to txn order after the walk) and the
// carries of keys continuing >= 3 blocks later into global memory (a singleton run's from its carry-in and its
// txn's level; a multi-entry run's from the ring, where W0 left it).  Returns the greatest level seen.
__device__ inline int bl_retire(int t, int nthr, const BlStage& s, const BlBounds& bd, const int* lv, const int2* ring,
                                int rb, int2* carry, uint32_t* __restrict__ Lr) {
    const uint32_t nt = bd.t1 - bd.t0;
    uint64_t rr[BL_SI];
    int2 ci[BL_SI];
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const int x = t + i * nthr;
        rr[i] = x < BL_CAP ? s.rec[x] : ~0ull;
        ci[i] = x < BL_CAP ? s.car[x] : make_int2(-1, -1);
    }
    int ls[BL_SI], lo[BL_SI];
    int2 rg[BL_SI];
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const int x = t + i * nthr;
        const uint32_t f = (uint32_t)(rr[i] >> 32);
        // unconditional reads (safe indexes): a conditional read merged at a branch join is waited for per slot
        const bool g = rr[i] != ~0ull && (f & (1u << BL_SH_G));
        const bool single = (f & (1u << BL_SH_HEAD)) != 0;     // a G entry is LAST: HEAD too = singleton run
        ls[i] = lv[g && single ? (f & BL_TL) : 0u];
        rg[i] = ring[rb + (x < BL_CAP ? x : 0)];
        lo[i] = lv[(uint32_t)x < nt ? x : 0];
    }
    int maxl = -1;
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const int x = t + i * nthr;
        const uint32_t f = (uint32_t)(rr[i] >> 32);
        if (rr[i] != ~0ull && (f & (1u << BL_SH_G))) {
            const int2 c = (f & (1u << BL_SH_HEAD))
                               ? make_int2(max(ci[i].x, ls[i]), bl_sel(f & (1u << BL_SH_W), ls[i], ci[i].y))
                               : rg[i];
            bl_carry_store(carry, bd.j0 + (uint32_t)x, c);
        }
        if ((uint32_t)x < nt) {
            Lr[bd.t0 + (uint32_t)x] = (uint32_t)lo[i];             // executeAt-rank order: coalesced
            maxl = max(maxl, lo[i]);
        }
    }
    return maxl;
}

template <class PK>
static __global__ __launch_bounds__(BL_WT) void k_level_blocks(uint32_t B, const uint32_t* __restrict__ boff, const uint32_t* __restrict__ tb,
                                                       const uint64_t* __restrict__ rec, const uint4* __restrict__ crec,
                                                       const uint32_t* __restrict__ mt, const uint64_t* __restrict__ la,
                                                       const uint32_t* __restrict__ lb, const uint32_t* __restrict__ lcnt,
                                                       int2* carry,
                                                       uint32_t* __restrict__ Lr,
                                                       uint32_t* __restrict__ stats) {
    __shared__ __align__(16) int lvb[4][BL_CAP + WAVE];     // levels of a block's txns (txn-in-block index), by
                                                            // block % 4; [BL_CAP + lane]: the rounds' sinks
    __shared__ int2 ring[3 * BL_CAP];          // carry-out of the slots of the last three blocks (by block % 3)
    __shared__ BlStage stg[2];
    __shared__ BlBounds bnd[4];
    __shared__ uint32_t sstuck;
    static_assert((BL_CAP + WAVE) % 16 == 0, "buffers are cleared 16 bytes at a time");
    const int tid = threadIdx.x, lane = __lane_id();
    if (tid == 0) sstuck = 0u;
    const uint64_t tstart = clock64();
    uint64_t tround = 0, twait = 0, tlist = 0, twork = 0, tret = 0, tclr = 0, tstg = 0, tph[2] = {0, 0}, sepl = 0;
    for (int x = tid; x < BL_CAP + WAVE; x += BL_WT) {
#pragma unroll
        for (int k = 0; k < 4; ++k) lvb[k][x] = 0;
    }
    __syncthreads();
    int maxl = -1;
    uint32_t rounds = 0;
    if (B > 0) {                               // block 0: staged by every thread
        BlPre p0;
        uint64_t vc[BL_SI], vh[BL_SI];
        bl_load_static(bl_load_bounds(0, boff, tb, mt, lcnt), tid, BL_WT, rec, crec, la, lb, p0);
        bl_load_carries(tid, BL_WT, p0, carry, vc, vh);
        bl_stage_write(tid, BL_WT, p0, vc, vh, stg[0], bnd[0], lvb[0]);
    }
    __syncthreads();
    // Each role runs its own loop (one barrier per block in both), so the workers' registers carried across
    // blocks do not add to wave 0's register pressure in the rounds.
    if (tid < WAVE) {
        for (uint32_t b = 0; b < B; ++b) {
            const uint64_t tb0 = bl_clk();
            BlStage& S = stg[b & 1];
            int* lv = lvb[b & 3];
            const int rb = (int)(b % 3) * BL_CAP;
            const uint32_t cnt = bnd[b & 3].cnt, na = cnt & 0xFFFFu, nbl = cnt >> 16;
            const int nm = (int)bnd[b & 3].m;
            // ring-sourced singleton runs: carry-in and txn lower bound
            for (uint32_t k = lane; k < na; k += WAVE) {
                const uint64_t e = S.la[k];
                const int2 c = ring[(uint32_t)e & 0xFFFu];
                S.car[(uint32_t)(e >> 32)] = c;
                const int lb = bl_sel(((uint32_t)e >> 12) & 1u, c.x, c.y) + 1;
                if (lb > 0) atomicMax(&lv[((uint32_t)e >> 13) & BL_TL], lb);
            }
            const uint64_t t1 = bl_clk();
            if (nm > 0) {
                uint32_t r;
                const int epl = (nm + WAVE - 1) / WAVE;        // entries per lane
                sepl += (uint64_t)epl;
                if (epl <= 2) r = bl_rounds<2, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                else if (epl <= 3) r = bl_rounds<3, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                else if (epl <= 4) r = bl_rounds<4, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                else if (epl <= 5) r = bl_rounds<5, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                else if (epl <= 6) r = bl_rounds<6, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                else if (epl <= 8) r = bl_rounds<8, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                else if (epl <= 12) r = bl_rounds<12, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                else r = bl_rounds<16, PK>(nm, S.cr, S.hc, lv, ring, rb, &sstuck, tph);
                rounds += r;
            }
            const uint64_t t2 = bl_clk();
            tround += t2 - t1;
            // ring-continuing singleton runs: carry-out (the txn's level is final now)
            for (uint32_t k = lane; k < nbl; k += WAVE) {
                const uint32_t e = S.lb[k];
                const uint32_t x = e & 0x3FFu;
                const int2 ci = S.car[x];
                const int l = lv[(e >> 10) & BL_TL];
                ring[rb + (int)x] = make_int2(max(ci.x, l), bl_sel((e >> 21) & 1u, l, ci.y));
            }
            const uint64_t t3 = bl_clk();
            tlist += (t1 - tb0) + (t3 - t2);
            bl_barrier();
            twait += bl_clk() - t3;
            if (sstuck) break;
        }
    } else if (BL_WT == 512 && tid / WAVE == 4) {
        for (uint32_t b = 0; b < B; ++b) {     // W0's SIMD partner: barriers only
            bl_barrier();
            if (sstuck) break;
        }
    } else {
        const int w = tid / WAVE;
        const int t = (BL_WT == 512 && w > 4 ? tid - 2 * WAVE : tid - WAVE), nthr = BL_NW;
        BlPre cur, nxt;                        // static inputs of blocks b + 1 and b + 2
        BlBnd bn{};                            // bounds of block b + 2
        if (B > 1) bl_load_static(bl_load_bounds(1, boff, tb, mt, lcnt), t, nthr, rec, crec, la, lb, cur);
        if (B > 2) bn = bl_load_bounds(2, boff, tb, mt, lcnt);
        for (uint32_t b = 0; b < B; ++b) {
            const uint64_t tb0 = bl_clk();
            // issue first: block b + 1's global carry-ins and block b + 2's static loads; retire block b - 1 and
            // clear block b + 2's buffers while they are in flight
            uint64_t vc[BL_SI], vh[BL_SI];
            if (b + 1 < B) bl_load_carries(t, nthr, cur, carry, vc, vh);
            if (b + 2 < B) bl_load_static(bn, t, nthr, rec, crec, la, lb, nxt);
            if (b + 3 < B) bn = bl_load_bounds(b + 3, boff, tb, mt, lcnt);
            const uint64_t tw1 = bl_clk();
            if (b > 0) {
                const uint32_t p = b - 1;
                maxl = max(maxl, bl_retire(t, nthr, stg[p & 1], bnd[p & 3], lvb[p & 3], ring, (int)(p % 3) * BL_CAP,
                                           carry, Lr));
            }
            const uint64_t tw2 = bl_clk();
            {   // the buffers of block b + 2 (last used by block b - 2, retired in the previous phase)
                int4* lc = reinterpret_cast<int4*>(lvb[(b + 2) & 3]);
                for (int x = t; x < (BL_CAP + WAVE) / 4; x += nthr) lc[x] = make_int4(0, 0, 0, 0);
            }
            const uint64_t tw3 = bl_clk();
            if (b + 1 < B) bl_stage_write(t, nthr, cur, vc, vh, stg[(b + 1) & 1], bnd[(b + 1) & 3], lvb[(b + 1) & 3]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");    // the retired block's G carries
            const uint64_t tw4 = bl_clk();
            twork += tw4 - tb0;
            tret += tw2 - tw1;
            tclr += tw3 - tw2;
            tstg += tw4 - tw3;
            bl_barrier();
            if (sstuck) break;
            cur = nxt;
        }
        if (B > 0 && !sstuck) {
            const uint32_t p = B - 1;
            maxl = max(maxl, bl_retire(t, nthr, stg[p & 1], bnd[p & 3], lvb[p & 3], ring, (int)(p % 3) * BL_CAP,
                                       carry, Lr));
        }
    }
    maxl = wave_max(maxl);
    if (lane == 0) atomicMax(&stats[0], (uint32_t)(maxl + 1));
    if (tid == 0) {
        stats[1] = rounds;
        const uint64_t tot = clock64() - tstart;
        stats[2] = (uint32_t)tround; stats[3] = (uint32_t)(tround >> 32);
        stats[4] = (uint32_t)tot; stats[5] = (uint32_t)(tot >> 32);
        stats[6] = sstuck;
        stats[7] = (uint32_t)(twait >> 8); stats[8] = (uint32_t)(tlist >> 8);
        stats[13] = (uint32_t)(tph[0] >> 8); stats[14] = (uint32_t)(tph[1] >> 8); stats[15] = (uint32_t)sepl;
    }
    if (tid == WAVE) {
        stats[9] = (uint32_t)(twork >> 8);
        stats[10] = (uint32_t)(tret >> 8); stats[11] = (uint32_t)(tclr >> 8); stats[12] = (uint32_t)(tstg >> 8);
    }
}

// levels from executeAt-rank order (the walk's coalesced output) to txn order
static __global__ __launch_bounds__(256) void k_bl_scatter(size_t n, const uint32_t* __restrict__ order,
                                                    const uint32_t* __restrict__ Lr, uint32_t* __restrict__ L) {
    const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) L[order[k]] = Lr[k];
}

struct BlockBufs {                             // grow-only, owned by LevelState
    uint64_t* rec = nullptr;                   // [P]
    uint32_t *epre = nullptr, *erank = nullptr, *bk = nullptr, *bv = nullptr, *bk2 = nullptr, *bv2 = nullptr;
    uint32_t *tb = nullptr, *boff = nullptr, *stats = nullptr, *rs = nullptr, *mt = nullptr, *lcnt = nullptr;
    uint32_t* tl = nullptr;                    // [P] txn-in-block index per chain position (k_bl_chain_block_tb)
    uint64_t* la = nullptr;                    // [P] per block: ring-sourced singleton runs (k_bl_compact)
    uint32_t* lb = nullptr;                    // [P] per block: ring-continuing singleton runs
    int2* carry = nullptr;
    uint4* crec = nullptr;                     // [P] compacted multi-entry run entries (k_bl_compact)
    size_t capP = 0, capN = 0, capB = 0, rs_cap = 0;
    uint32_t nblocks = 0;                      // blocks of the last run
};

inline void free_block_bufs(BlockBufs& b) {
    void* ps[] = {b.rec, b.epre, b.erank, b.bk, b.bv, b.bk2, b.bv2, b.tb, b.boff, b.stats, b.rs, b.carry, b.crec, b.mt,
                  b.lcnt, b.la, b.lb, b.tl};
    for (void* p : ps) if (p) hipFree(p);
    b = BlockBufs{};
}

}  // namespace ad
