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
//   bit  61     LAST entry whose key continues 1 or 2 blocks later (its carry goes to the LDS ring only)
constexpr int BL_SH_W = 11, BL_SH_HEAD = 12, BL_SH_LAST = 13, BL_SH_G = 14, BL_SH_SRC = 15, BL_SH_RING = 17,
              BL_SH_R = 29;
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
        if (last && q + 1 < P && (uint32_t)seg_start[q + 1] == key)
            fl |= 1ull << (bl_block_of(q + 1, c_txn, erank, epre, bcap) >= b + 3 ? BL_SH_G : BL_SH_R);
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
//   y  epoch id (11) | run id << 11 (11) | block slot << 22 (10)          (ids count from 1 inside the block)
//   z  carry slot (the key's segment head)      w  LDS ring index of the head's carry source (SRC 1)
constexpr int BC_DS = 17;
struct BlPackSum {                            // rn (11) | ep << 11 (11) | d << 22 (12) | cnt << 34 (11)
    using S = unsigned long long;
    __device__ S identity() const { return 0ull; }
    __device__ S combine(S a, S b) const { return a + b; }
};
static __global__ __launch_bounds__(BL_T) void k_bl_compact(uint32_t B, const uint32_t* __restrict__ boff, const uint64_t* __restrict__ rec,
                                                     uint4* __restrict__ crec, uint32_t* __restrict__ mt) {
    __shared__ unsigned long long sred[BL_T / WAVE];
    const uint32_t b = blockIdx.x;
    if (b >= B) return;
    const uint32_t j0 = boff[b], j1 = boff[b + 1];
    const int tid = threadIdx.x;
    uint32_t fl[BL_EPT];
    unsigned long long v[BL_EPT], tot = 0;
#pragma unroll
    for (int e = 0; e < BL_EPT; ++e) {
        const uint32_t j = j0 + (uint32_t)(tid * BL_EPT + e);
        fl[e] = BL_NONE;
        v[e] = 0;
        if (j >= j1) continue;
        const uint32_t f = (uint32_t)(rec[j] >> 32);
        const bool head = f & (1u << BL_SH_HEAD), last = f & (1u << BL_SH_LAST), w = f & (1u << BL_SH_W);
        if (head && last) continue;                                  // a singleton run: not compacted
        fl[e] = f;
        uint32_t d = 0;
        if (w) d = head ? 1u : (((uint32_t)(rec[j - 1] >> 32) & (1u << BL_SH_W)) ? 1u : 2u);
        v[e] = (unsigned long long)(head ? 1u : 0u) | ((unsigned long long)((w || head) ? 1u : 0u) << 11) |
               ((unsigned long long)d << 22) | (1ull << 34);
        tot += v[e];
    }
    unsigned long long total;
    unsigned long long run = block_exclusive_scan<BlPackSum, BL_T>(BlPackSum{}, tot, sred, &total);
#pragma unroll
    for (int e = 0; e < BL_EPT; ++e) {
        if (fl[e] == BL_NONE) continue;
        run += v[e];
        const uint32_t rn = (uint32_t)(run & 0x7FFu), ep = (uint32_t)((run >> 11) & 0x7FFu);
        const uint32_t ds = (uint32_t)((run >> 22) & 0xFFFu), c = (uint32_t)(run >> 34) - 1u;
        const uint32_t j = j0 + (uint32_t)(tid * BL_EPT + e);
        const uint32_t key = (uint32_t)rec[j];
        crec[j0 + c] = make_uint4((fl[e] & 0x1FFFFu) | (ds << BC_DS), ep | (rn << 11) | ((j - j0) << 22), key,
                                  (fl[e] >> BL_SH_RING) & 0xFFFu);
    }
    if (tid == 0) mt[b] = (uint32_t)(total >> 34);
}

// w ? a : b on values (a ternary over the members of an int2 held in a register array was compiled into a pointer
// select and a scratch round trip per slot)
__device__ inline int bl_sel(bool w, int a, int b) { return b + ((a - b) & -(int)w); }
// a key's global carry (y, w) moves as one 8-byte word: one memory transaction per carry instead of two
__device__ inline int2 bl_carry_load(const int2* carry, uint32_t slot) {
    const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(&carry[slot]), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
    return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
}
__device__ inline void bl_carry_store(int2* carry, uint32_t slot, int2 c) {
    const uint64_t v = (uint64_t)(uint32_t)c.x | ((uint64_t)(uint32_t)c.y << 32);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(&carry[slot]), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
template <class PK>
struct BzMax {
    using S = PK;
    __device__ S identity() const { return (PK)0; }
    __device__ S combine(S a, S b) const { return a > b ? a : b; }
};

// Jacobi rounds over the block's compacted multi-entry runs by ONE wave, E consecutive entries per lane: per
// round the two packed max scans above give every entry's level candidate x; x > a raises the txn (LDS
// atomicMax).  Until no txn with a non-LAST entry rises (nl).  Absent entries (beyond nm) read and raise the
// lane's sink slot past BL_CAP.  A head whose carry comes from the ring (-2, ring index) reads it first (this
// wave wrote it one or two blocks earlier).  Then the carry-out of every LAST entry -- y' = max(y0, the levels
// of the run's txns), w' = max(w0, the levels of its Writes) -- into the ring.  Returns the rounds.
template <int E, class PK>
__device__ inline uint32_t bl_rounds(int nm, const uint4* __restrict__ cr, const int2* __restrict__ hc, int* lv,
                                     const uint8_t* nl, int2* ring, int rb, uint32_t* stuck) {
    const int lane = __lane_id();
    uint32_t slot[E], ds[E], ep[E], rn[E];
    bool wr[E], hd[E], lst[E], nle[E];
    int y0[E], w0[E], a[E];
    int2 h[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int k = lane * E + e;
        const bool v = k < nm;
        const uint4 c = v ? cr[k] : make_uint4(0u, 0u, 0u, 0u);
        slot[e] = v ? (c.x & BL_TL) : (uint32_t)(BL_CAP + lane);
        wr[e] = (c.x >> BL_SH_W) & 1u;
        hd[e] = (c.x >> BL_SH_HEAD) & 1u;
        lst[e] = (c.x >> BL_SH_LAST) & 1u;
        ds[e] = c.x >> BC_DS;
        ep[e] = c.y & 0x7FFu;
        rn[e] = (c.y >> 11) & 0x7FFu;
        h[e] = hd[e] ? hc[k] : make_int2(-1, -1);
        nle[e] = nl[slot[e]] != 0;                       // static for the block: read once, not per round
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
        if (h[e].x != -2) continue;
        h[e] = ring[h[e].y];
        const int lb = bl_sel(wr[e], h[e].x, h[e].y) + 1;
        if (lb > 0) atomicMax(&lv[slot[e]], lb);
    }
#pragma unroll
    for (int e = 0; e < E; ++e) { y0[e] = h[e].x; w0[e] = h[e].y; }
    const BzMax<PK> op{};
    uint32_t it = 0;
    while (true) {
#pragma unroll
        for (int e = 0; e < E; ++e) a[e] = lv[slot[e]];
        // scan 1: Read values by epoch (a Write opens its epoch with the bare segment word)
        PK r1 = 0, pre1[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            pre1[e] = r1;
            const PK rv = wr[e] ? bz_pack<PK>(ep[e], -BZ_BIAS) : bz_pack<PK>(ep[e], hd[e] ? max(a[e], y0[e]) : a[e]);
            r1 = r1 > rv ? r1 : rv;
        }
        const PK in1 = wave_shift_up1(op, wave_incl_scan(op, r1));
        // scan 2: z by run
        PK r2 = 0, inc2[E];
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const PK prev = in1 > pre1[e] ? in1 : pre1[e];         // the previous epoch's greatest Read value
            const int d = (int)ds[e];
            const int b = hd[e] ? max(a[e], y0[e] + 1) : max(a[e], bz_val<PK>(prev) + 1);
            const int z = hd[e] ? (wr[e] ? max(w0[e] - d + 1, b - d) : w0[e] - d) : b - d;
            const PK zv = (wr[e] || hd[e]) ? bz_pack<PK>(rn[e], z) : (PK)0;
            r2 = r2 > zv ? r2 : zv;
            inc2[e] = r2;
        }
        const PK in2 = wave_shift_up1(op, wave_incl_scan(op, r2));
        bool up = false;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            const PK zm = in2 > inc2[e] ? in2 : inc2[e];
            const int X = (int)ds[e] + bz_val<PK>(zm);
            const int x = wr[e] ? X : max(a[e], X + 1);
            const bool r = x > a[e];
            if (r) atomicMax(&lv[slot[e]], x);               // rare after the first rounds
            up |= r && nle[e];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // this round's raises before the next reads
        ++it;
        if (!__ballot(up)) break;
        // each round finalises at least the lowest unfinished txn of the block: more rounds than txns + 1 is
        // a broken invariant; stop (the host reports it) instead of spinning
        if (it > (uint32_t)BL_CAP + 1) { *stuck = 1u; break; }
    }
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
        ring[rb + (int)(cr[k].y >> 22)] = make_int2(bz_val<PK>(my), bz_val<PK>(mw));
    }
    return it;
}

// The sequential walk over the blocks (one workgroup; see the file header).  Only wave 0 (W0) is on the
// sequential path, and it touches LDS only; waves 1-3 (the workers) do all global memory traffic one block
// ahead / one block behind.  Per block b, ONE phase R_b:
//   W0       the singleton runs of b whose carry comes from the ring (list la: their key's previous run ended
//            one or two blocks earlier) -> carry-in, txn lower bound; the rounds of b's multi-entry runs and
//            their carry-outs into the ring; the carry-outs of b's singleton runs whose key continues one or two
//            blocks later (list lb) into the ring.
//   workers  block b - 1's levels into L and its carry-outs for keys continuing >= 3 blocks later into global
//            memory (the "G" carries); clear the buffers block b + 2 will use; load block b + 1 (records,
//            compacted entries, order slice, then the dependent global carry-ins, all issued before any is
//            used), prefill its txn levels from every head whose carry is known (a singleton run is then
//            final), flag its non-last entries, and build its la / lb lists; release their global stores.
// Levels / flags / bounds / list counts live in four buffers by b % 4 (W0's b, the workers' b - 1, b + 1 and the
// cleared b + 2); staged block data in two by b % 2: a worker reads block b - 1's slot x and then overwrites it
// with block b + 1's, and the two use the same slot -> thread mapping, so no barrier is needed between them.
// A G carry stored while block b - 1 is retired (R_b) is read by the staging of block >= b + 2 (R_{b+1} or
// later), after the workers' release fence and the barrier that ends R_b.
// stats[0] = greatest level + 1, stats[1] = rounds, stats[2..3] = clock64 in rounds, stats[4..5] = total,
// stats[6] = a block's rounds did not converge, stats[7] = clock64 / 256 W0 waited for the workers,
// stats[8] = W0's list work, stats[9] = the workers' work (thread WAVE).
constexpr int BL_SI = (BL_CAP + (BL_T - WAVE) - 1) / (BL_T - WAVE);   // slots per worker thread (3 waves)
// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits for the wave's outstanding global stores
// (s_waitcnt vmcnt(0)); the workers release their global stores themselves (end of their phase).
__device__ inline void bl_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct BlSum32 {
    using S = uint32_t;
    __device__ S identity() const { return 0u; }
    __device__ S combine(S a, S b) const { return a + b; }
};
struct BlStage {                               // one block's staged data in LDS (two of these, by block parity)
    uint64_t rec[BL_CAP];                      // slot records (~0: none)
    int2 car[BL_CAP];                          // singleton runs' carry-in (ring-sourced ones: written by W0)
    uint32_t ord[BL_CAP];                      // txn of each txn slot
    uint4 cr[BL_CAP];                          // compacted multi-entry run entries
    int2 hc[BL_CAP];                           // their heads' carry-in ((-2, ring index): W0 reads the ring)
    uint64_t la[BL_CAP];                       // ring-sourced singleton runs: ring | W << 12 | txn << 13 | slot << 32
    uint32_t lb[BL_CAP];                       // ring-continuing singleton runs: slot | txn << 10 | W << 21
};
struct BlBounds { uint32_t j0, j1, t0, t1, m, cnt; };   // cnt: la entries | lb entries << 16

// Load block b into `s` and prefill its levels (lv / nl: its buffers) from every head whose carry is known now.
// Called by whole waves (the list appends are wave-aggregated).
__device__ inline void bl_stage_prefill(uint32_t b, int t, int nthr, const uint32_t* __restrict__ boff,
                                        const uint32_t* __restrict__ tb, const uint64_t* __restrict__ rec,
                                        const uint4* __restrict__ crec, const uint32_t* __restrict__ mt, const int2* carry,
                                        const uint32_t* __restrict__ order, BlStage& s, BlBounds& bd, int* lv, uint8_t* nl) {
    const uint32_t j0 = boff[b], j1 = boff[b + 1], t0 = tb[b], t1 = tb[b + 1], m = mt[b];
    uint64_t r[BL_SI];
    uint4 q[BL_SI];
    uint32_t o[BL_SI];
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const uint32_t x = (uint32_t)(t + i * nthr);
        r[i] = (x < (uint32_t)BL_CAP && j0 + x < j1) ? rec[j0 + x] : ~0ull;
        o[i] = x < t1 - t0 ? order[t0 + x] : 0u;
        q[i] = x < m ? crec[j0 + x] : make_uint4(0u, 0u, 0u, 0u);
    }
    int2 c[BL_SI], h[BL_SI];
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const uint32_t x = (uint32_t)(t + i * nthr);
        c[i] = make_int2(-1, -1);
        h[i] = make_int2(-1, -1);
        const uint32_t f = (uint32_t)(r[i] >> 32);
        if (r[i] != ~0ull && (f & (1u << BL_SH_HEAD)) && (f & (1u << BL_SH_LAST)) && ((f >> BL_SH_SRC) & 3u) == 2u)
            c[i] = bl_carry_load(carry, (uint32_t)r[i]);
        if (x < m && ((q[i].x >> BL_SH_HEAD) & 1u)) {
            const uint32_t src = (q[i].x >> BL_SH_SRC) & 3u;
            if (src == 2u) h[i] = bl_carry_load(carry, q[i].z);
            else if (src == 1u) h[i] = make_int2(-2, (int)q[i].w);
        }
    }
    uint32_t cnt = 0;
    bool ia[BL_SI], ib[BL_SI];
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const uint32_t x = (uint32_t)(t + i * nthr);
        ia[i] = ib[i] = false;
        if (x >= (uint32_t)BL_CAP) continue;
        s.rec[x] = r[i];
        s.car[x] = c[i];
        s.ord[x] = o[i];
        const uint32_t f = (uint32_t)(r[i] >> 32);
        if (r[i] != ~0ull) {
            const bool head = f & (1u << BL_SH_HEAD), last = f & (1u << BL_SH_LAST);
            if (head && last) {
                if (((f >> BL_SH_SRC) & 3u) != 1u) {
                    const int lb = bl_sel(f & (1u << BL_SH_W), c[i].x, c[i].y) + 1;
                    if (lb > 0) atomicMax(&lv[f & BL_TL], lb);
                } else {
                    ia[i] = true;
                }
                ib[i] = (f >> BL_SH_R) & 1u;
            }
            if (!last) nl[f & BL_TL] = 1;
        }
        cnt += (ia[i] ? 1u : 0u) + (ib[i] ? 1u << 16 : 0u);
        if (x < m) {
            s.cr[x] = q[i];
            s.hc[x] = h[i];
            if (((q[i].x >> BL_SH_HEAD) & 1u) && h[i].x != -2) {
                const int lb = bl_sel((q[i].x >> BL_SH_W) & 1u, h[i].x, h[i].y) + 1;
                if (lb > 0) atomicMax(&lv[q[i].x & BL_TL], lb);
            }
        }
    }
    // wave-aggregated list append: one LDS atomic per wave for both lists
    const uint32_t inc = wave_incl_scan(BlSum32{}, cnt);
    uint32_t base = 0;
    if (__lane_id() == WAVE - 1) base = atomicAdd(&bd.cnt, inc);
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, WAVE - 1) + inc - cnt;
    uint32_t pa = base & 0xFFFFu, pb = base >> 16;
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const uint32_t x = (uint32_t)(t + i * nthr);
        const uint32_t f = (uint32_t)(r[i] >> 32);
        const uint32_t tl = f & BL_TL, w = (f >> BL_SH_W) & 1u;
        if (ia[i]) s.la[pa++] = (uint64_t)(((f >> BL_SH_RING) & 0xFFFu) | (w << 12) | (tl << 13)) | ((uint64_t)x << 32);
        if (ib[i]) s.lb[pb++] = x | (tl << 10) | (w << 21);
    }
    if (t == 0) { bd.j0 = j0; bd.j1 = j1; bd.t0 = t0; bd.t1 = t1; bd.m = m; }
}

// Retire block b (workers, the same slot -> thread mapping as bl_stage_prefill): its levels into L and the
// carries of keys continuing >= 3 blocks later into global memory (a singleton run's from its carry-in and its
// txn's level; a multi-entry run's from the ring, where W0 left it).  Returns the greatest level seen.
__device__ inline int bl_retire(int t, int nthr, const BlStage& s, const BlBounds& bd, const int* lv, const int2* ring,
                                int rb, int2* carry, uint32_t* __restrict__ L) {
    const uint32_t nt = bd.t1 - bd.t0;
    uint64_t rr[BL_SI];
    uint32_t od[BL_SI];
    int2 ci[BL_SI];
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const int x = t + i * nthr;
        rr[i] = x < BL_CAP ? s.rec[x] : ~0ull;
        ci[i] = x < BL_CAP ? s.car[x] : make_int2(-1, -1);
        od[i] = (uint32_t)x < nt ? s.ord[x] : 0u;
    }
    int ls[BL_SI], lo[BL_SI];
    int2 rg[BL_SI];
#pragma unroll
    for (int i = 0; i < BL_SI; ++i) {
        const int x = t + i * nthr;
        const uint32_t f = (uint32_t)(rr[i] >> 32);
        const bool g = rr[i] != ~0ull && (f & (1u << BL_SH_G));
        const bool single = (f & (1u << BL_SH_HEAD)) != 0;     // a G entry is LAST: HEAD too = singleton run
        ls[i] = g && single ? lv[f & BL_TL] : 0;
        rg[i] = g && !single ? ring[rb + x] : make_int2(0, 0);
        lo[i] = (uint32_t)x < nt ? lv[x] : -1;
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
            bl_carry_store(carry, (uint32_t)rr[i], c);
        }
        if ((uint32_t)x < nt) {
            L[od[i]] = (uint32_t)lo[i];
            maxl = max(maxl, lo[i]);
        }
    }
    return maxl;
}

template <class PK>
static __global__ __launch_bounds__(BL_T) void k_level_blocks(uint32_t B, const uint32_t* __restrict__ boff, const uint32_t* __restrict__ tb,
                                                       const uint64_t* __restrict__ rec, const uint4* __restrict__ crec,
                                                       const uint32_t* __restrict__ mt, int2* carry,
                                                       const uint32_t* __restrict__ order, uint32_t* __restrict__ L,
                                                       uint32_t* __restrict__ stats) {
    __shared__ __align__(16) int lvb[4][BL_CAP + WAVE];     // levels of a block's txns (txn-in-block index), by
                                                            // block % 4; [BL_CAP + lane]: the rounds' sinks
    __shared__ __align__(16) uint8_t nlb[4][BL_CAP + WAVE];  // txn has an entry that is not its key's last
    __shared__ int2 ring[3 * BL_CAP];          // carry-out of the slots of the last three blocks (by block % 3)
    __shared__ BlStage stg[2];
    __shared__ BlBounds bnd[4];
    __shared__ uint32_t sstuck;
    static_assert((BL_CAP + WAVE) % 16 == 0, "buffers are cleared 16 bytes at a time");
    const int tid = threadIdx.x, lane = __lane_id();
    if (tid == 0) sstuck = 0u;
    if (tid < 4) bnd[tid].cnt = 0u;
    const uint64_t tstart = clock64();
    uint64_t tround = 0, twait = 0, tlist = 0, twork = 0;
    for (int x = tid; x < BL_CAP + WAVE; x += BL_T) {
#pragma unroll
        for (int k = 0; k < 4; ++k) { lvb[k][x] = 0; nlb[k][x] = 0; }
    }
    __syncthreads();
    int maxl = -1;
    uint32_t rounds = 0;
    if (B > 0) bl_stage_prefill(0, tid, BL_T, boff, tb, rec, crec, mt, carry, order, stg[0], bnd[0], lvb[0], nlb[0]);
    __syncthreads();
    for (uint32_t b = 0; b < B; ++b) {
        const uint64_t tb0 = clock64();
        if (tid < WAVE) {
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
            const uint64_t t1 = clock64();
            if (nm > 0) {
                uint8_t* nl = nlb[b & 3];
                uint32_t r;
                const int epl = (nm + WAVE - 1) / WAVE;        // entries per lane
                if (epl <= 2) r = bl_rounds<2, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                else if (epl <= 3) r = bl_rounds<3, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                else if (epl <= 4) r = bl_rounds<4, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                else if (epl <= 5) r = bl_rounds<5, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                else if (epl <= 6) r = bl_rounds<6, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                else if (epl <= 8) r = bl_rounds<8, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                else if (epl <= 12) r = bl_rounds<12, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                else r = bl_rounds<16, PK>(nm, S.cr, S.hc, lv, nl, ring, rb, &sstuck);
                rounds += r;
            }
            const uint64_t t2 = clock64();
            tround += t2 - t1;
            // ring-continuing singleton runs: carry-out (the txn's level is final now)
            for (uint32_t k = lane; k < nbl; k += WAVE) {
                const uint32_t e = S.lb[k];
                const uint32_t x = e & 0x3FFu;
                const int2 ci = S.car[x];
                const int l = lv[(e >> 10) & BL_TL];
                ring[rb + (int)x] = make_int2(max(ci.x, l), bl_sel((e >> 21) & 1u, l, ci.y));
            }
            const uint64_t t3 = clock64();
            tlist += (t1 - tb0) + (t3 - t2);
            bl_barrier();
            twait += clock64() - t3;
        } else {
            const int t = tid - WAVE, nthr = BL_T - WAVE;
            if (b > 0) {
                const uint32_t p = b - 1;
                maxl = max(maxl, bl_retire(t, nthr, stg[p & 1], bnd[p & 3], lvb[p & 3], ring, (int)(p % 3) * BL_CAP,
                                           carry, L));
            }
            {   // clear the buffers of block b + 2 (last used by block b - 2, retired in the previous phase)
                int4* lc = reinterpret_cast<int4*>(lvb[(b + 2) & 3]);
                int4* nc = reinterpret_cast<int4*>(nlb[(b + 2) & 3]);
                for (int x = t; x < (BL_CAP + WAVE) / 4; x += nthr) lc[x] = make_int4(0, 0, 0, 0);
                for (int x = t; x < (BL_CAP + WAVE) / 16; x += nthr) nc[x] = make_int4(0, 0, 0, 0);
                if (t == 0) bnd[(b + 2) & 3].cnt = 0u;
            }
            if (b + 1 < B)
                bl_stage_prefill(b + 1, t, nthr, boff, tb, rec, crec, mt, carry, order, stg[(b + 1) & 1],
                                 bnd[(b + 1) & 3], lvb[(b + 1) & 3], nlb[(b + 1) & 3]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");    // the retired block's G carries
            twork += clock64() - tb0;
            bl_barrier();
        }
        if (sstuck) break;
    }
    if (tid >= WAVE && B > 0 && !sstuck) {
        const uint32_t p = B - 1;
        maxl = max(maxl, bl_retire(tid - WAVE, BL_T - WAVE, stg[p & 1], bnd[p & 3], lvb[p & 3], ring,
                                   (int)(p % 3) * BL_CAP, carry, L));
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
    }
    if (tid == WAVE) stats[9] = (uint32_t)(twork >> 8);
}

struct BlockBufs {                             // grow-only, owned by LevelState
    uint64_t* rec = nullptr;                   // [P]
    uint32_t *epre = nullptr, *erank = nullptr, *bk = nullptr, *bv = nullptr, *bk2 = nullptr, *bv2 = nullptr;
    uint32_t *tb = nullptr, *boff = nullptr, *stats = nullptr, *rs = nullptr, *mt = nullptr;
    int2* carry = nullptr;
    uint4* crec = nullptr;                     // [P] compacted multi-entry run entries (k_bl_compact)
    size_t capP = 0, capN = 0, capB = 0, rs_cap = 0;
    uint32_t nblocks = 0;                      // blocks of the last run
};

inline void free_block_bufs(BlockBufs& b) {
    void* ps[] = {b.rec, b.epre, b.erank, b.bk, b.bv, b.bk2, b.bv2, b.tb, b.boff, b.stats, b.rs, b.carry, b.crec, b.mt};
    for (void* p : ps) if (p) hipFree(p);
    b = BlockBufs{};
}

}  // namespace ad
