// seg_fuse_kernels.h — the deps stage's front for PreAccept batches of small key txns (C2), one kernel instead of
// three: the sorted entries' gather, CommandsForKey.mapReduceActive's per-key elision state (the ElideOp scan) and
// the count walk, per tile of whole key segments in LDS.
//
// The elision state is a SEGMENTED prefix (it restarts at every key: CommandsForKey.java:925-983 reads one key's
// byId), so a tile that starts and ends on key-segment boundaries needs nothing from its neighbours: each tile of
// SF_TILE nominal sorted positions moves its start and end forward to the next segment head (one 64-lane ballot
// per step), loads its keys, gathers the records of the entries in multi-entry segments (an entry alone in its
// segment is read by no query of the batch: complete_entries fills it in for the stages that read every entry),
// resolves each segment's state serially in LDS (a C2 segment holds ~1.5 entries), runs every non-head entry's query
// against the LDS copy, and writes the global entry state (txn, meta, executeAt + 1, segment start, last always-emitted
// entry, the two prefix maxima) only for the segments a later kernel re-walks (complete_entries rebuilds it for the
// stages that read every entry).
// Replaces k_gather_entries<true> + the three ElideOp scan launches + k_deps_walk<count>, whose reads of the
// per-entry arrays were spread over every sorted position (C2: 767,867 queries among 4,194,304 entries; the walk
// fetched 9.5x its byte model).  ElideOp's store: the tiles' head counts go to 256 partial sums (one atomic per tile,
// spread over 256 words: a single counter serialised 16K tiles' atomics, +65 us) that k_seg_heads adds into n_keys_u;
// no dense non-head list is built (its one user, the level chain build, then runs over every sorted position); the
// distinct keys and segment starts only on demand (k_seg_tile_scan + k_seg_ukeys, from complete_entries).
// A tile longer than SF_CAP (a key segment of more than ~SF_CAP - SF_TILE entries: Zipf hot keys) raises *overflow and
// the host runs the three-kernel path instead (the handle then remembers the batch had long segments).
#pragma once
#include "deps_kernels.h"
#include "level_kernels.h"

namespace ad {

constexpr int SF_T = 256;
constexpr int SF_TILE = 256;                   // nominal sorted positions per tile
constexpr int SF_CAP = 384;                    // LDS entries per tile: the tile + its last segment's tail (~17 KB of LDS:
                                               // eight workgroups per CU)

struct SegFuseArgs {
    size_t P, ntiles;
    const uint32_t* skey;                      // sorted (key - key_min), 32-bit spreads
    const PairRec* prec;
    uint32_t* tile_lo;                         // [ntiles + 1] each tile's first sorted position
    uint32_t* tile_cnt;                        // [4 * ntiles]: heads, non-heads; then their exclusive offsets
    uint32_t* hpart;                           // [2 * SF_PARTS] head-count, then multi-entry-segment partial sums (zeroed)
    uint32_t* sec;                             // [ntiles * SF_SEC]: each tile's multi-entry segments' second entries
    uint32_t* sec_cnt;                         // [ntiles]            (the level chain build's threads)
    uint32_t* overflow;
    uint32_t *e_txn;                           // global entry state (written)
    uint8_t* e_meta;
    uint64_t* e_exec1;
    int32_t *seg_start, *ud_prev;
    uint64_t *pm_w, *pm_c;
    // the pull pass's key chains (ad_run_pipeline; c_txn == null: the level stage builds them): each multi-entry
    // segment's chain from the LDS copy (chain_build_range in pred mode) -- replaces the level stage's k_chain_build
    uint32_t* c_txn;
    uint8_t* c_meta;
    uint64_t* c_exec1;
    uint32_t* c_pair;
    uint2* succ;
    uint32_t *any_long, *any_far;
};

constexpr int SF_PARTS = 256;
constexpr int SF_SEC = SF_CAP / 2;             // second entries per tile: at most one per two entries
constexpr uint32_t SF_NONE = 0xFFFFFFFFu;
// first segment head at or after x (x == P: P), searched by one wave 64 positions at a time; SF_NONE if none within
// SF_CAP positions
__device__ inline uint32_t sf_next_head(const uint32_t* __restrict__ skey, size_t P, size_t x) {
    const int lane = __lane_id();
    for (uint32_t d = 0; d < (uint32_t)SF_CAP + 64; d += WAVE) {
        const size_t y = x + d + lane;
        const bool h = y >= P || y == 0 || skey[y] != skey[y - 1];
        const uint64_t m = __ballot(h);
        if (m) return (uint32_t)(x + d + (__ffsll((unsigned long long)m) - 1));
    }
    return SF_NONE;
}

// wave-aggregated append of v to an LDS list (order inside the list is immaterial to its users)
__device__ inline void sf_list_append(bool want, uint16_t v, uint16_t* list, uint32_t* count) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int lane = __lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (want) list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = v;
}

template <int NV, bool DIRECT>
static __global__ __launch_bounds__(SF_T) void k_seg_fuse(SegFuseArgs f, WalkArgs w) {
    __shared__ uint32_t s_key[SF_CAP + 1];
    __shared__ uint32_t s_txn[SF_CAP];
    __shared__ uint8_t s_meta[SF_CAP];
    __shared__ uint8_t s_eq[SF_CAP];             // the entry's executeAt == TxnId (PREC_EXEQ)
    __shared__ uint64_t s_ex1[SF_CAP];
    __shared__ int32_t s_ss[SF_CAP];
    __shared__ int32_t s_ud[SF_CAP];
    __shared__ uint64_t s_pw[SF_CAP];
    __shared__ uint64_t s_pc[SF_CAP];
    __shared__ uint16_t s_glist[SF_CAP];
    __shared__ uint16_t s_qlist[SF_CAP];
    __shared__ uint16_t s_slist[SF_SEC];
    __shared__ uint8_t s_need[SF_CAP];           // by segment head: some query of the segment is re-walked later
    __shared__ uint32_t s_bounds[2];
    __shared__ uint32_t s_cnt[5];
    const size_t b = blockIdx.x;
    const int tid = threadIdx.x, wv = tid / WAVE;
    const size_t P = f.P;
    if (wv < 2) {
        const size_t x = (b + wv) * (size_t)SF_TILE;
        const uint32_t hd = x >= P ? (uint32_t)P : sf_next_head(f.skey, P, x);
        if (__lane_id() == 0) s_bounds[wv] = hd;
    }
    if (tid == 0) { s_cnt[0] = 0; s_cnt[1] = 0; s_cnt[2] = 0; s_cnt[3] = 0; s_cnt[4] = 0; }
    __syncthreads();
    if (s_bounds[0] == SF_NONE || s_bounds[1] == SF_NONE || s_bounds[1] - min(s_bounds[0], s_bounds[1]) > (uint32_t)SF_CAP) {
        // a key segment too long for one tile: the host takes the three-kernel path
        if (tid == 0) *f.overflow = 1u;
        return;
    }
    const uint32_t lo = s_bounds[0];
    const uint32_t hi = max(s_bounds[1], lo);
    if (tid == 0) {
        f.tile_lo[b] = lo;
        if (b + 1 == f.ntiles) f.tile_lo[f.ntiles] = (uint32_t)P;
    }
    const uint32_t L = hi - lo;
    for (uint32_t i = tid; i < L; i += SF_T) s_key[i] = f.skey[lo + i];
    __syncthreads();
    // flags per entry; the multi-entry segments' entries (gathered) and the non-head entries (queried) listed densely
    // in LDS, so the random gathers and the query walks run on full waves (~34 % / ~18 % of a C2 tile's entries)
    uint32_t heads = 0, nonheads = 0;
    for (uint32_t i0 = 0; i0 < L; i0 += SF_T) {
        const uint32_t i = i0 + tid;
        const bool in = i < L;
        const bool head = in && (i == 0 || s_key[i] != s_key[i - 1]);
        const bool last = in && (i + 1 == L || s_key[i + 1] != s_key[i]);
        heads += head ? 1u : 0u;
        nonheads += (in && !head) ? 1u : 0u;
        if (in) s_need[i] = 0;
        sf_list_append(in && !(head && last), (uint16_t)i, s_glist, &s_cnt[2]);
        sf_list_append(in && !head, (uint16_t)i, s_qlist, &s_cnt[3]);
        // the second entry of a segment (its predecessor is the head)
        const bool second = in && !head && (i == 1 || s_key[i - 2] != s_key[i - 1]);
        sf_list_append(second, (uint16_t)i, s_slist, &s_cnt[4]);
    }
    atomicAdd(&s_cnt[0], heads);
    atomicAdd(&s_cnt[1], nonheads);
    __syncthreads();
    const uint32_t ng = s_cnt[2], nq = s_cnt[3];
    // (list slots dealt round-robin over the waves instead — slot = lane * waves + wave, so that every wave takes a
    // quarter of a tile's ~47 queries — measured slower: 156 -> 186 us)
    const uint32_t rr = (uint32_t)tid;
    for (uint32_t x = rr; x < ng; x += SF_T) {
        const uint32_t i = s_glist[x];
        const PairRec r = f.prec[w.sval[lo + i]];
        s_txn[i] = r.txn; s_meta[i] = (uint8_t)r.meta; s_ex1[i] = r.ex1; s_eq[i] = (r.meta & PREC_EXEQ) ? 1 : 0;
    }
    __syncthreads();
    // per multi-entry segment (its head's thread): the elision scan state, serially (ElideOp::combine restarted at the
    // head)
    for (uint32_t i = tid; i < L; i += SF_T) {
        if (!(i == 0 || s_key[i] != s_key[i - 1]) || i + 1 == L || s_key[i + 1] != s_key[i]) continue;
        const int32_t hs = (int32_t)(lo + i);
        int32_t ud = -1;
        uint64_t pw = 0, pc = 0;
        for (uint32_t q = i; q < L && s_key[q] == s_key[i]; ++q) {
            const uint32_t m = s_meta[q];
            const uint32_t cat = category(m);
            const uint64_t x1 = s_ex1[q];
            if (cat == CAT_ALWAYS) ud = (int32_t)(lo + q);
            if (cat == CAT_ELIDABLE) {
                pc = x1 > pc ? x1 : pc;
                if (meta_kind(m) == AD_KIND_WRITE) pw = x1 > pw ? x1 : pw;
            }
            s_ss[q] = hs; s_ud[q] = ud; s_pw[q] = pw; s_pc[q] = pc;
        }
    }
    __syncthreads();
    if (tid == 0) {
        f.tile_cnt[2 * b] = s_cnt[0]; f.tile_cnt[2 * b + 1] = s_cnt[1];
        if (s_cnt[0]) atomicAdd(&f.hpart[b % SF_PARTS], s_cnt[0]);
        if (s_cnt[4]) atomicAdd(&f.hpart[SF_PARTS + b % SF_PARTS], s_cnt[4]);    // multi-entry segments
        f.sec_cnt[b] = s_cnt[4];
    }
    for (uint32_t x = tid; x < s_cnt[4]; x += SF_T) f.sec[b * (size_t)SF_SEC + x] = lo + s_slist[x];
    // the queries of the non-head entries, against the LDS copy (sorted position s -> s - lo)
    WalkArgs a = w;
    a.e_txn = s_txn - lo; a.e_meta = s_meta - lo; a.e_exec1 = s_ex1 - lo; a.seg_start = s_ss - lo; a.ud_prev = s_ud - lo;
    a.pm_w = s_pw - lo; a.pm_c = s_pc - lo;
    // (the PreAccept bound TxnId + 1 from the record when executeAt == TxnId: no random tx_ts read for ~90 % of them)
    for (uint32_t x = rr; x < nq; x += SF_T) {
        const uint32_t q = s_qlist[x];
        if (walk_pair_entry<NV, false, DIRECT>(a, (size_t)lo + q, s_eq[q] ? s_ex1[q] : 0ull)) s_need[s_ss[q] - (int32_t)lo] = 1;
    }
    __syncthreads();
    // The global entry state (gathered record + elision state) only for the segments a later kernel re-walks from it
    // (overflowed lists: k_txn_finish_ovf; wide txns: the fill walk) — C2: a few segments per batch.  Every other
    // stage that reads the entries (levels other than the pull pass, MaxConflicts, recovery, CFK retain, sharded
    // levels) calls complete_entries first, which rebuilds the whole state with the gather + ElideOp scan (the
    // scattered state writes were ~60 % of this kernel's HBM write traffic).
    for (uint32_t x = rr; x < ng; x += SF_T) {
        const uint32_t i = s_glist[x];
        if (!s_need[s_ss[i] - (int32_t)lo]) continue;
        f.e_txn[lo + i] = s_txn[i]; f.e_meta[lo + i] = s_meta[i]; f.e_exec1[lo + i] = s_ex1[i];
        f.seg_start[lo + i] = s_ss[i]; f.ud_prev[lo + i] = s_ud[i]; f.pm_w[lo + i] = s_pw[i]; f.pm_c[lo + i] = s_pc[i];
    }
    if (f.c_txn) {
        bool lng = false, far = false;
        for (uint32_t x = tid; x < s_cnt[4]; x += SF_T) {
            const uint32_t i = s_slist[x], s0 = i - 1;            // the segment's second entry and its head
            uint32_t e = i + 1;
            while (e < L && s_key[e] == s_key[s0]) ++e;
            chain_build_range((size_t)lo + s0, (size_t)lo + e, s_txn - lo, s_meta - lo, s_ex1 - lo, w.sval, f.c_txn,
                              f.c_meta, f.c_exec1, f.c_pair, nullptr, f.succ, 0, 1, lng, far);
        }
        wave_set_flag(lng, f.any_long);
        wave_set_flag(far, f.any_far);
    }
}

// n_keys_u = the tiles' heads (after k_seg_fuse; nothing after an overflow: the host re-runs the batch)
static __global__ __launch_bounds__(SF_PARTS) void k_seg_heads(const uint32_t* __restrict__ hpart, Params* prm,
                                                              const uint32_t* __restrict__ overflow) {
    __shared__ uint32_t s_w[SF_PARTS / WAVE], s_m[SF_PARTS / WAVE];
    if (overflow && *(const volatile uint32_t*)overflow) return;
    uint32_t v = hpart[threadIdx.x], u = hpart[SF_PARTS + threadIdx.x];
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) { v += __shfl_xor(v, o); u += __shfl_xor(u, o); }
    if (__lane_id() == 0) { s_w[threadIdx.x / WAVE] = v; s_m[threadIdx.x / WAVE] = u; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0, m = 0;
        for (int k = 0; k < SF_PARTS / WAVE; ++k) { t += s_w[k]; m += s_m[k]; }
        prm->n_keys_u = t;
        prm->n_multi = m;
    }
}

// Exclusive prefix of the tiles' head / non-head counts (one workgroup); useg[U] = P (U = the heads, = n_keys_u).
// Runs on demand (complete_entries), after the host saw no overflow.
static __global__ __launch_bounds__(1024) void k_seg_tile_scan(size_t ntiles, size_t P, uint32_t* __restrict__ tile_cnt,
                                                               uint32_t* __restrict__ useg) {
    __shared__ uint32_t s_h[1024], s_n[1024];
    uint32_t carry_h = 0, carry_n = 0;
    for (size_t base = 0; base < ntiles; base += 1024) {
        const size_t t = base + threadIdx.x;
        const uint32_t h = t < ntiles ? tile_cnt[2 * t] : 0u, nn = t < ntiles ? tile_cnt[2 * t + 1] : 0u;
        s_h[threadIdx.x] = h; s_n[threadIdx.x] = nn;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {
            const uint32_t yh = threadIdx.x >= (unsigned)o ? s_h[threadIdx.x - o] : 0u;
            const uint32_t yn = threadIdx.x >= (unsigned)o ? s_n[threadIdx.x - o] : 0u;
            __syncthreads();
            s_h[threadIdx.x] += yh; s_n[threadIdx.x] += yn;
            __syncthreads();
        }
        if (t < ntiles) {
            tile_cnt[2 * ntiles + 2 * t] = carry_h + s_h[threadIdx.x] - h;
            tile_cnt[2 * ntiles + 2 * t + 1] = carry_n + s_n[threadIdx.x] - nn;
        }
        carry_h += s_h[1023]; carry_n += s_n[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) useg[carry_h] = (uint32_t)P;
}

// On demand (complete_entries: only the stages that read every key need it, not the C2 pipeline): the distinct
// keys (ukey) and their segment starts (useg), in order.
static __global__ __launch_bounds__(SF_T) void k_seg_ukeys(size_t ntiles, const uint32_t* __restrict__ tile_lo,
                                                           const uint32_t* __restrict__ tile_cnt,
                                                           const uint32_t* __restrict__ skey, uint64_t key_min,
                                                           uint64_t* __restrict__ ukey, uint32_t* __restrict__ useg) {
    __shared__ uint32_t s_w[SF_T / WAVE];
    const size_t b = blockIdx.x;
    const uint32_t lo = tile_lo[b], hi = tile_lo[b + 1];
    uint32_t ch = tile_cnt[2 * ntiles + 2 * b];
    const int tid = threadIdx.x, lane = __lane_id(), wv = tid / WAVE;
    const uint64_t below = (1ull << lane) - 1ull;
    for (uint32_t base = lo; base < hi; base += SF_T) {
        const uint32_t s = base + tid;
        const bool head = s < hi && (s == 0 || skey[s] != skey[s - 1]);
        const uint64_t mh = __ballot(head);
        if (lane == 0) s_w[wv] = (uint32_t)__popcll(mh);
        __syncthreads();
        uint32_t ph = ch, th = 0;
        for (int k = 0; k < SF_T / WAVE; ++k) {
            if (k < wv) ph += s_w[k];
            th += s_w[k];
        }
        if (head) {
            const uint32_t u = ph + (uint32_t)__popcll(mh & below);
            ukey[u] = (uint64_t)skey[s] + key_min;
            useg[u] = s;
        }
        ch += th;
        __syncthreads();
    }
}

}  // namespace ad
