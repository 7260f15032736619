// level_kernels.h — execution levels (Kahn wavefront index) over the resolved dependency graph.
//
// Semantics (the reference's dynamic release order, local/Commands.java:617-821 and
// local/cfk/CommandsForKey.java:1208-1330), level[T] = 1 + max level over T's predecessors (0 if none):
//   (a) managed T (key Read/Write), on every key of T: a Write waits for all earlier-executeAt Reads and
//       Writes, a Read for earlier-executeAt Writes (notifyManaged, unappliedCounters :1291-1330);
//   (b) every T: its merged direct-key and range deps with an earlier executeAt
//       (Commands.updateWaitingOn :740-755);
//   (c) unmanaged T (range txns), per key of its merged KeyDeps: every managed txn on that key with
//       executeAt <= the greatest executeAt among T's deps there below T's own (Updating.updateUnmanaged
//       :740-757 -> Unmanaged APPLY: "wait for it and all earlier txn to Apply", CommandsForKey.java:437-445).
// Every edge raises executeAt, so the levels are a topological wavefront numbering and `order` = txns
// sorted by (level, executeAt).
//
// Device algorithm (no per-level launches — C3 chains are ~10^5 deep):
//   1. chain order: the (key, TxnId)-sorted entries are re-sorted by executeAt inside each key segment
//      (in-place fix-up; nearly sorted because only slow-path txns move).
//   2. along one key chain (a) is a max-plus affine map on the state (y = max level so far, w = max
//      Write level so far):  Read: y' = max(y, w+1, a), w' = w;  Write: y' = w' = max(y+1, a), where a is
//      the txn's current level from its other constraints.  Maps compose associatively, so one segmented
//      scan (scan.h) resolves an entire chain at once, whatever its depth; it also materialises the
//      inclusive prefix max pm_all used by (c).
//   3. (b) and (c) are relaxations over the merged CSRs (atomicMax on the level array).
//   4. 2-3 repeat until no level changes; the iteration count is the number of chain-to-chain hops on
//      the critical path (C2: ~9).
//   5. order: LSD radix sorts by executeAt (64-bit, two 32-bit halves) then stably by level.
#pragma once
#include <functional>
#include <chrono>
#include <cstring>

#include "radix_sort.h"
#include "union_kernels.h"
#include "block_levels.h"

namespace ad {

constexpr int NEG = -(1 << 29);
__device__ inline int mp_add(int x, int y) { return (x <= NEG || y <= NEG) ? NEG : x + y; }
__device__ inline int mp_max(int x, int y) { return x > y ? x : y; }

// Re-queue the other chain segments of txn t after its level rose to x (worklist fixpoint).
struct PushCtx {
    const uint32_t* key_off;     // [n+1] txn -> pair range
    const int32_t* pair_seg;     // [P] head position of each pair's chain segment
    const uint32_t* seg_len;     // [P] valid at head positions
    uint32_t* stamp;             // [P] at heads: the iteration the segment is (re)queued for
    uint32_t* long_dirty;        // long segments must be rescanned next iteration
    uint32_t iter1;              // current iteration + 1
};
constexpr uint32_t SHORT_SEG = 64;   // chains up to this length: one thread walks them

// Returns true if some short segment was newly queued for the next iteration (the caller reports it
// once per wave, so the "work left" flag sees one store per wave, not one per push).
// Fire-and-forget atomics: the caller already saw L[t] < x, so it re-queues t's other segments without
// waiting for the atomics' round trips (a concurrent higher raise only makes the re-queue redundant; the
// fixpoint still terminates because a segment whose inputs did not rise raises nothing).
__device__ inline bool raise_level(uint32_t* L, uint32_t t, uint32_t x, int32_t own_seg, const PushCtx& c) {
    atomicMax(&L[t], x);
    bool queued = false;
    for (uint32_t p = c.key_off[t]; p < c.key_off[t + 1]; ++p) {
        const int32_t h = c.pair_seg[p];          // push target: short chain head, -1 singleton, -2 long chain
        if (h == own_seg || h == -1) continue;
        if (h == -2) {
            if (*(volatile uint32_t*)c.long_dirty == 0u) *c.long_dirty = 1u;
            continue;
        }
        atomicMax(&c.stamp[h], c.iter1);
        queued = true;
    }
    return queued;
}

// Long chains: the (a) recurrence as a segmented max-plus scan over the concatenated long segments
// (positions through `idx`), whatever their depth.
struct ChainOp {
    struct S {
        int m00, m01, m10, m11;   // max-plus matrix
        int c0, c1;               // constant
        int a;                    // element only: the txn's level estimate
        uint32_t flags;           // element only: bit0 head, bit1 participates, bit2 write
    };
    const uint32_t* idx;          // scan index -> chain position
    const uint32_t* c_txn;
    const uint8_t* c_meta;
    const int32_t* seg_start;     // key segments (same in (key,TxnId) and (key,executeAt) order)
    uint32_t* L;
    int32_t* pm_all;              // inclusive prefix max level along the chain
    PushCtx push;
    uint32_t* work_left;          // some short segment is queued for the next iteration
    const uint32_t* enable;       // previous iteration dirtied a long chain (nullptr: always run)

    __device__ S identity() const { return S{0, NEG, NEG, 0, NEG, NEG, 0, 0u}; }
    __device__ S load(size_t i) const {
        if (enable && !*enable) return identity();
        const uint32_t pos = idx[i];
        const uint32_t m = c_meta[pos];
        const bool head = seg_start[pos] == (int32_t)pos;
        const bool part = manages_execution(m);
        const bool wr = meta_kind(m) == AD_KIND_WRITE;
        S s = identity();
        s.flags = (head ? 1u : 0u) | (part ? 2u : 0u) | (wr ? 4u : 0u);
        if (!part) {
            if (head) { s.m00 = s.m01 = s.m10 = s.m11 = NEG; s.c0 = -1; s.c1 = -1; }
            return s;
        }
        const int a = (int)L[c_txn[pos]];
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
        if (enable && !*enable) return;
        const uint32_t pos = idx[i];
        int py, pw;
        if (el.flags & 1u) { py = -1; pw = -1; }
        else {
            py = mp_max(mp_max(mp_add(ex.m00, -1), mp_add(ex.m01, -1)), ex.c0);
            pw = mp_max(mp_max(mp_add(ex.m10, -1), mp_add(ex.m11, -1)), ex.c1);
        }
        if (!(el.flags & 2u)) {
            pm_all[pos] = py;
            return;
        }
        const int x = (el.flags & 4u) ? mp_max(py + 1, el.a) : mp_max(pw + 1, el.a);
        pm_all[pos] = mp_max(py, x);
        if (x > el.a && raise_level(L, c_txn[pos], (uint32_t)x, seg_start[pos], push))
            if (*(volatile uint32_t*)work_left == 0u) *work_left = 1u;
    }
};

// Short chains: one thread per short multi-entry segment; segments not queued for this iteration
// (stamp != it) exit at once.  Walks the chain in executeAt order with the same recurrence.
static __global__ __launch_bounds__(256) void k_seg_short(const uint32_t* __restrict__ heads, uint32_t count, uint32_t it,
                                                   const uint32_t* __restrict__ c_txn, const uint8_t* __restrict__ c_meta,
                                                   uint32_t* L, int32_t* __restrict__ pm_all, PushCtx push,
                                                   uint32_t* __restrict__ work_left) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool queued = false;
    if (i < count) {
        const uint32_t h = heads[i];
        if (push.stamp[h] == it) {
            const uint32_t len = push.seg_len[h];
            int y = -1, w = -1;
            for (uint32_t p = h; p < h + len; ++p) {
                const uint32_t m = c_meta[p];
                if (manages_execution(m)) {
                    const uint32_t t = c_txn[p];
                    const int a = (int)L[t];
                    const bool wr = meta_kind(m) == AD_KIND_WRITE;
                    const int x = wr ? mp_max(y + 1, a) : mp_max(w + 1, a);
                    if (x > a) queued |= raise_level(L, t, (uint32_t)x, (int32_t)h, push);
                    y = mp_max(y, x);
                    if (wr) w = mp_max(w, x);
                }
                pm_all[p] = y;
            }
        }
    }
    wave_set_flag(queued, work_left);
}

// Segment table: length and stamp at each head; per position: is it the head of a short multi-entry
// segment (-> heads list), is it inside a long segment (-> long positions list).
static __global__ __launch_bounds__(256) void k_seg_table(size_t P, const int32_t* __restrict__ seg_start, uint32_t* __restrict__ seg_len,
                                                   uint32_t* __restrict__ stamp, uint32_t* __restrict__ any_long) {
    const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool lng = false;
    if (s < P) {
        const int32_t h = seg_start[s];
        if (s + 1 == P || seg_start[s + 1] != h) {
            const uint32_t len = (uint32_t)(s + 1 - (size_t)h);
            seg_len[h] = len;
            stamp[h] = 0u;
            lng = len > SHORT_SEG;
        }
    }
    wave_set_flag(lng, any_long);
}
struct SegListOp {                 // two compactions in one scan: short multi heads, long positions
    struct S { uint32_t a, b; };
    const int32_t* seg_start;
    const uint32_t* seg_len;
    uint32_t* heads;
    uint32_t* long_pos;
    uint32_t* totals;              // [0] heads, [1] long positions
    size_t n;
    __device__ S load(size_t i) const {
        const int32_t h = seg_start[i];
        const uint32_t len = seg_len[h];
        S s;
        s.a = (h == (int32_t)i && len >= 2 && len <= SHORT_SEG) ? 1u : 0u;
        s.b = len > SHORT_SEG ? 1u : 0u;
        return s;
    }
    __device__ S identity() const { return S{0u, 0u}; }
    __device__ S combine(const S& x, const S& y) const { return S{x.a + y.a, x.b + y.b}; }
    __device__ void store(size_t i, const S& ex, const S& inc, const S& el) const {
        if (el.a) heads[ex.a] = (uint32_t)i;
        if (el.b) long_pos[ex.b] = (uint32_t)i;
        if (i + 1 == n) { totals[0] = inc.a; totals[1] = inc.b; }
    }
};
static __global__ __launch_bounds__(256) void k_stamp_reset(const uint32_t* __restrict__ heads, uint32_t count, uint32_t* __restrict__ stamp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) stamp[heads[i]] = 0u;
}

// txn pair -> push target: head position of its chain if that chain is short and has 2+ entries,
// -1 for nothing to re-walk, -2 for a long chain (rescanned by the segmented scan).  One thread per chain
// position (executeAt order); the target is scattered to the pair (c_pair).
// Without (c) constraints a raise of T only matters to the entries of the chain that wait for T: a Write
// has dependants iff it is not the chain's last entry, a Read iff a Write follows it.  A pair with no
// dependants gets -1, so raising T does not re-walk that chain.  With (c), every position's prefix max
// (pm_all) is read by unmanaged txns, so every chain containing T is re-walked.
static __global__ __launch_bounds__(256) void k_pair_seg(size_t P, const uint32_t* __restrict__ c_pair, const uint8_t* __restrict__ c_meta,
                                                  const int32_t* __restrict__ seg_start, const uint32_t* __restrict__ seg_len,
                                                  int32_t* __restrict__ pair_seg, int prune) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const int32_t h = seg_start[q];
    const uint32_t len = seg_len[h];
    int32_t tgt = len < 2 ? -1 : (len > SHORT_SEG ? -2 : h);
    if (prune && tgt >= 0) {
        const size_t end = (size_t)h + len;
        bool dep = false;
        if (meta_kind(c_meta[q]) == AD_KIND_WRITE) dep = q + 1 < end;
        else
            for (size_t x = q + 1; x < end && !dep; ++x) dep = meta_kind(c_meta[x]) == AD_KIND_WRITE;
        if (!dep) tgt = -1;
    }
    pair_seg[c_pair[q]] = tgt;
}

static __global__ __launch_bounds__(256) void k_chain_copy(size_t P, const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                                    const uint64_t* __restrict__ e_exec1, const uint32_t* __restrict__ sval,
                                                    uint32_t* __restrict__ c_txn, uint8_t* __restrict__ c_meta,
                                                    uint64_t* __restrict__ c_exec1, uint32_t* __restrict__ c_pair) {
    const size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P) return;
    c_txn[s] = e_txn[s];
    c_meta[s] = e_meta[s];
    c_exec1[s] = e_exec1[s];
    c_pair[s] = sval[s];
}

// Per-segment fix-up: entries of one key ordered by executeAt (insertion sort; one thread per segment).
static __global__ __launch_bounds__(256) void k_chain_order(size_t P, const int32_t* __restrict__ seg_start,
                                                     uint32_t* __restrict__ c_txn, uint8_t* __restrict__ c_meta,
                                                     uint64_t* __restrict__ c_exec1, uint32_t* __restrict__ c_pair) {
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
        uint32_t px = c_pair[x];
        size_t y = x;
        while (y > s && c_exec1[y - 1] > kx) {
            c_exec1[y] = c_exec1[y - 1]; c_txn[y] = c_txn[y - 1]; c_meta[y] = c_meta[y - 1]; c_pair[y] = c_pair[y - 1];
            --y;
        }
        c_exec1[y] = kx; c_txn[y] = tx; c_meta[y] = mx; c_pair[y] = px;
    }
}

// Rejects kinds the batch execution order does not model (local-only txns are not globally visible).
static __global__ __launch_bounds__(256) void k_level_kinds(size_t n, const uint8_t* __restrict__ meta, uint32_t* __restrict__ flag) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (t < n) bad = meta_kind(meta[t]) == AD_KIND_LOCAL_ONLY;
    wave_set_flag(bad, flag);
}

// Txn.Kind.awaitsOnlyDeps (Txn.java:211-214): ExclusiveSyncPoint and EphemeralRead wait for every dependency,
// whatever its executeAt (Commands.initialiseWaitingOn :690-691 waits at maxForEpoch).
__device__ inline bool awaits_only_deps(uint32_t m) {
    const uint32_t k = meta_kind(m);
    return k == AD_KIND_EXCLUSIVE_SYNC_POINT || k == AD_KIND_EPHEMERAL_READ;
}
__device__ inline bool is_sync_point(uint32_t m) {
    const uint32_t k = meta_kind(m);
    return k == AD_KIND_SYNC_POINT || k == AD_KIND_EXCLUSIVE_SYNC_POINT;
}

struct EdgeArgs {
    size_t n;
    const uint8_t* meta;
    const uint64_t* ex1;
    uint32_t* L;
    // (b) merged direct / range deps: unique dependency lists
    const uint32_t* ent_off[2];
    const uint32_t* tcnt[2];
    const uint32_t* txns[2];
    // (c) unmanaged txns, merged KeyDeps
    const uint32_t* mk_key_off;
    const uint64_t* mk_keys;
    const uint32_t* mk_k2t_off;
    const int32_t* mk_k2t;
    const uint32_t* mk_ent_off;
    const uint32_t* mk_txns;
    int32_t* cons_pos;           // [merged key slot] chain position or -1
    const int32_t* pm_all;
    const uint64_t* ukey;
    const uint32_t* useg;
    uint32_t U;
    const uint64_t* c_exec1;
    const uint32_t* c_txn;
    const int32_t* seg_start;
    // sync points: the key's entries in TxnId order (CommandsForKey.byId)
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    PushCtx push;
    uint32_t* changed;           // any edge raised a level this iteration
    uint32_t* work_left;
};

// (c) preparation: for unmanaged T and each key of its merged KeyDeps, the last chain position (in
// executeAt order) whose executeAt <= bnd = max executeAt of T's qualifying deps on that key
// (Updating.updateUnmanaged :740-792): below T's own executeAt, any for an EphemeralRead, any earlier TxnId
// for an ExclusiveSyncPoint; sync points also fold the key's managed-execution entries between their first
// and last dependency in TxnId order (:760-777; a loop over that byId range).
// One wave per txn, one lane per key of its merged KeyDeps (a C4 range txn has ~3*10^3 of them).
static __global__ __launch_bounds__(256) void k_unmanaged_prep(EdgeArgs a) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n) return;
    const uint32_t kb = a.mk_key_off[t], ke = a.mk_key_off[t + 1];
    const uint32_t mt = a.meta[t];
    const bool unmanaged = !manages_execution(mt);
    const bool any_exec = awaits_only_deps(mt);            // ESP deps all have earlier TxnIds
    const bool sync = is_sync_point(mt);
    const uint32_t nk = ke - kb;
    const uint32_t mb = a.mk_k2t_off[t];
    const uint32_t tb = a.mk_ent_off[t];
    const uint64_t my = a.ex1[t];
    uint32_t ulo = 0;                                      // this lane's previous key's position in ukey
    for (uint32_t ki = __lane_id(); ki < nk; ki += WAVE) {
        int32_t pos = -1;
        if (unmanaged) {
            const uint32_t from = mb + (ki == 0 ? nk : (uint32_t)a.mk_k2t[mb + ki - 1]);
            const uint32_t to = mb + (uint32_t)a.mk_k2t[mb + ki];
            uint64_t bnd = 0;
            for (uint32_t x = from; x < to; ++x) {
                const uint64_t e = a.ex1[a.mk_txns[tb + (uint32_t)a.mk_k2t[x]]];
                if ((any_exec || e < my) && e > bnd) bnd = e;
            }
            const uint64_t key = a.mk_keys[kb + ki];
            uint32_t u = a.U;
            if (from < to) {
                // the txn's keys ascend and sit among ukey's: gallop from the lane's previous key (a range txn's
                // keys are nearly consecutive in ukey, 64 apart per lane) instead of a full binary search
                uint32_t lo = ulo, hi = a.U, step = WAVE;
                while (true) {
                    const uint32_t p = lo + step;
                    if (p >= a.U) break;
                    if (a.ukey[p] < key) { lo = p + 1; step <<= 1; } else { hi = p + 1; break; }
                }
                u = lb_u64(a.ukey, lo, hi, key);
                ulo = u;
            }
            const bool found = u < a.U && a.ukey[u] == key;
            if (sync && found) {
                // per-key lists are ascending: first and last dependency (batch ranks = TxnId order)
                const uint32_t f = a.mk_txns[tb + (uint32_t)a.mk_k2t[from]], l = a.mk_txns[tb + (uint32_t)a.mk_k2t[to - 1]];
                const uint32_t s0 = a.useg[u], s1 = a.useg[u + 1];
                uint32_t lo = s0, hi = s1;
                while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (a.e_txn[m] < f) lo = m + 1; else hi = m; }
                for (uint32_t x = lo; x < s1 && a.e_txn[x] <= l; ++x) {
                    const uint32_t em = a.e_meta[x];
                    const uint64_t e = a.e_exec1[x];
                    if (manages_execution(em) && (any_exec || e < my) && e > bnd) bnd = e;
                }
            }
            if (bnd != 0 && found) {
                const uint32_t s0 = a.useg[u], s1 = a.useg[u + 1];
                const uint32_t p = ub_u64(a.c_exec1, s0, s1, bnd);     // first executeAt+1 > bnd
                pos = p > s0 ? (int32_t)(p - 1) : -1;
            }
        }
        a.cons_pos[kb + ki] = pos;
    }
}

// (b) + (c) relaxation, one thread per txn.
static __global__ __launch_bounds__(256) void k_level_edges(EdgeArgs a, int do_b, int do_c, const uint32_t* prev) {
    if (prev && !(prev[0] | prev[1] | prev[2])) return;     // nothing changed in the previous iteration
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool raised = false, queued = false;
    if (t < a.n) {
        const uint64_t my = a.ex1[t];
        int best = -1;
        if (do_b) {
            const bool all = awaits_only_deps(a.meta[t]);
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                if (!a.txns[c]) continue;
                const uint32_t b = a.ent_off[c][t], e = b + a.tcnt[c][t];
                for (uint32_t x = b; x < e; ++x) {
                    const uint32_t d = a.txns[c][x];
                    if (all || a.ex1[d] < my) best = max(best, (int)a.L[d]);
                }
            }
        }
        if (do_c && !manages_execution(a.meta[t])) {
            for (uint32_t x = a.mk_key_off[t]; x < a.mk_key_off[t + 1]; ++x) {
                const int32_t p = a.cons_pos[x];
                if (p < 0) continue;
                // singleton chains are never walked: their prefix max is the entry's own level
                const bool single = a.push.seg_len[a.seg_start[p]] < 2;
                best = max(best, single ? (int)a.L[a.c_txn[p]] : a.pm_all[p]);
            }
        }
        if (best >= 0) {
            const uint32_t v = (uint32_t)(best + 1);
            if (v > a.L[t]) {
                const uint32_t old = a.L[t];
                queued = raise_level(a.L, (uint32_t)t, v, -1, a.push);
                raised = old < v;
            }
        }
    }
    wave_set_flag(raised, a.changed);
    wave_set_flag(queued, a.work_left);
}

static __global__ __launch_bounds__(256) void k_exec_split(size_t n, const uint64_t* __restrict__ ex1, const uint32_t* __restrict__ idx,
                                                    uint32_t* __restrict__ key, int hi) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t t = idx ? idx[i] : (uint32_t)i;
    const uint64_t e = ex1[t] - 1;
    key[i] = hi ? (uint32_t)(e >> 32) : (uint32_t)e;
}
static __global__ __launch_bounds__(256) void k_iota(size_t n, uint32_t* __restrict__ v) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (uint32_t)i;
}
// gather + block-reduced max (one atomic per block)
static __global__ __launch_bounds__(256) void k_gather_u32(size_t n, const uint32_t* __restrict__ src, const uint32_t* __restrict__ idx,
                                                    uint32_t* __restrict__ dst, uint32_t* __restrict__ maxv) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v = 0;
    if (i < n) { v = src[idx[i]]; dst[i] = v; }
    v = wave_max(v);
    __shared__ uint32_t red[256 / WAVE];
    if (__lane_id() == 0) red[threadIdx.x / WAVE] = v;
    __syncthreads();
    if (threadIdx.x == 0 && maxv) {
        uint32_t m = red[0];
        for (int k = 1; k < 256 / WAVE; ++k) m = m > red[k] ? m : red[k];
        atomicMax(maxv, m);
    }
}

// ---------------------------------------------------------------------------------------------------
// Kahn wavefront for shallow key-chain graphs (no chain longer than SHORT_SEG, no (b)/(c) constraints):
// every txn is visited once, when its last predecessor is released, instead of re-walking chains until
// a fixpoint.  Per chain position the (a) rule reduces to a transitive reduction:
//   Read R   waits for the last Write before it (1 edge, if any);
//   Write W  waits for the Reads since the last Write before it, or for that Write if none; with no
//            earlier Write, for every earlier entry (all Reads).
// so each position's successors are one contiguous run of its chain: after a Write, the Reads that follow
// it (or the next Write if a Write follows directly); after a Read, the next Write.  Same chain order and
// rule as the fixpoint walk, so the levels are identical.  k_chain_build derives both per segment.
// ---------------------------------------------------------------------------------------------------
// Register version of the chain build for segments of at most CB_REG entries (C2: all multi-entry
// segments): odd-even transposition sort on (executeAt, arrival) in registers, both passes unrolled, and
// only c_txn (what the wavefronts read) is written back.
constexpr int CB_REG = 8;
constexpr uint32_t PRED_TXN = 0x80000000u;   // pred mode: the run is one txn, stored in .x
// pred mode feeds the one-pass pull levels, whose lanes wait for their predecessors' lanes: a predecessor more
// than PULL_FAR rows AFTER its dependant (a slow-path bump moved its executeAt far back) may sit in a workgroup
// not yet resident while the waiting ones occupy the chip, so such batches take the Kahn wavefronts instead
constexpr uint32_t PULL_FAR = 1u << 16;
__device__ inline void chain_build_regs(size_t s, int len, const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                        const uint64_t* __restrict__ e_exec1, const uint32_t* __restrict__ sval,
                                        uint32_t* __restrict__ c_txn, uint32_t* __restrict__ indeg, uint2* __restrict__ succ,
                                        uint8_t* __restrict__ c_meta, uint64_t* __restrict__ c_exec1, bool pred_mode, bool& far) {
    uint64_t k[CB_REG];
    uint32_t t[CB_REG], pr[CB_REG], wr[CB_REG], ord[CB_REG];
#pragma unroll
    for (int i = 0; i < CB_REG; ++i) {
        const bool v = i < len;
        k[i] = v ? e_exec1[s + i] : ~0ull;
        t[i] = v ? e_txn[s + i] : 0u;
        pr[i] = v ? sval[s + i] : 0u;
        wr[i] = v ? (uint32_t)e_meta[s + i] : 0u;        // meta byte (kind tested below)
        ord[i] = (uint32_t)i;
    }
#pragma unroll
    for (int r = 0; r < CB_REG; ++r) {
#pragma unroll
        for (int i = r & 1; i + 1 < CB_REG; i += 2) {
            const bool sw = k[i] > k[i + 1] || (k[i] == k[i + 1] && ord[i] > ord[i + 1]);
            if (sw) {
                uint64_t a = k[i]; k[i] = k[i + 1]; k[i + 1] = a;
                uint32_t b = t[i]; t[i] = t[i + 1]; t[i + 1] = b;
                b = pr[i]; pr[i] = pr[i + 1]; pr[i + 1] = b;
                b = wr[i]; wr[i] = wr[i + 1]; wr[i + 1] = b;
                b = ord[i]; ord[i] = ord[i + 1]; ord[i + 1] = b;
            }
        }
    }
    if (c_exec1) {                        // (c) constraints search the executeAt-ordered chain
#pragma unroll
        for (int q = 0; q < CB_REG; ++q)
            if (q < len) { c_exec1[s + q] = k[q]; c_meta[s + q] = (uint8_t)wr[q]; }
    }
#pragma unroll
    for (int q = 0; q < CB_REG; ++q) wr[q] = meta_kind((uint8_t)wr[q]) == AD_KIND_WRITE ? 1u : 0u;
    bool seen_w = false;
    uint32_t reads = 0, lw_txn = 0;
#pragma unroll
    for (int q = 0; q < CB_REG; ++q) {
        if (q < len) {
            c_txn[s + q] = t[q];
            if (pred_mode) {
                // the same reduced edges as predecessor runs: a Read's last Write before it; a Write's Reads
                // since the last Write, else that Write.  A single predecessor is stored as its txn
                // (PRED_TXN): the pull pass then needs no c_txn hop.
                uint2 pe = make_uint2(0u, 0u);
                if (wr[q] && reads > 1) pe = make_uint2((uint32_t)(s + q) - reads, reads);
                else if (wr[q] && reads == 1) pe = make_uint2(t[q > 0 ? q - 1 : 0], 1u | PRED_TXN);
                else if (seen_w) pe = make_uint2(lw_txn, 1u | PRED_TXN);
                if (pe.y) succ[pr[q]] = pe;
                // the latest predecessor row: a Write's Reads since the last Write, or that Write
                uint32_t pmax = 0;
#pragma unroll
                for (int x = 0; x < CB_REG; ++x)
                    if (wr[q] && reads > 1 && x < q && x >= q - (int)reads) pmax = t[x] > pmax ? t[x] : pmax;
                if (pe.y & PRED_TXN) pmax = pe.x;
                if (pmax > t[q] + PULL_FAR) far = true;
            } else {
                const uint32_t pc = wr[q] ? (reads > 0 ? reads : (seen_w ? 1u : 0u)) : (seen_w ? 1u : 0u);
                if (pc) atomicAdd(&indeg[t[q]], pc);
            }
            if (wr[q]) { seen_w = true; reads = 0; lw_txn = t[q]; } else ++reads;
        }
    }
    if (pred_mode) return;
    int next_w = len;
#pragma unroll
    for (int q = CB_REG - 1; q >= 0; --q) {
        if (q < len) {
            uint2 sc = make_uint2(0u, 0u);
            if (wr[q]) {
                if (q + 1 < len) sc = next_w == q + 1 ? make_uint2((uint32_t)(s + q + 1), 1u)
                                                      : make_uint2((uint32_t)(s + q + 1), (uint32_t)(next_w - (q + 1)));
                next_w = q;
            } else if (next_w < len) {
                sc = make_uint2((uint32_t)(s + next_w), 1u);
            }
            if (sc.y) succ[pr[q]] = sc;        // succ was cleared: empty runs need no store
        }
    }
}

// Kahn path chain build, one thread per multi-entry key segment (fuses k_chain_copy, k_chain_order,
// k_seg_table and k_kahn_prep): the segment is copied into executeAt order (stable insertion: entries
// arrive in TxnId order and only slow-path ones move), then a forward pass counts each position's reduced
// predecessors (indeg) and a backward pass gives its successor run (succ[pair]).  Single-entry segments
// have no edges and are skipped; a segment longer than SHORT_SEG raises *any_long and the caller falls
// back to the fixpoint (whose chain preparation handles long chains).
// The chain of the key segment [s, end) (sorted positions; e_* may point into LDS: k_seg_fuse builds the chains of
// its tile's segments from its LDS copy).
__device__ inline void chain_build_range(size_t s, size_t end,
                                         const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                         const uint64_t* __restrict__ e_exec1, const uint32_t* __restrict__ sval,
                                         uint32_t* __restrict__ c_txn, uint8_t* __restrict__ c_meta,
                                         uint64_t* __restrict__ c_exec1, uint32_t* __restrict__ c_pair,
                                         uint32_t* __restrict__ indeg, uint2* __restrict__ succ, int full, int pred_mode,
                                         bool& lng, bool& far) {
    {
        if (end - s > SHORT_SEG) {
            lng = true;
        } else if (end - s <= CB_REG) {
            chain_build_regs(s, (int)(end - s), e_txn, e_meta, e_exec1, sval, c_txn, indeg, succ, full ? c_meta : nullptr,
                             full ? c_exec1 : nullptr, pred_mode != 0, far);
        } else {
            for (size_t x = s; x < end; ++x) {
                const uint64_t kx = e_exec1[x];
                const uint32_t tx = e_txn[x], px = sval[x];
                const uint8_t mx = e_meta[x];
                size_t y = x;
                while (y > s && c_exec1[y - 1] > kx) {
                    c_exec1[y] = c_exec1[y - 1]; c_txn[y] = c_txn[y - 1]; c_meta[y] = c_meta[y - 1]; c_pair[y] = c_pair[y - 1];
                    --y;
                }
                c_exec1[y] = kx; c_txn[y] = tx; c_meta[y] = mx; c_pair[y] = px;
            }
            // predecessors: a Read waits for the last Write before it; a Write for the Reads since the last
            // Write, else for that Write (k_kahn_prep states the reduction)
            bool seen_w = false;
            uint32_t reads = 0;
            size_t lw = s;
            for (size_t q = s; q < end; ++q) {
                const bool wr = meta_kind(c_meta[q]) == AD_KIND_WRITE;
                if (pred_mode) {
                    uint2 pe = make_uint2(0u, 0u);
                    if (wr && reads > 1) pe = make_uint2((uint32_t)(q - reads), reads);
                    else if (wr && reads == 1) pe = make_uint2(c_txn[q - 1], 1u | PRED_TXN);
                    else if (seen_w) pe = make_uint2(c_txn[lw], 1u | PRED_TXN);
                    if (pe.y) succ[c_pair[q]] = pe;
                    uint32_t pmax = (pe.y & PRED_TXN) ? pe.x : 0u;
                    if (wr && reads > 1)
                        for (size_t y = q - reads; y < q; ++y) pmax = c_txn[y] > pmax ? c_txn[y] : pmax;
                    if (pmax > c_txn[q] + PULL_FAR) far = true;
                } else {
                    const uint32_t pc = wr ? (reads > 0 ? reads : (seen_w ? 1u : 0u)) : (seen_w ? 1u : 0u);
                    if (pc) atomicAdd(&indeg[c_txn[q]], pc);
                }
                if (wr) { seen_w = true; reads = 0; lw = q; } else ++reads;
            }
            // successors: after a Write the Reads that follow it (or the next Write if one follows
            // directly); after a Read the next Write
            size_t next_w = end;
            for (size_t q = end; !pred_mode && q-- > s;) {
                const bool wr = meta_kind(c_meta[q]) == AD_KIND_WRITE;
                uint2 sc = make_uint2(0u, 0u);
                if (wr) {
                    if (q + 1 < end) sc = next_w == q + 1 ? make_uint2((uint32_t)(q + 1), 1u)
                                                          : make_uint2((uint32_t)(q + 1), (uint32_t)(next_w - (q + 1)));
                    next_w = q;
                } else if (next_w < end) {
                    sc = make_uint2((uint32_t)next_w, 1u);
                }
                succ[c_pair[q]] = sc;
            }
        }
    }
}
// The chain of the key segment whose second entry is s2 (s2 = 0 or not a second entry: nothing).
__device__ inline void chain_build_seg(size_t P, size_t s2, const int32_t* __restrict__ seg_start,
                                       const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                       const uint64_t* __restrict__ e_exec1, const uint32_t* __restrict__ sval,
                                       uint32_t* __restrict__ c_txn, uint8_t* __restrict__ c_meta,
                                       uint64_t* __restrict__ c_exec1, uint32_t* __restrict__ c_pair,
                                       uint32_t* __restrict__ indeg, uint2* __restrict__ succ, int full, int pred_mode,
                                       bool& lng, bool& far) {
    const size_t s = s2 - 1;
    if (s2 > 0 && seg_start[s2] == (int32_t)s) {
        size_t end = s + 2;
        while (end < P && seg_start[end] == (int32_t)s && end - s <= SHORT_SEG) ++end;
        chain_build_range(s, end, e_txn, e_meta, e_exec1, sval, c_txn, c_meta, c_exec1, c_pair, indeg, succ, full,
                          pred_mode, lng, far);
    }
}

// One thread per non-head entry (ElideOp's dense list); the second entry of each segment builds it.  nh == null (the
// batches whose deps stage ran k_seg_fuse, which builds no list): each workgroup covers CB_SPAN sorted positions and
// first compacts its segments' second entries into LDS, so the builders run on full waves (one thread per position
// left ~85 % of the lanes of this latency-bound kernel idle: 41 -> 115 us on C2)
constexpr int CB_SPAN = 1536;             // ~230 builders per workgroup of 256 on C2
static __global__ __launch_bounds__(256) void k_chain_build(size_t P, const uint32_t* __restrict__ nh, const Params* __restrict__ prm,
                                                     const int32_t* __restrict__ seg_start,
                                                     const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                                     const uint64_t* __restrict__ e_exec1, const uint32_t* __restrict__ sval,
                                                     uint32_t* __restrict__ c_txn, uint8_t* __restrict__ c_meta,
                                                     uint64_t* __restrict__ c_exec1, uint32_t* __restrict__ c_pair,
                                                     uint32_t* __restrict__ indeg, uint2* __restrict__ succ,
                                                     uint32_t* __restrict__ any_long, int full, int pred_mode = 0,
                                                     uint32_t* __restrict__ any_far = nullptr,
                                                     const uint32_t* __restrict__ sec = nullptr,
                                                     const uint32_t* __restrict__ sec_cnt = nullptr, int sec_cap = 0,
                                                     uint32_t sec_tiles = 0) {
    bool lng = false, far = false;
    if (sec) {
        // k_seg_fuse's per-tile lists of the segments' second entries: one wave per tile
        const uint32_t tile = blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
        if (tile < sec_tiles) {
            const uint32_t c = sec_cnt[tile];
            for (uint32_t x = __lane_id(); x < c; x += WAVE)
                chain_build_seg(P, sec[(size_t)tile * sec_cap + x], seg_start, e_txn, e_meta, e_exec1, sval, c_txn, c_meta,
                                c_exec1, c_pair, indeg, succ, full, pred_mode, lng, far);
        }
    } else if (nh) {
        const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
        const size_t s2 = x < P - prm->n_keys_u ? (size_t)nh[x] : 0;
        chain_build_seg(P, s2, seg_start, e_txn, e_meta, e_exec1, sval, c_txn, c_meta, c_exec1, c_pair, indeg, succ, full,
                        pred_mode, lng, far);
    } else {
        __shared__ uint32_t q[CB_SPAN];
        __shared__ uint32_t qn;
        if (threadIdx.x == 0) qn = 0;
        __syncthreads();
        const size_t base = (size_t)blockIdx.x * CB_SPAN;
        const int lane = __lane_id();
        for (int k = 0; k < CB_SPAN / 256; ++k) {
            const size_t s2 = base + (size_t)k * 256 + threadIdx.x + 1;
            const bool want = s2 < P && seg_start[s2] == (int32_t)(s2 - 1);
            const uint64_t m = __ballot(want);
            if (!m) continue;
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t b0 = 0;
            if (lane == leader) b0 = atomicAdd(&qn, (uint32_t)__popcll(m));
            b0 = __shfl(b0, leader);
            if (want) q[b0 + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)s2;
        }
        __syncthreads();
        const uint32_t nq = qn;
        for (uint32_t k = threadIdx.x; k < nq; k += blockDim.x)
            chain_build_seg(P, q[k], seg_start, e_txn, e_meta, e_exec1, sval, c_txn, c_meta, c_exec1, c_pair, indeg, succ,
                            full, pred_mode, lng, far);
    }
    wave_set_flag(lng, any_long);
    if (any_far) wave_set_flag(far, any_far);
}

// One wavefront: the txns released at level `lvl` (level 0: indeg == 0 in the snapshot; later levels:
// L == lvl, which only a release sets) release their successors; the last release of S sets L[S] = lvl+1.
// prev: the previous wavefront's "released something" flag (nullptr: run); *work: this one released some.
// gate: the previous wavefront's "released something" flag (run if set), or for the first wavefront of a
// batch (gate_is_abort) the chain build's long-chain flag (run if clear).
// Grid-stride over a bounded grid (an empty wavefront costs one small launch).  For txns with up to 4
// keys the first successor of every pair is released with all loads and atomics issued together (the
// returning atomics are the latency of this kernel); longer runs and wider txns go serially.
constexpr int KAHN_GRID = 2048;
__device__ inline void kahn_release(uint32_t s, uint32_t lvl, uint32_t* __restrict__ rem, uint32_t* __restrict__ L, bool& released) {
    if (atomicSub(&rem[s], 1u) == 1u) { L[s] = lvl + 1; released = true; }
}
// Release ids[x] for x = b, b + stride, ... < e, KR_ILP at a time: the id loads, then the returning atomics, then
// the checks, so a lane keeps KR_ILP memory round trips in flight instead of one.  A wavefront lasts as long as
// its longest serial release chain (a Write followed by several Reads, a range txn's thousands of dependants):
// one atomic round trip per successor made those chains the kernel time.
constexpr int KR_ILP = 8;
template <class I>
__device__ inline void kahn_release_run(const uint32_t* __restrict__ ids, I b, I e, I stride, uint32_t lvl,
                                        uint32_t* __restrict__ rem, uint32_t* __restrict__ L, bool& released) {
    for (I x = b; x < e; x += stride * (I)KR_ILP) {
        uint32_t sv[KR_ILP], rv[KR_ILP];
#pragma unroll
        for (int u = 0; u < KR_ILP; ++u) { const I y = x + (I)u * stride; sv[u] = y < e ? ids[y] : 0u; }
#pragma unroll
        for (int u = 0; u < KR_ILP; ++u) { const I y = x + (I)u * stride; rv[u] = y < e ? atomicSub(&rem[sv[u]], 1u) : 0u; }
#pragma unroll
        for (int u = 0; u < KR_ILP; ++u)
            if (rv[u] == 1u) { L[sv[u]] = lvl + 1; released = true; }
    }
}
// ---------------------------------------------------------------------------------------------------
// any key segment longer than SHORT_SEG: the chain build's long-chain test alone (no chain is built)
static __global__ __launch_bounds__(256) void k_any_long_seg(size_t P, const int32_t* __restrict__ seg_start,
                                                     uint32_t* __restrict__ any_long) {
    const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool lng = false;
    if (j < P) {
        const int32_t h = seg_start[j];
        lng = h >= 0 && j - (size_t)h >= SHORT_SEG;
    }
    wave_set_flag(lng, any_long);
}

// Kahn chain build for batches with long chains (C3's Zipf hot keys: ~10^5 entries on one key), all
// positions in parallel instead of one thread per segment:
//   1. k_chain_rank: executeAt order inside each key segment by windowed inversion ranks (entries arrive in
//      TxnId order; only slow-path bumps move, a few positions): rank = i + #{later j in the segment and
//      the +-CR_D window with a smaller executeAt} - #{earlier j with a larger one}, scattered with the
//      entry; k_chain_check verifies every slot was filled and executeAt ascends per segment (else the
//      serial k_chain_order runs).
//   2. two segmented scans: last Write before each position, next Write after it (or the segment end);
//   3. k_chain_links: the transitive reduction of the (a) rule from those two positions: in-degree per
//      txn and the successor run per pair, the same edges k_chain_build derives serially.
constexpr int CR_N = 1024, CR_D = 64, CR_T = 256;
static __global__ __launch_bounds__(CR_T) void k_chain_rank(size_t P, const int32_t* __restrict__ seg_start,
                                                     const uint32_t* __restrict__ e_txn, const uint8_t* __restrict__ e_meta,
                                                     const uint64_t* __restrict__ e_exec1, const uint32_t* __restrict__ sval,
                                                     uint32_t* __restrict__ c_txn, uint8_t* __restrict__ c_meta,
                                                     uint64_t* __restrict__ c_exec1, uint32_t* __restrict__ c_pair) {
    __shared__ uint64_t sk[CR_N + 2 * CR_D];
    __shared__ int32_t ss[CR_N + 2 * CR_D];
    const long base = (long)blockIdx.x * CR_N;
    for (int x = threadIdx.x; x < CR_N + 2 * CR_D; x += CR_T) {
        const long g = base + x - CR_D;
        const bool in = g >= 0 && g < (long)P;
        sk[x] = in ? e_exec1[g] : 0ull;
        ss[x] = in ? seg_start[g] : -2;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < CR_N; e += CR_T) {
        const long i = base + e;
        if (i >= (long)P) break;
        const uint64_t key = sk[e + CR_D];
        const int32_t sg = ss[e + CR_D];
        int r = 0;
#pragma unroll 16
        for (int k = 1; k <= CR_D; ++k) {
            r += (ss[e + CR_D + k] == sg && sk[e + CR_D + k] < key) ? 1 : 0;
            r -= (ss[e + CR_D - k] == sg && sk[e + CR_D - k] > key) ? 1 : 0;
        }
        const long q = i + r;
        if (q < 0 || q >= (long)P) continue;          // the check pass sees the hole
        c_txn[q] = e_txn[i];
        c_meta[q] = e_meta[i];
        c_exec1[q] = key;
        c_pair[q] = sval[i];
    }
}
static __global__ __launch_bounds__(256) void k_chain_check(size_t P, const int32_t* __restrict__ seg_start,
                                                     const uint64_t* __restrict__ c_exec1, const uint32_t* __restrict__ c_pair,
                                                     uint32_t* __restrict__ bad) {
    bool b = false;
    for (size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x; q < P; q += (size_t)gridDim.x * blockDim.x) {
        if (c_pair[q] == 0xFFFFFFFFu) b = true;
        else if (q + 1 < P && seg_start[q + 1] == seg_start[q] && c_exec1[q] > c_exec1[q + 1]) b = true;
    }
    wave_set_flag(b, bad);
}
// MIN = false: exclusive prefix max of Write positions per segment (-1: none) = last Write before q.
// MIN = true (scanned from the end): exclusive suffix min of Write positions per segment, the segment end
// when none = next Write after q.
template <bool MIN>
struct WriteLinkOp {
    struct S { int32_t f, v; };
    size_t P;
    const int32_t* seg_start;
    const uint8_t* c_meta;
    int32_t* out;
    __device__ size_t pos(size_t i) const { return MIN ? P - 1 - i : i; }
    __device__ S identity() const { return S{0, MIN ? 0x7FFFFFFF : -1}; }
    __device__ S load(size_t i) const {
        const size_t q = pos(i);
        const bool wr = meta_kind(c_meta[q]) == AD_KIND_WRITE;
        S s;
        if (MIN) {
            const bool last = q + 1 == P || seg_start[q + 1] != seg_start[q];
            s.f = last ? 1 : 0;
            s.v = wr ? (int32_t)q : (last ? (int32_t)(q + 1) : 0x7FFFFFFF);
        } else {
            s.f = seg_start[q] == (int32_t)q ? 1 : 0;
            s.v = wr ? (int32_t)q : -1;
        }
        return s;
    }
    __device__ S combine(const S& x, const S& y) const {
        if (y.f) return y;
        return S{x.f, MIN ? (x.v < y.v ? x.v : y.v) : (x.v > y.v ? x.v : y.v)};
    }
    __device__ void store(size_t i, const S& ex, const S&, const S& el) const {
        const size_t q = pos(i);
        out[q] = el.f ? (MIN ? (int32_t)(q + 1) : -1) : ex.v;
    }
};
static __global__ __launch_bounds__(256) void k_chain_links(size_t P, const int32_t* __restrict__ seg_start,
                                                     const uint32_t* __restrict__ c_txn, const uint8_t* __restrict__ c_meta,
                                                     const uint32_t* __restrict__ c_pair, const int32_t* __restrict__ last_w,
                                                     const int32_t* __restrict__ next_w, uint32_t* __restrict__ indeg,
                                                     uint2* __restrict__ succ) {
    const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= P) return;
    const int32_t s0 = seg_start[q];
    const bool wr = meta_kind(c_meta[q]) == AD_KIND_WRITE;
    const int32_t lw = last_w[q], nw = next_w[q];
    const bool last = q + 1 == P || seg_start[q + 1] != s0;
    uint32_t pc;
    if (wr) pc = lw >= 0 ? ((int32_t)q - lw - 1 > 0 ? (uint32_t)((int32_t)q - lw - 1) : 1u) : (uint32_t)((int32_t)q - s0);
    else pc = lw >= 0 ? 1u : 0u;
    if (pc) atomicAdd(&indeg[c_txn[q]], pc);
    uint2 sc = make_uint2(0u, 0u);
    if (wr) {
        if (!last) sc = nw == (int32_t)q + 1 ? make_uint2((uint32_t)q + 1, 1u) : make_uint2((uint32_t)q + 1, (uint32_t)(nw - ((int32_t)q + 1)));
    } else if (nw < (int32_t)P && seg_start[nw] == s0) {
        sc = make_uint2((uint32_t)nw, 1u);
    }
    if (sc.y) succ[c_pair[q]] = sc;
}

// Extra successors (mixed key + range batches): xs[xoff[t] .. xoff[t+1]) are the txns waiting on t through a
// (b) dependency edge or a (c) chain-prefix constraint (k_xedges).  A txn with at most XLIGHT of them releases
// them itself; heavier ones (a range txn can have thousands of dependants) are released by the whole wave,
// 64 lanes per edge run.
constexpr uint64_t XLIGHT = 8;

static __global__ __launch_bounds__(256) void k_kahn_step(size_t n, uint32_t lvl, const uint32_t* __restrict__ indeg0,
                                                   uint32_t* __restrict__ rem, uint32_t* __restrict__ L,
                                                   const uint32_t* __restrict__ key_off, const uint2* __restrict__ succ,
                                                   const uint32_t* __restrict__ c_txn, const uint32_t* gate, int gate_is_abort,
                                                   uint32_t* __restrict__ work, const uint64_t* __restrict__ xoff,
                                                   const uint32_t* __restrict__ xs) {
    if (gate_is_abort ? *gate != 0u : *gate == 0u) return;
    bool released = false;
    // block-aligned stride: every lane of a wave runs the same iterations (the heavy-run ballot below)
    for (size_t base = (size_t)blockIdx.x * blockDim.x; base < n; base += (size_t)gridDim.x * blockDim.x) {
        const size_t t = base + threadIdx.x;
        const bool mine = t < n && (lvl == 0 ? indeg0[t] == 0u : L[t] == lvl);
        if (mine && key_off) {                 // key_off == nullptr: an explicit edge graph (xoff / xs) only
            const uint32_t b = key_off[t], e = key_off[t + 1];
            if (e - b <= 4) {
                uint2 sc[4];
                uint32_t sx[4], rr[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) sc[j] = b + j < e ? succ[b + j] : make_uint2(0u, 0u);
#pragma unroll
                for (int j = 0; j < 4; ++j) sx[j] = sc[j].y ? c_txn[sc[j].x] : 0u;
#pragma unroll
                for (int j = 0; j < 4; ++j) rr[j] = sc[j].y ? atomicSub(&rem[sx[j]], 1u) : 0u;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (sc[j].y && rr[j] == 1u) { L[sx[j]] = lvl + 1; released = true; }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (sc[j].y > 1) kahn_release_run<uint32_t>(c_txn, sc[j].x + 1, sc[j].x + sc[j].y, 1u, lvl, rem, L, released);
            } else {
                for (uint32_t p = b; p < e; ++p) {
                    const uint2 sc = succ[p];
                    if (sc.y) kahn_release_run<uint32_t>(c_txn, sc.x, sc.x + sc.y, 1u, lvl, rem, L, released);
                }
            }
        }
        if (xoff) {
            uint64_t xb = 0, xe = 0;
            if (mine) { xb = xoff[t]; xe = xoff[t + 1]; }
            const bool heavy = xe - xb > XLIGHT;
            if (mine && !heavy)
                kahn_release_run<uint64_t>(xs, xb, xe, 1ull, lvl, rem, L, released);
            uint64_t hm = __ballot(heavy);
            while (hm) {
                const int l = __ffsll((unsigned long long)hm) - 1;
                hm &= hm - 1;
                const uint64_t b0 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(xb >> 32), l) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((uint32_t)xb, l);
                const uint64_t e0 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(xe >> 32), l) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((uint32_t)xe, l);
                kahn_release_run<uint64_t>(xs, b0 + __lane_id(), e0, (uint64_t)WAVE, lvl, rem, L, released);
            }
        }
    }
    wave_set_flag(released, work);
}

// ---------------------------------------------------------------------------------------------------
// One-pass levels for shallow key-chain batches (C2: 10 levels, chains of a few entries).  (Tried for mixed key +
// range batches with the (b)/(c) sources read per txn from its merged deps: on C4's 5,650 levels ~10^6 lanes
// wait at once and their polling swamps the memory side, so the pass hit its cap; mixed batches stay on the
// Kahn wavefronts.)  Kahn pays one grid
// launch plus the slowest lane's chain of returning atomics per level.  Here every txn pulls instead: its
// level = 1 + the maximum level of its predecessor runs (the same reduced (a) edges, written by the chain
// build in pred mode), 0 without predecessors, and it publishes the level with LV_FINAL once every
// predecessor's is final.  One launch: a wave retries its unfinished lanes until all have published (a lane
// never blocks inside the wave, so a predecessor in the same wave is never starved).  Predecessors have a
// smaller executeAt, i.e. almost always a smaller TxnId, so the txns a lane waits for sit in the same or an
// earlier workgroup; a slow-path bump points at most a few workgroups ahead, and those are dispatched as
// earlier ones retire.  A lane that has waited ~1 s raises *abort and publishes a placeholder (so no
// lane waits for ever); the caller then recomputes the batch with the Kahn wavefronts.  Levels are read and
// written with agent-scope atomics: the 8 XCDs' L2s are not coherent with each other.
constexpr uint32_t LV_FINAL = 0x80000000u;
constexpr uint64_t PULL_CAP_TICKS = 100000000ull;    // wall_clock64 at 100 MHz: a lane gives up after ~1 s
static __global__ __launch_bounds__(256) void k_level_pull(size_t n, const uint32_t* __restrict__ key_off, const uint2* __restrict__ pred,
                                                    const uint32_t* __restrict__ c_txn, uint32_t* L, const uint32_t* gate,
                                                    const uint32_t* gate_far, uint32_t* abort_flag, uint32_t* __restrict__ bmax,
                                                    int force_abort) {
    __shared__ uint32_t wm[256 / WAVE];
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    // long chains (block path) or far predecessors (Kahn): the caller takes another path
    const bool gated = *gate != 0u || *gate_far != 0u;
    bool done = t >= n || gated;
    if (!done && force_abort) {                         // tests: every lane takes the abort path at once
        __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&L[t], LV_FINAL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        done = true;
    }
    uint32_t b = 0, e = 0, m = 0, tries = 0;
    if (!done) { b = key_off[t]; e = key_off[t + 1]; }
    const uint64_t t0 = wall_clock64();
    while (__ballot(!done)) {
        if (!done) {
            bool ready = true;
            uint32_t mm = 0;
            for (uint32_t p = b; p < e && ready; ++p) {
                const uint2 r = pred[p];
                const bool one = (r.y & PRED_TXN) != 0u;
                const uint32_t len = r.y & ~PRED_TXN;
                for (uint32_t x = 0; x < len; ++x) {
                    const uint32_t j = one ? r.x : c_txn[r.x + x];
                    const uint32_t v = __hip_atomic_load(&L[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (!(v & LV_FINAL)) { ready = false; break; }
                    const uint32_t lv = (v & ~LV_FINAL) + 1u;
                    mm = lv > mm ? lv : mm;
                }
            }
            if (ready) {
                __hip_atomic_store(&L[t], mm | LV_FINAL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                m = mm;
                done = true;
            } else if ((++tries & 63u) == 0u &&
                       (wall_clock64() - t0 > PULL_CAP_TICKS ||
                        __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                // waited too long (or another lane did): placeholder, and the caller redoes the batch
                __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&L[t], LV_FINAL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                done = true;
            } else {
                __builtin_amdgcn_s_sleep(1);
                if (tries > 64) __builtin_amdgcn_s_sleep(8);      // back off as the wait grows
            }
        }
    }
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) { const uint32_t y = __shfl_xor(m, o); m = y > m ? y : m; }
    if (__lane_id() == 0) wm[threadIdx.x / WAVE] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x = 0;
        for (int w = 0; w < 256 / WAVE; ++w) x = wm[w] > x ? wm[w] : x;
        bmax[blockIdx.x] = x;
    }
}
// max of the per-workgroup maxima (one workgroup); strips LV_FINAL from the levels afterwards
// the greatest level from k_level_pull's per-block maxima (one workgroup); then the FINAL bits cleared
static __global__ __launch_bounds__(1024) void k_level_pull_max(uint32_t nb, const uint32_t* __restrict__ bmax, uint32_t* out) {
    __shared__ uint32_t wm[1024 / WAVE];
    uint32_t m = 0;
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) m = bmax[i] > m ? bmax[i] : m;
    m = wave_max(m);
    if (__lane_id() == 0) wm[threadIdx.x / WAVE] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x = 0;
        for (int w = 0; w < 1024 / WAVE; ++w) x = wm[w] > x ? wm[w] : x;
        *out = x;
    }
}
static __global__ __launch_bounds__(256) void k_level_strip(size_t n, uint32_t* __restrict__ L) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) L[t] &= ~LV_FINAL;
}

// Deep graphs (C3: the hot key's ~10^5 Writes make ~10^5 levels, a handful of txns each): one launch per
// wavefront costs more than the wavefront.  k_kahn_small runs consecutive wavefronts inside ONE workgroup:
// the frontier is an explicit list (LDS counter, global slots), released successors are appended to the
// next list, a workgroup barrier separates levels.  It stops when a frontier exceeds KS_MAX (the
// grid-wide k_kahn_step takes over from that level: its L == lvl test needs no list) or is empty.
// k_frontier_collect builds the list of the txns at level lvl for the switch.
constexpr int KS_T = 1024;
constexpr uint32_t KS_MAX = 4096;
static __global__ __launch_bounds__(256) void k_frontier_collect(size_t n, uint32_t lvl, const uint32_t* __restrict__ indeg0,
                                                          const uint32_t* __restrict__ L, uint32_t* __restrict__ F,
                                                          uint32_t* __restrict__ count) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = t < n && (lvl == 0 ? indeg0[t] == 0u : L[t] == lvl);
    const uint64_t m = __ballot(in);
    if (!in) return;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if ((int)__lane_id() == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    const uint32_t pos = base + (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
    if (pos < KS_MAX) F[pos] = (uint32_t)t;
}
// state[0] = frontier size in (level lvl0, list in F0); out: [0] = the size of the frontier left (0 = done,
// all levels final), [1] = its level (the grid-wide steps resume there through L == lvl).
static __global__ __launch_bounds__(KS_T) void k_kahn_small(uint32_t lvl0, uint32_t* __restrict__ state, uint32_t* __restrict__ F0,
                                                      uint32_t* __restrict__ F1, uint32_t* __restrict__ rem,
                                                      uint32_t* __restrict__ L, const uint32_t* __restrict__ key_off,
                                                      const uint2* __restrict__ succ, const uint32_t* __restrict__ c_txn,
                                                      const uint64_t* __restrict__ xoff = nullptr,
                                                      const uint32_t* __restrict__ xs = nullptr) {
    __shared__ uint32_t nf;
    __shared__ uint32_t fa[KS_MAX], fb[KS_MAX];      // frontier lists live in LDS
    uint32_t count = state[0], lvl = lvl0;
    for (uint32_t i = threadIdx.x; i < count && i < KS_MAX; i += KS_T) fa[i] = F0[i];
    uint32_t* cur = fa;
    uint32_t* nxt = fb;
    int which = 0;
    auto release = [&](uint32_t sx, uint32_t r) {
        if (r == 1u) {
            L[sx] = lvl + 1;
            const uint32_t pos = atomicAdd(&nf, 1u);
            if (pos < KS_MAX) nxt[pos] = sx;
        }
    };
    while (count > 0 && count <= KS_MAX) {
        if (threadIdx.x == 0) nf = 0;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < count; i += KS_T) {
            const uint32_t t = cur[i];
            if (xoff)
                for (uint64_t x = xoff[t]; x < xoff[t + 1]; ++x) {
                    const uint32_t y = xs[x];
                    release(y, atomicSub(&rem[y], 1u));
                }
            if (!key_off) continue;
            const uint32_t b = key_off[t], e = key_off[t + 1];
            if (e - b <= 4) {
                // every key's first successor: loads and atomics issued together (one dependent chain)
                uint2 sc[4];
                uint32_t sx[4], rr[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) sc[j] = b + j < e ? succ[b + j] : make_uint2(0u, 0u);
#pragma unroll
                for (int j = 0; j < 4; ++j) sx[j] = sc[j].y ? c_txn[sc[j].x] : 0u;
#pragma unroll
                for (int j = 0; j < 4; ++j) rr[j] = sc[j].y ? atomicSub(&rem[sx[j]], 1u) : 0u;
#pragma unroll
                for (int j = 0; j < 4; ++j) if (sc[j].y) release(sx[j], rr[j]);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    for (uint32_t x = sc[j].x + 1; x < sc[j].x + sc[j].y; ++x) {
                        const uint32_t y = c_txn[x];
                        release(y, atomicSub(&rem[y], 1u));
                    }
            } else {
                for (uint32_t p = b; p < e; ++p) {
                    const uint2 sc = succ[p];
                    for (uint32_t x = sc.x; x < sc.x + sc.y; ++x) {
                        const uint32_t y = c_txn[x];
                        release(y, atomicSub(&rem[y], 1u));
                    }
                }
            }
        }
        __threadfence_block();
        __syncthreads();
        const uint32_t c = nf;
        __syncthreads();
        if (c == 0) { count = 0; break; }
        ++lvl;
        count = c;
        uint32_t* tmp = cur; cur = nxt; nxt = tmp;
        which ^= 1;
        if (count > KS_MAX) break;       // too wide for one workgroup: the grid-wide steps continue at lvl
    }
    if (threadIdx.x == 0) { state[0] = count; state[1] = lvl; state[2] = (uint32_t)which; }
}

// (b) and (c) as explicit Kahn edges, one thread per txn T (count pass: per-source out-degrees and T's
// in-degree; fill pass: T appended to each source's successor run):
//   (b) every merged direct-key / range dependency D of T with executeAt(D) < executeAt(T) (every D when T
//       awaits only its deps);
//   (c) unmanaged T, per key of its merged KeyDeps with a constraint position p (k_unmanaged_prep): every
//       managed entry of that key's chain at positions <= p.  The chain rule already orders the prefix, so
//       its maximum level sits on the last Write at or before p or on a Read after it: the edges come from
//       the Reads in (last Write, p] and that Write (all entries down to the segment head if none).
struct XEdgeArgs {
    EdgeArgs e;
    const uint8_t* c_meta;
    int do_b, do_c;
    int done_aware;                      // CFK history batches: no edge into or out of an APPLIED / INVALID txn
    uint32_t* indeg;
    unsigned long long* outcnt;          // count pass: [n] per-source out-degree
    unsigned long long* cur;             // fill pass: [n] per-source write cursor (starts at xoff)
    uint32_t* xs;
};
// The (b) / (c) sources of txn t, emit(src) each (an edge src -> t).  (c) walks the executeAt chain down from
// the constraint position over the managed entries only (key-domain sync points / ephemeral reads sit in the
// key segments but not in the execution chains).
__device__ inline bool status_done(uint32_t m) {
    const uint32_t s = meta_status(m);
    return s == AD_ST_APPLIED || s == AD_ST_INVALID;
}
template <class Emit>
__device__ inline void xedges_visit(const XEdgeArgs& a, size_t t, Emit&& emit) {
    const EdgeArgs& e = a.e;
    if (a.done_aware && status_done(e.meta[t])) return;
    if (a.do_b) {
        const uint64_t my = e.ex1[t];
        const bool all = awaits_only_deps(e.meta[t]);
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            if (!e.txns[c]) continue;
            const uint32_t b = e.ent_off[c][t], end = b + e.tcnt[c][t];
            for (uint32_t x = b; x < end; ++x) {
                const uint32_t d = e.txns[c][x];
                if ((all || e.ex1[d] < my) && !(a.done_aware && status_done(e.meta[d]))) emit(d);
            }
        }
    }
    if (a.do_c && !manages_execution(e.meta[t])) {
        for (uint32_t x = e.mk_key_off[t]; x < e.mk_key_off[t + 1]; ++x) {
            const int32_t p = e.cons_pos[x];
            if (p < 0) continue;
            const int32_t s0 = e.seg_start[p];
            for (int32_t q = p;; --q) {
                const uint32_t mq = a.c_meta[q];
                if (manages_execution(mq)) {
                    if (!(a.done_aware && status_done(mq))) emit(e.c_txn[q]);
                    if (meta_kind(mq) == AD_KIND_WRITE) break;
                }
                if (q == s0) break;
            }
        }
    }
}
template <bool FILL>
static __global__ __launch_bounds__(256) void k_xedges(XEdgeArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.e.n) return;
    uint32_t local = 0;
    xedges_visit(a, t, [&](uint32_t src) {
        if (FILL) a.xs[atomicAdd(&a.cur[src], 1ull)] = (uint32_t)t;
        else atomicAdd(&a.outcnt[src], 1ull);
        ++local;
    });
    if (!FILL && local) atomicAdd(&a.indeg[t], local);
}

// ---------------------------------------------------------------------------------------------------
// One-pass levels for mixed key + range batches (C4): every txn pulls its level from its sources — (a) its
// key-chain predecessor runs (the chain build in pred mode), (b)/(c) the same sources k_xedges turns into Kahn
// edges — instead of the sources pushing ~10^9 releases through the wavefronts (C4: 1.74·10^9 (b)/(c) edges, one
// returning atomic each, plus 5,650 grid-wide wavefront launches).  Every source of T has a strictly smaller
// executeAt (no ExclusiveSyncPoint / EphemeralRead in the batch: those await deps of any executeAt), so the txns
// are taken in executeAt order (k_window_rank's permutation): a grid of co-resident waves (sized from the
// occupancy) walks the ranks, wave w taking ranks w, w + W, w + 2W, ...; each txn is pulled by the whole wave,
// its lanes striding over the source lists MP_ILP loads at a time and waiting on sources not yet final.  By
// induction on the rank the lowest unfinished txn's wave is at it and every source it waits on is final, so
// nothing deadlocks, and the waiting is bounded to the resident window instead of the whole batch (the earlier
// per-txn pull of mixed batches kept ~10^6 lanes polling; 64-txn chunks per wave serialised their txns).
// The (c) sources are listed per txn beforehand (k_csrc).  A wait longer than ~1 s raises *abort; every wave
// then leaves and the caller runs the Kahn path.
struct MixPullArgs {
    size_t n;
    const uint32_t* perm;                // executeAt rank -> txn
    const uint32_t* key_off;
    const uint2* pred;                   // (a) predecessor runs per pair (PRED_TXN: one txn in .x)
    const uint32_t* c_txn;
    const uint8_t* c_meta;
    EdgeArgs e;                          // (b) merged direct / range deps; (c) merged KeyDeps + cons_pos
    int do_b, do_c;
    const unsigned long long* coff;      // (c) sources as a list per txn (k_csrc): cs[coff[t] .. coff[t + 1])
    const uint32_t* cs;
    uint32_t* L;                         // levels | LV_FINAL
    uint32_t* abort_flag;
    uint32_t* maxlvl;
    int force_abort;                     // tests (AD_LEVELS_PULL_ABORT): every wave aborts at once, Kahn recomputes
};
constexpr int MP_GRID = 2048;         // co-resident workgroups at most (8 per CU)
// the (c) sources of unmanaged t this lane owns (its share of t's merged KeyDeps keys): per key with a
// constraint position p, the Reads after the last Write at or before p and that Write (k_xedges' rule)
template <class F>
__device__ inline void mp_c_walk(const MixPullArgs& a, uint32_t t, uint32_t lane, F&& f) {
    const EdgeArgs& e = a.e;
    for (uint32_t x = e.mk_key_off[t] + lane; x < e.mk_key_off[t + 1]; x += WAVE) {
        const int32_t p = e.cons_pos[x];
        if (p < 0) continue;
        const int32_t s0 = e.seg_start[p];
        for (int32_t q = p;; --q) {
            const uint32_t mq = a.c_meta[q];
            if (manages_execution(mq)) {
                f(e.c_txn[q]);
                if (meta_kind(mq) == AD_KIND_WRITE) break;
            }
            if (q == s0) break;
        }
    }
}
// (c) source lists, one wave per txn (lanes stride its keys): count pass -> cnt[t]; fill pass (offsets scanned)
// -> each lane writes its sources after the lanes before it.  No atomics: a txn writes its own run.
template <bool FILL>
static __global__ __launch_bounds__(256) void k_csrc(MixPullArgs a, unsigned long long* __restrict__ cnt, uint32_t* __restrict__ cs) {
    const size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (t >= a.n) return;
    const uint32_t lane = (uint32_t)__lane_id();
    if (manages_execution(a.e.meta[t])) {
        if (!FILL && lane == 0) cnt[t] = 0;
        return;
    }
    uint32_t c = 0;
    mp_c_walk(a, (uint32_t)t, lane, [&](uint32_t) { ++c; });
    if (!FILL) {
        c = wave_sum(c);
        if (lane == 0) cnt[t] = c;
        return;
    }
    uint32_t inc = c;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d);
        if ((int)lane >= d) inc += y;
    }
    unsigned long long w = a.coff[t] + (inc - c);
    mp_c_walk(a, (uint32_t)t, lane, [&](uint32_t src) { cs[w++] = src; });
}
__device__ inline uint32_t mp_load(uint32_t* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// wait until L[s] is final (or the pull is abandoned: *ab); returns it
__device__ inline uint32_t mp_wait(const MixPullArgs& a, uint32_t s, uint32_t v, bool& ab) {
    uint32_t spins = 0;
    const uint64_t w0 = wall_clock64();
    while (!(v & LV_FINAL)) {
        if ((++spins & 63u) == 0u && (wall_clock64() - w0 > PULL_CAP_TICKS || mp_load(a.abort_flag) != 0u)) {
            ab = true;
            return LV_FINAL;
        }
        __builtin_amdgcn_s_sleep(2);
        v = mp_load(&a.L[s]);
    }
    return v;
}
// a heavy txn's share of one source list ids[b, e) (lane-strided), MP_ILP ids at a time: the id loads, (b) the
// executeAt filter, the level loads, then the waits — a few memory round trips per MP_ILP * 64 sources
constexpr int MP_ILP = 8;
template <bool FILTER, class I>
__device__ inline void mp_wait_list(const MixPullArgs& a, const uint32_t* __restrict__ ids, I b, I e, uint32_t lane, uint64_t my,
                                    uint32_t& m, bool& ab) {
    for (I x = b + lane; x < e && !ab; x += (I)WAVE * MP_ILP) {
        uint32_t sv[MP_ILP], lv[MP_ILP];
        bool use[MP_ILP];
#pragma unroll
        for (int u = 0; u < MP_ILP; ++u) { const I y = x + (I)u * WAVE; use[u] = y < e; sv[u] = use[u] ? ids[y] : 0u; }
        if (FILTER) {
#pragma unroll
            for (int u = 0; u < MP_ILP; ++u) use[u] = use[u] && a.e.ex1[sv[u]] < my;
        }
#pragma unroll
        for (int u = 0; u < MP_ILP; ++u) lv[u] = use[u] ? mp_load(&a.L[sv[u]]) : LV_FINAL;
#pragma unroll
        for (int u = 0; u < MP_ILP; ++u) {
            if (!use[u]) continue;
            const uint32_t v = (lv[u] & LV_FINAL) ? lv[u] : mp_wait(a, sv[u], lv[u], ab);
            const uint32_t l = (v & ~LV_FINAL) + 1u;
            m = l > m ? l : m;
        }
    }
}
static __global__ __launch_bounds__(256) void k_level_pull_mixed(MixPullArgs a) {
    const uint32_t lane = (uint32_t)__lane_id();
    const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    const size_t W = (size_t)gridDim.x * blockDim.x / WAVE;
    uint32_t wmax = 0;
    if (a.force_abort) {
        if (lane == 0) __hip_atomic_store(a.abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    for (size_t r = w; r < a.n; r += W) {
        const uint32_t t = a.perm[r];
        uint32_t m = 0;
        bool ab = false;
        // (a) predecessor runs (a handful): lane-strided over the pairs
        for (uint32_t p = a.key_off[t] + lane; p < a.key_off[t + 1] && !ab; p += WAVE) {
            const uint2 pr = a.pred[p];
            const bool one = (pr.y & PRED_TXN) != 0u;
            const uint32_t len = pr.y & ~PRED_TXN;
            for (uint32_t x = 0; x < len && !ab; ++x) {
                const uint32_t src = one ? pr.x : a.c_txn[pr.x + x];
                const uint32_t v = mp_wait(a, src, mp_load(&a.L[src]), ab);
                const uint32_t l = (v & ~LV_FINAL) + 1u;
                m = l > m ? l : m;
            }
        }
        if (a.do_b) {
            const uint64_t my = a.e.ex1[t];
#pragma unroll
            for (int c = 0; c < 2; ++c)
                if (a.e.txns[c]) {
                    const uint32_t b0 = a.e.ent_off[c][t];
                    mp_wait_list<true, uint32_t>(a, a.e.txns[c], b0, b0 + a.e.tcnt[c][t], lane, my, m, ab);
                }
        }
        if (a.do_c) mp_wait_list<false, unsigned long long>(a, a.cs, a.coff[t], a.coff[t + 1], lane, 0ull, m, ab);
        if (__ballot(ab)) {
            if (lane == 0) __hip_atomic_store(a.abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        m = wave_max(m);
        if (lane == 0) __hip_atomic_store(&a.L[t], m | LV_FINAL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wmax = m > wmax ? m : wmax;
    }
    if (lane == 0 && wmax) atomicMax(a.maxlvl, wmax);
}
// kinds a mixed pull cannot take: ExclusiveSyncPoint / EphemeralRead (their deps need not precede them in executeAt)
static __global__ __launch_bounds__(256) void k_mix_kinds(size_t n, const uint8_t* __restrict__ meta, uint32_t* __restrict__ flag) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    wave_set_flag(t < n && awaits_only_deps(meta[t]), flag);
}
// the executeAt permutation from k_window_rank: every slot filled and the keys ascending, else *bad
static __global__ __launch_bounds__(256) void k_perm_check(size_t n, const uint64_t* __restrict__ key, const uint32_t* __restrict__ perm,
                                                    uint32_t* __restrict__ bad) {
    bool b = false;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (perm[i] == 0xFFFFFFFFu || (i + 1 < n && key[i] > key[i + 1])) b = true;
    wave_set_flag(b, bad);
}

// Small device results to the host without a stream sync (the engine's host-mapped coherent buffer, see
// engine.hip read_totals_params): copy a[0..na) and b[0..nb) to pub[off..], fence, bump pub[0] = seq.
static __global__ __launch_bounds__(128) void k_publish2(const uint32_t* __restrict__ a, int na, const uint32_t* __restrict__ b, int nb,
                                                  uint32_t* pub, int off, uint32_t seq) {
    const int i = threadIdx.x;
    if (i < na) pub[off + i] = a[i];
    if (i < nb) pub[off + na + i] = b[i];
    __syncthreads();
    if (i == 0) {
        __threadfence_system();
        __hip_atomic_store(pub, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
struct Publisher {
    uint32_t* host = nullptr;           // mapped coherent host words ([0] = sequence)
    uint32_t* dev = nullptr;
    uint32_t* seq = nullptr;            // the owner's sequence counter
    int off = 0, cap = 0;               // the words this user may write: [off, off + cap)
};
// a[0..na) -> ha, b[0..nb) -> hb, waiting on the mapped buffer (else a copy + stream sync)
// between (nullable): work enqueued after the read-back and before the host waits for it (speculation)
inline bool publish_read(const Publisher& p, hipStream_t st, const uint32_t* a, int na, uint32_t* ha,
                         const uint32_t* b, int nb, uint32_t* hb, const std::function<void()>* between = nullptr) {
    if (!p.host || na + nb > p.cap || na > 128 || nb > 128) {
        if (na && hipMemcpyAsync(ha, a, (size_t)na * 4, hipMemcpyDeviceToHost, st) != hipSuccess) return false;
        if (nb && hipMemcpyAsync(hb, b, (size_t)nb * 4, hipMemcpyDeviceToHost, st) != hipSuccess) return false;
        if (between) (*between)();
        return hipStreamSynchronize(st) == hipSuccess;
    }
    const uint32_t seq = ++*p.seq;
    k_publish2<<<1, 128, 0, st>>>(a, na, b, nb, p.dev, p.off, seq);
    if (between) (*between)();
    uint64_t spins = 0;
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(p.host, __ATOMIC_ACQUIRE) != seq) {
        if ((++spins & 0x3FF) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q != hipSuccess && q != hipErrorNotReady) return false;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                if (hipStreamSynchronize(st) != hipSuccess) return false;
                if (__atomic_load_n(p.host, __ATOMIC_ACQUIRE) != seq) return false;
                break;
            }
        }
    }
    if (na) std::memcpy(ha, p.host + p.off, (size_t)na * 4);
    if (nb) std::memcpy(hb, p.host + p.off + na, (size_t)nb * 4);
    return true;
}

struct LevelState {
    size_t capP = 0, capN = 0, capK = 0;
    Publisher pub;                      // set by the engine: flag read-backs without a stream sync
    bool pull_off = false;              // AD_LEVELS_KAHN: skip the one-pass pull levels
    bool mixpull_off = false;           // AD_LEVELS_NO_MIXPULL: mixed batches straight to the Kahn wavefronts
    int mixpull_path = 0;               // last mixed pull: 0 none, 1 pulled, 2 long chain, 3 kinds, 4 rank miss, 5 aborted
    bool pull_force_abort = false;      // AD_LEVELS_PULL_ABORT (tests): every pull lane aborts, Kahn recomputes
    int pull_path = 0;                  // last pull attempt: 0 none, 1 pulled, 2 far predecessors -> Kahn, 3 aborted -> Kahn
    int kb_hint = 0;                    // wavefronts in the first Kahn launch batch (previous depth + 1)
    uint32_t* c_txn = nullptr;
    uint8_t* c_meta = nullptr;
    uint64_t* c_exec1 = nullptr;
    int32_t* pm_all = nullptr;
    uint32_t* c_pair = nullptr;         // chain position -> pair
    int32_t* pair_seg = nullptr;
    uint32_t *seg_len = nullptr, *stamp = nullptr, *heads = nullptr, *long_pos = nullptr;
    int32_t* cons_pos = nullptr;
    uint32_t *indeg = nullptr, *rem = nullptr;   // Kahn path: [n] predecessor counts (snapshot, remaining)
    uint2* succ = nullptr;                       // Kahn path: [P] successor run of each pair
    uint32_t* flags = nullptr;          // [0] heads, [1] long entries, [2] long dirty (next), [3] edge changed,
                                        // [4] max level, [5] unsupported kinds, [6] work left (next)
    void* agg = nullptr;
    size_t agg_cap = 0;
    uint32_t *sk0 = nullptr, *sv0 = nullptr, *sk1 = nullptr, *sv1 = nullptr;
    uint64_t* key64 = nullptr;           // executeAt keys of the order fast path
    uint32_t* rs = nullptr;              // radix scratch
    size_t rs_cap = 0;
    uint32_t* iflags = nullptr;          // per iteration of a launch batch: [long dirty, edge changed, work left, -]
    bool chains_ready = false;           // chain order / segment table valid for the current batch
    uint32_t nheads = 0, nlong = 0;
    // Kahn path with (b)/(c) edges: per-source out-degree, successor offsets, write cursor, successors
    unsigned long long *xcnt = nullptr, *xoff = nullptr, *xcur = nullptr;
    uint32_t* xs = nullptr;
    uint32_t* kfront = nullptr;          // k_kahn_small: two frontier lists of KS_MAX + state[4]
    size_t capX = 0, xs_cap = 0;
    BlockBufs bl;                        // deep key-chain batches: executeAt blocks (block_levels.h)
    uint32_t bl_rounds = 0;              // block scan rounds of the last block-path run
    bool bl_used = false;                // the last run_levels took the block path
    bool long_hint = false;              // the previous batch had long key chains: test for them up front
};

// The buffers order_rows needs for m rows (run_levels sizes them too; callers ordering rows without a
// run_levels pass on the handle reserve them here).
// The chain buffers of the pull pass (capP group) and the flags, before the deps stage: k_seg_fuse builds the pull
// pass's chains from its LDS copy in ad_run_pipeline (LevelInputs.chains_prebuilt); run_levels finds them reserved.
inline bool ls_reserve_chains(LevelState& ls, size_t P, hipStream_t st) {
    auto grow = [&](void** p, size_t bytes) -> bool {
        if (*p) { hipStreamSynchronize(st); hipFree(*p); *p = nullptr; }
        return hipMalloc(p, bytes) == hipSuccess;
    };
    if (ls.capP < P || !ls.c_txn) {
        const size_t c = std::max<size_t>(P, 1);
        if (!grow((void**)&ls.c_txn, c * 4) || !grow((void**)&ls.c_meta, c) || !grow((void**)&ls.c_exec1, c * 8) ||
            !grow((void**)&ls.pm_all, c * 4) || !grow((void**)&ls.c_pair, c * 4) || !grow((void**)&ls.succ, c * 8) ||
            !grow((void**)&ls.pair_seg, c * 4) || !grow((void**)&ls.seg_len, c * 4) || !grow((void**)&ls.stamp, c * 4) ||
            !grow((void**)&ls.heads, c * 4) || !grow((void**)&ls.long_pos, c * 4))
            return false;
        ls.capP = c;
    }
    if (!ls.flags && !grow((void**)&ls.flags, 256)) return false;
    return true;
}
inline bool ls_reserve_order(LevelState& ls, size_t m, hipStream_t st) {
    auto grow = [&](void** p, size_t bytes) -> bool {
        if (*p) { hipStreamSynchronize(st); hipFree(*p); *p = nullptr; }
        return hipMalloc(p, bytes) == hipSuccess;
    };
    if (ls.capN < m || !ls.sk0) {
        const size_t c = std::max<size_t>(m, 1);
        if (!grow((void**)&ls.sk0, c * 4) || !grow((void**)&ls.sv0, c * 4) || !grow((void**)&ls.sk1, c * 4) ||
            !grow((void**)&ls.sv1, c * 4) || !grow((void**)&ls.key64, c * 8) || !grow((void**)&ls.indeg, c * 4) ||
            !grow((void**)&ls.rem, c * 4))
            return false;
        ls.capN = c;
    }
    if (!ls.flags && !grow((void**)&ls.flags, 256)) return false;
    const size_t rneed = (3 * (radix_hist_len(std::max<size_t>(m, 1)) + 128) + 64 * 1024) * 4;
    if (ls.rs_cap < rneed) {
        if (!grow((void**)&ls.rs, rneed)) return false;
        ls.rs_cap = rneed;
    }
    return true;
}

inline void free_level_state(LevelState& s) {
    void* ps[] = {s.c_txn, s.c_meta, s.c_pair, s.c_exec1, s.indeg, s.rem, s.succ, s.pm_all, s.pair_seg, s.seg_len, s.stamp, s.heads, s.long_pos, s.iflags, s.cons_pos, s.flags, s.agg, s.sk0, s.sv0, s.sk1, s.sv1, s.key64, s.rs, s.xcnt, s.xoff, s.xcur, s.xs, s.kfront};
    for (void* p : ps) if (p) hipFree(p);
    free_block_bufs(s.bl);
    s = LevelState{};
}

inline size_t level_scratch_bytes(size_t, size_t) { return 0; }

struct LevelInputs {
    size_t n, P;
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const int32_t* seg_start;
    const uint32_t* sval;                // sorted position -> pair
    const uint32_t* nh;                  // non-head entries (ElideOp), P - prm->n_keys_u of them
    const uint32_t* sec = nullptr;       // or k_seg_fuse's per-tile second-entry lists (sec_cap per tile, sec_cnt each)
    const uint32_t* sec_cnt = nullptr;
    int sec_cap = 0;
    uint32_t sec_tiles = 0;
    const Params* prm;
    const uint32_t* key_off;
    const uint8_t* meta;
    const uint64_t* ex1;
    uint32_t* lvl;
    uint32_t* order;
    const DevCsr* merged_key;
    const DevCsr* merged_direct;
    const DevCsr* merged_range;
    const uint64_t* ukey;
    const uint32_t* useg;
    uint32_t U;
    uint32_t n_large;
    uint32_t n_special;                  // key-domain sync points / ephemeral reads (unmanaged execution)
    uint32_t exec_bits;
    int keep_levels;                     // sharded rounds: start from the given levels, reuse the chains
    int kahn_ok;                         // single-store batch: the Kahn wavefront may replace the fixpoint
    int chains_prebuilt = 0;             // k_seg_fuse built the pull pass's chains (succ, c_txn, flags 7 / 18) and k_pack
                                         // zeroed succ and the flags before it: the pull pass skips k_chain_build
    int force_blocks;                    // pure key-chain batches: executeAt blocks even for short chains (tests)
    int wide_words;                      // block path: 64-bit scan words even for batches of <= 2^20 txns (tests)
    int (*complete)(void*);              // nullable: fills in every sorted entry before a path other than the pull pass
    void* complete_ctx;
    uint32_t* order_verify;              // optimistic order: host-mapped word (device address) receiving the fast-path
                                         // failure flag; null: the order syncs on its own check
    bool* order_pending;                 // set when the caller must check *order_verify after its sync
};

// Execution order over m txns (rows[k], or k when rows is null): LSD radix sort by executeAt (two 32-bit
// halves) then stably by level; order_out[k'] = k of the k'-th txn.  ls.sk*/sv*/rs must hold m entries.
static __global__ __launch_bounds__(256) void k_exec_split_rows(size_t m, const uint64_t* __restrict__ ex1, const uint32_t* __restrict__ rows,
                                                         const uint32_t* __restrict__ perm, uint32_t* __restrict__ key, int hi) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t k = perm ? perm[i] : (uint32_t)i;
    const uint64_t e = ex1[rows ? rows[k] : k] - 1;
    key[i] = hi ? (uint32_t)(e >> 32) : (uint32_t)e;
}

// Near-sorted fast path for the executeAt order: executeAt == TxnId on the fast path and a slow-path bump
// moves a txn only a few ranks, so every inversion of the TxnId order is between ranks less than WR_D
// apart.  Then each txn's rank in (executeAt, row) order is its row index corrected by the inversions
// inside a +-WR_D window:  rank_i = i + #{j in (i, i+D] : e_j < e_i} - #{j in [i-D, i) : e_j > e_i}
// (one LDS tile of 1024 rows plus halos per block, 128 compares per row), and the row is scattered to
// its rank together with its executeAt and level.  A check pass verifies that every slot was written
// (no collision, via a sentinel) and that the keys ascend; otherwise the full LSD radix sort runs.
constexpr int WR_N = 1024, WR_D = 64, WR_T = 256;
constexpr uint32_t WR_EMPTY = 0xFFFFFFFFu;
// strip != null (== lvl, rows == null: the pull pass's levels): the levels' LV_FINAL bit cleared here, written back
// (k_level_strip's pass folded into this one)
static __global__ __launch_bounds__(WR_T) void k_window_rank(size_t m, const uint64_t* __restrict__ ex1, const uint32_t* __restrict__ rows,
                                                      const uint32_t* lvl, uint64_t* __restrict__ okey,
                                                      uint32_t* __restrict__ oidx, uint32_t* __restrict__ olvl,
                                                      uint32_t* __restrict__ bad, uint32_t* strip = nullptr) {
    __shared__ uint64_t sk[WR_N + 2 * WR_D];
    const long base = (long)blockIdx.x * WR_N;
    for (int x = threadIdx.x; x < WR_N + 2 * WR_D; x += WR_T) {
        const long g = base + x - WR_D;
        // out-of-range neighbours: 0 before the batch (never greater), ~0 after it (never smaller)
        sk[x] = g < 0 ? 0ull : (g >= (long)m ? ~0ull : ex1[rows ? rows[g] : (size_t)g]);
    }
    __syncthreads();
    bool oob = false;
    for (int e = threadIdx.x; e < WR_N; e += WR_T) {
        const long i = base + e;
        if (i >= (long)m) break;
        const uint64_t key = sk[e + WR_D];
        int r = 0;
#pragma unroll 16
        for (int k = 1; k <= WR_D; ++k) {
            r += sk[e + WR_D + k] < key ? 1 : 0;
            r -= sk[e + WR_D - k] > key ? 1 : 0;
        }
        uint32_t lv = lvl[rows ? rows[i] : (size_t)i];
        if (strip) { lv &= ~LV_FINAL; strip[i] = lv; }
        const long rank = i + r;
        if (rank < 0 || rank >= (long)m) { oob = true; continue; }
        okey[rank] = key;
        oidx[rank] = (uint32_t)i;
        olvl[rank] = lv;
    }
    wave_set_flag(oob, bad);
}
// flags[0] = max level, flags[1] |= 1 unless okey ascends and every slot is filled
static __global__ __launch_bounds__(256) void k_rank_check(size_t m, const uint64_t* __restrict__ okey, const uint32_t* __restrict__ oidx,
                                                    const uint32_t* __restrict__ olvl, uint32_t* __restrict__ flags,
                                                    uint32_t* fail_out, uint32_t max_level) {
    uint32_t v = 0;
    bool bad = false;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) {
        if (oidx[i] == WR_EMPTY) { bad = true; continue; }
        const uint32_t x = olvl[i];
        v = x > v ? x : v;
        if (i + 1 < m && okey[i] > okey[i + 1]) bad = true;
    }
    v = wave_max(v);
    const bool wbad = __ballot(bad) != 0;
    __shared__ uint32_t red[256 / WAVE], rb[256 / WAVE];
    if (__lane_id() == 0) { red[threadIdx.x / WAVE] = v; rb[threadIdx.x / WAVE] = wbad ? 1u : 0u; }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t mx = red[0], b = rb[0];
        for (int k = 1; k < 256 / WAVE; ++k) { mx = mx > red[k] ? mx : red[k]; b |= rb[k]; }
        atomicMax(&flags[0], mx);
        if (mx > max_level) b = 1;                                 // the optimistic level pass was too narrow
        if (b) atomicOr(&flags[1], 1u);
        if (b && fail_out) *(volatile uint32_t*)fail_out = 1u;    // host-mapped: read after the caller's sync
    }
}
// The optimistic order's check fused into the level pass's digit histogram (levels <= 255: one 8-bit digit): per
// RS_TILE tile of the executeAt-rank-ordered rows, the level histogram k_radix_hist writes, and k_rank_check's
// verification (every slot filled, executeAt ascending, no level above the assumed depth) on the same reads.
static __global__ __launch_bounds__(RS_BLOCK) void k_rank_check_hist(size_t m, const uint64_t* __restrict__ okey,
                                                                     const uint32_t* __restrict__ oidx,
                                                                     const uint32_t* __restrict__ olvl, int ntiles,
                                                                     uint32_t* __restrict__ hist, uint32_t* __restrict__ flags,
                                                                     uint32_t* fail_out, uint32_t max_level) {
    __shared__ uint32_t h[RS_WAVES][256];
    __shared__ uint32_t red[RS_WAVES], rb[RS_WAVES];
    const int w = threadIdx.x / WAVE;
    for (int i = threadIdx.x; i < RS_WAVES * 256; i += RS_BLOCK) (&h[0][0])[i] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
    uint32_t v = 0;
    bool bad = false;
#pragma unroll 4
    for (int k = 0; k < RS_ITEMS; ++k) {
        const size_t i = base + (size_t)k * RS_BLOCK + threadIdx.x;
        if (i < m) {
            const uint32_t x = olvl[i];
            atomicAdd(&h[w][x & 0xFF], 1u);
            v = x > v ? x : v;
            if (oidx[i] == WR_EMPTY || (i + 1 < m && okey[i] > okey[i + 1])) bad = true;
        }
    }
    v = wave_max(v);
    const bool wbad = __ballot(bad) != 0;
    if (__lane_id() == 0) { red[w] = v; rb[w] = wbad ? 1u : 0u; }
    __syncthreads();
    for (int d = threadIdx.x; d < 256; d += RS_BLOCK) {
        uint32_t c = 0;
#pragma unroll
        for (int x = 0; x < RS_WAVES; ++x) c += h[x][d];
        hist[(size_t)d * ntiles + blockIdx.x] = c;
    }
    if (threadIdx.x == 0) {
        uint32_t mx = red[0], b = rb[0];
        for (int k = 1; k < RS_WAVES; ++k) { mx = mx > red[k] ? mx : red[k]; b |= rb[k]; }
        atomicMax(&flags[0], mx);
        if (mx > max_level) b = 1;
        if (b) atomicOr(&flags[1], 1u);
        if (b && fail_out) *(volatile uint32_t*)fail_out = 1u;    // host-mapped: read after the caller's sync
    }
}

// level of each txn in `perm` order (dst) + max level (fallback path).  Grid-stride over a bounded grid:
// one atomic per block.
constexpr int ORDER_GRID = 1024;
static __global__ __launch_bounds__(256) void k_gather_level_rows(size_t m, const uint32_t* __restrict__ lvl, const uint32_t* __restrict__ rows,
                                                           const uint32_t* __restrict__ perm, uint32_t* __restrict__ dst,
                                                           uint32_t* __restrict__ flags) {
    uint32_t v = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t k = perm[i];
        const uint32_t x = lvl[rows ? rows[k] : k];
        dst[i] = x;
        v = x > v ? x : v;
    }
    v = wave_max(v);
    __shared__ uint32_t red[256 / WAVE];
    if (__lane_id() == 0) red[threadIdx.x / WAVE] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t mx = red[0];
        for (int k = 1; k < 256 / WAVE; ++k) mx = mx > red[k] ? mx : red[k];
        atomicMax(&flags[0], mx);
    }
}

// Returns true when the order was produced optimistically (known_maxl >= 0: the level count is known,
// so no host sync is needed here): the fast path's verification failure is then stored by k_rank_check into
// *verify_dev (a host-mapped word the caller zeroed; a device-to-pageable copy here would stall the stream for
// a host round trip), and the caller, after its own stream sync, reruns order_rows with known_maxl = -1 if set.
// prefilled: the caller's earlier fill already cleared ls.flags[8..9] and set ls.sv0 to the sentinel (the pull path)
// strip: lvl holds the pull pass's levels with their LV_FINAL bits (rows == null): k_window_rank clears them
inline bool order_rows(LevelState& ls, size_t m, const uint32_t* rows, const uint64_t* ex1, const uint32_t* lvl,
                       uint32_t exec_bits, uint32_t* order_out, hipStream_t st, int known_maxl = -1,
                       uint32_t* verify_dev = nullptr, bool prefilled = false, bool strip = false) {
    KScope ks(K_ORDER, m);
    RadixScratch rs;
    const size_t hl = radix_hist_len(m);
    rs.hist = ls.rs;
    rs.offs = rs.hist + hl + 64;
    rs.agg = rs.offs + hl + 64;
    const int g = ceil_div((long)m, 256);
    uint32_t *k = ls.sk0, *v = ls.sv0, *ko = ls.sk1, *vo = ls.sv1;
    uint32_t* of = ls.flags + 8;                              // [0] max level, [1] fast path failed
    const int gg = std::min(g, ORDER_GRID);
    const bool optimistic = known_maxl >= 0 && verify_dev != nullptr;
    uint32_t fl[2] = {0, 0};
    // fast path: windowed inversion ranks + verification
    if (!prefilled) fill_multi(st, {{of, 8, 0}, {v, m * 4, 0xFF}});   // flags; WR_EMPTY: detects rank collisions
    k_window_rank<<<ceil_div((long)m, WR_N), WR_T, 0, st>>>(m, ex1, rows, lvl, ls.key64, v, k, of + 1,
                                                            strip && !rows ? const_cast<uint32_t*>(lvl) : nullptr);
    if (optimistic && known_maxl > 0 && known_maxl <= 255) {
        // one stable pass by level whose histogram kernel is also the check, written straight into order_out
        const int ntiles = ceil_div((long)m, RS_TILE);
        k_rank_check_hist<<<ntiles, RS_BLOCK, 0, st>>>(m, ls.key64, v, k, ntiles, rs.hist, of, verify_dev,
                                                       (uint32_t)known_maxl);
        k_radix_rowscan<<<256, 1024, 0, st>>>(rs.hist, ntiles, rs.offs, rs.agg);
        k_radix_scatter<<<ntiles, RS_BLOCK, 0, st>>>(k, v, ko, order_out, m, 0, ntiles, rs.offs, rs.agg);
        return true;
    }
    k_rank_check<<<gg, 256, 0, st>>>(m, ls.key64, v, k, of, optimistic ? verify_dev : nullptr,
                                     optimistic ? (uint32_t)known_maxl : 0xFFFFFFFFu);
    if (optimistic) {
        fl[0] = (uint32_t)known_maxl;
    } else {
        hipMemcpyAsync(fl, of, 8, hipMemcpyDeviceToHost, st);
        hipStreamSynchronize(st);
    }
    if (fl[1]) {
        // general executeAt distribution: LSD radix sort by executeAt (two 32-bit halves)
        const int eb = (int)exec_bits;
        k_exec_split_rows<<<g, 256, 0, st>>>(m, ex1, rows, nullptr, k, 0);
        k_iota<<<g, 256, 0, st>>>(m, v);
        if (radix_sort_pairs(k, v, ko, vo, m, eb < 32 ? eb : 32, rs, st)) { std::swap(k, ko); std::swap(v, vo); }
        if (eb > 32) {
            k_exec_split_rows<<<g, 256, 0, st>>>(m, ex1, rows, v, k, 1);
            if (radix_sort_pairs(k, v, ko, vo, m, eb - 32, rs, st)) { std::swap(k, ko); std::swap(v, vo); }
        }
        k_gather_level_rows<<<gg, 256, 0, st>>>(m, lvl, rows, v, k, of);
    }
    const uint32_t maxl = fl[0];
    const int lb = maxl == 0 ? 0 : 32 - __builtin_clz(maxl);
    if (lb > 0 && lb <= 8) {         // one stable pass by level, written straight into order_out
        radix_sort_pairs(k, v, ko, order_out, m, lb, rs, st);
        return optimistic;
    }
    if (radix_sort_pairs(k, v, ko, vo, m, lb, rs, st)) { std::swap(k, ko); std::swap(v, vo); }
    hipMemcpyAsync(order_out, v, m * 4, hipMemcpyDeviceToDevice, st);
    return optimistic;
}

// Levels of a pure key-chain batch (no direct / range deps, no range txns) by executeAt blocks.  Leaves the
// levels in in.lvl; *depth = greatest level + 1; *rounds_out = scan rounds over all blocks.
inline int run_block_levels(LevelState& ls, BlockBufs& bb, const LevelInputs& in, hipStream_t st, int* depth,
                            uint32_t* rounds_out, std::string& err) {
    const size_t n = in.n, P = in.P;
    auto grow = [&](void** p, size_t bytes) -> bool {
        if (*p) { hipStreamSynchronize(st); hipFree(*p); *p = nullptr; }
        return hipMalloc(p, bytes) == hipSuccess;
    };
    const uint32_t bcap = BL_CAP - 16;         // n_large == 0: at most 16 keys per txn
    const size_t B = P / bcap + 2;             // upper bound on blocks (the entry prefix counts key-less txns too)
    const size_t Bmax = (P + n) / bcap + 2;
    if (bb.capP < P || !bb.rec || !bb.tl) {
        const size_t c = std::max<size_t>(P, 1);
        if (!grow((void**)&bb.rec, c * 8) || !grow((void**)&bb.bk, c * 4) || !grow((void**)&bb.bv, c * 4) ||
            !grow((void**)&bb.bk2, c * 4) || !grow((void**)&bb.bv2, c * 4) || !grow((void**)&bb.carry, c * 8) ||
            !grow((void**)&bb.crec, c * 16) || !grow((void**)&bb.la, c * 8) || !grow((void**)&bb.lb, c * 4) ||
            !grow((void**)&bb.tl, c * 4))
            goto oom;
        bb.capP = c;
    }
    if (bb.capN < n + 1 || !bb.epre) {
        const size_t c = n + 1;
        if (!grow((void**)&bb.epre, c * 4) || !grow((void**)&bb.erank, c * 4)) goto oom;
        bb.capN = c;
    }
    if (bb.capB < Bmax + 1 || !bb.tb) {
        const size_t c = Bmax + 1;
        if (!grow((void**)&bb.tb, c * 4) || !grow((void**)&bb.boff, c * 4) || !grow((void**)&bb.mt, c * 4) ||
            !grow((void**)&bb.lcnt, c * 4))
            goto oom;
        bb.capB = c;
    }
    if (!bb.stats && !grow((void**)&bb.stats, BL_STATS_BYTES)) goto oom;
    {
        const size_t rneed = (3 * (radix_hist_len(std::max<size_t>(P, 1)) + 128) + 64 * 1024) * 4;
        if (bb.rs_cap < rneed) { if (!grow((void**)&bb.rs, rneed)) goto oom; bb.rs_cap = rneed; }
        const size_t sneed = device_scan_scratch<BlCntOp>(n) + 256;
        if (ls.agg_cap < sneed) { if (!grow(&ls.agg, sneed)) goto oom; ls.agg_cap = sneed; }
    }
    (void)B;
    {
        const int gP = ceil_div((long)P, 256), gn = ceil_div((long)n, 256);
        // 1. chain order (key, executeAt): windowed inversion ranks, else the serial per-key insertion
        hipMemsetAsync(ls.c_pair, 0xFF, P * 4, st);
        hipMemsetAsync(bb.stats, 0, BL_STATS_BYTES, st);
        k_chain_rank<<<ceil_div((long)P, CR_N), CR_T, 0, st>>>(P, in.seg_start, in.e_txn, in.e_meta, in.e_exec1, in.sval,
                                                               ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
        k_chain_check<<<std::min(gP, 2048), 256, 0, st>>>(P, in.seg_start, ls.c_exec1, ls.c_pair, bb.stats + 2);
        // 2. executeAt order of the txns (levels all zero: order_rows sorts by executeAt only)
        hipMemsetAsync(in.lvl, 0, n * 4, st);
        order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st);    // syncs: reads its own flags
        uint32_t bad = 0;
        if (hipMemcpyAsync(&bad, bb.stats + 2, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
            err = "exec levels: device error";
            return AD_ERR_DEVICE;
        }
        if (bad) {
            k_chain_copy<<<gP, 256, 0, st>>>(P, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
            k_chain_order<<<gP, 256, 0, st>>>(P, in.seg_start, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
        }
        // 3. blocks: entry prefix in executeAt order, block of every chain position, stable sort by block
        k_bl_erank<<<gn, 256, 0, st>>>(n, in.order, bb.erank);
        device_scan(BlCntOp{in.order, in.key_off, bb.epre, n}, n, (uint32_t*)ls.agg, st);
        uint32_t etot = 0;
        if (hipMemcpyAsync(&etot, bb.epre + n, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
            err = "exec levels: device error";
            return AD_ERR_DEVICE;
        }
        const uint32_t nb = etot / bcap + 1;
        bb.nblocks = nb;
        const uint32_t* tlq = nullptr;           // lb: free until compact
        if (nb + 1 <= (uint32_t)BL_TB_LDS) {
            k_bl_tbounds<<<ceil_div((long)nb + 1, 256), 256, 0, st>>>(nb, n, bb.epre, bcap, bb.tb);
            k_bl_chain_block_tb<<<std::min(gP, 2048), 256, 0, st>>>(P, nb, ls.c_txn, bb.erank, bb.tb, bb.bk, bb.bv, bb.lb, bb.tl);
            tlq = bb.tl;
        } else {
            k_bl_chain_block<<<gP, 256, 0, st>>>(P, ls.c_txn, bb.erank, bb.epre, bcap, bb.bk, bb.bv, bb.lb);
        }
        RadixScratch rs;
        const size_t hl = radix_hist_len(P);
        rs.hist = bb.rs;
        rs.offs = rs.hist + hl + 64;
        rs.agg = rs.offs + hl + 64;
        uint32_t *sk = bb.bk, *sv = bb.bv;
        const int bits = 32 - __builtin_clz(std::max<uint32_t>(nb, 1));
        if (radix_sort_pairs(bb.bk, bb.bv, bb.bk2, bb.bv2, P, bits, rs, st)) { sk = bb.bk2; sv = bb.bv2; }
        k_bl_bounds<<<ceil_div((long)nb + 1, 256), 256, 0, st>>>(nb, n, P, bb.epre, bcap, sk, bb.tb, bb.boff);
        uint32_t* inv = sk == bb.bk ? bb.bk2 : bb.bk;         // the sort's free ping-pong buffer
        k_bl_inverse<<<gP, 256, 0, st>>>(P, sv, inv);
        k_bl_records<<<gP, 256, 0, st>>>(P, bb.lb, inv, ls.c_txn, ls.c_meta, in.seg_start, bb.erank, bb.tb, bb.boff, bb.rec,
                                         bb.stats + BL_STAT_RECORDS_BAD, tlq);
        k_bl_compact<<<nb, BL_T, 0, st>>>(nb, bb.boff, bb.rec, bb.crec, bb.mt, bb.la, bb.lb, bb.lcnt);
        // 4. the walk (packed scan words: 32-bit while every level fits 20 bits)
        // (no carry initialisation: a head reads a global carry only from a producer flagged to store it)
        uint32_t* Lr = bb.erank;                   // free after the records: the levels by executeAt rank
        if (n <= (1u << 20) && !in.wide_words)
            k_level_blocks<uint32_t><<<1, BL_WT, 0, st>>>(nb, bb.boff, bb.tb, bb.rec, bb.crec, bb.mt, bb.la, bb.lb, bb.lcnt, bb.carry, Lr,
                                                              bb.stats);
        else
            k_level_blocks<uint64_t><<<1, BL_WT, 0, st>>>(nb, bb.boff, bb.tb, bb.rec, bb.crec, bb.mt, bb.la, bb.lb, bb.lcnt, bb.carry, Lr,
                                                              bb.stats);
        k_bl_scatter<<<ceil_div((long)n, 256), 256, 0, st>>>(n, in.order, Lr, in.lvl);
        uint32_t s4[BL_STATS_BYTES / 4] = {};
        if (hipMemcpyAsync(s4, bb.stats, BL_STATS_BYTES, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
            err = "exec levels: device error";
            return AD_ERR_DEVICE;
        }
        if (s4[BL_STAT_RECORDS_BAD]) {
            err = "exec levels: block layout invariant violated (txn index beyond the block)";
            return AD_ERR_STATE;
        }
        if (s4[6]) {
            err = "exec levels: a block's rounds did not converge";
            return AD_ERR_STATE;
        }
        *depth = (int)s4[0];
        if (rounds_out) *rounds_out = s4[1];
        if (getenv("AD_DEBUG_LEVELS")) {
            uint32_t s6[16];
            hipMemcpy(s6, bb.stats, 64, hipMemcpyDeviceToHost);
            const double tr = (double)((uint64_t)s6[3] << 32 | s6[2]), tt = (double)((uint64_t)s6[5] << 32 | s6[4]);
            fprintf(stderr, "block levels: %u blocks, %u rounds, depth %u; clock64 rounds %.0f (%.1f%%) of %.0f; W0 waited %.0f, "
                            "W0 lists %.0f; workers' phase work %.0f (retire %.0f, clear %.0f, stage %.0f); rounds' init %.0f, "
                            "carry-out %.0f; entries per lane %.2f\n", nb, s6[1],
                    s6[0], tr, 100.0 * tr / (tt > 0 ? tt : 1), tt, 256.0 * s6[7], 256.0 * s6[8], 256.0 * s6[9],
                    256.0 * s6[10], 256.0 * s6[11], 256.0 * s6[12], 256.0 * s6[13], 256.0 * s6[14], (double)s6[15] / nb);
        }
    }
    return AD_OK;
oom:
    err = "exec levels: out of device memory";
    return AD_ERR_NOMEM;
}

inline bool level_strip_pass() {
    static const bool on = [] { const char* e = getenv("AD_LEVEL_STRIP"); return e && e[0] == '1'; }();
    return on;
}
inline int run_levels(LevelState& ls, const LevelInputs& in, bool want_order, hipStream_t st, int* iters,
                      std::string& err) {
    const size_t n = in.n, P = in.P;
    auto grow = [&](void** p, size_t bytes) -> bool {
        if (*p) { hipStreamSynchronize(st); hipFree(*p); *p = nullptr; }
        if (hipMalloc(p, bytes) != hipSuccess) { *p = nullptr; return false; }
        return true;
    };
    const size_t nkm = in.merged_key ? in.merged_key->nkeys : 0;
    if (ls.capP < P || !ls.c_txn) {
        size_t c = std::max<size_t>(P, 1);
        if (!grow((void**)&ls.c_txn, c * 4) || !grow((void**)&ls.c_meta, c) || !grow((void**)&ls.c_exec1, c * 8) ||
            !grow((void**)&ls.pm_all, c * 4) || !grow((void**)&ls.c_pair, c * 4) || !grow((void**)&ls.succ, c * 8) || !grow((void**)&ls.pair_seg, c * 4) || !grow((void**)&ls.seg_len, c * 4) ||
            !grow((void**)&ls.stamp, c * 4) || !grow((void**)&ls.heads, c * 4) || !grow((void**)&ls.long_pos, c * 4))
            goto oom;
        ls.capP = c;
    }
    if (ls.capN < n || !ls.sk0) {
        size_t c = std::max<size_t>(n, 1);
        if (!grow((void**)&ls.sk0, c * 4) || !grow((void**)&ls.sv0, c * 4) || !grow((void**)&ls.sk1, c * 4) ||
            !grow((void**)&ls.sv1, c * 4) || !grow((void**)&ls.key64, c * 8) ||
            !grow((void**)&ls.indeg, c * 4) || !grow((void**)&ls.rem, c * 4))
            goto oom;
        ls.capN = c;
    }
    if (ls.capK < nkm || !ls.cons_pos) {
        size_t c = std::max<size_t>(nkm, 1);
        if (!grow((void**)&ls.cons_pos, c * 4)) goto oom;
        ls.capK = c;
    }
    if (!ls.flags && !grow((void**)&ls.flags, 256)) goto oom;
    if (!ls.iflags && !grow((void**)&ls.iflags, 4 * 64 * 4)) goto oom;
    {
        const size_t need = std::max(std::max(device_scan_scratch<ChainOp>(std::max<size_t>(P, 1)),
                                              device_scan_scratch<SegListOp>(std::max<size_t>(P, 1))),
                                     device_scan_scratch<SumOp<unsigned long long>>(std::max<size_t>(n, 1))) + 256;
        if (ls.agg_cap < need) { if (!grow(&ls.agg, need)) goto oom; ls.agg_cap = need; }
        const size_t rneed = (3 * (radix_hist_len(std::max<size_t>(n, 1)) + 128) + 64 * 1024) * 4;
        if (ls.rs_cap < rneed) { if (!grow((void**)&ls.rs, rneed)) goto oom; ls.rs_cap = rneed; }
    }

    ls.pull_path = 0;
    ls.mixpull_path = 0;
    {
        // flags; levels (unless given); the pull path's predecessor runs (zero: none) for pure key batches
        const bool pull_try = in.kahn_ok && !in.keep_levels && P > 0 && !ls.pull_off && in.n_large == 0 && in.n_special == 0 &&
                              !(in.merged_direct && in.merged_direct->ncap > 0) && !(in.merged_range && in.merged_range->ncap > 0);
        // (and the pull path's order: its collision sentinel, order_rows prefilled)
        const bool pre = in.chains_prebuilt && pull_try;
        fill_multi(st, {{pre ? nullptr : ls.flags, 128, 0}, {in.keep_levels ? nullptr : in.lvl, std::max<size_t>(n, 1) * 4, 0},
                        {pull_try && !pre ? ls.succ : nullptr, P * 8, 0}, {pull_try ? ls.sv0 : nullptr, n * 4, 0xFF}});
        // local-only txns are key-domain specials (n_special): a pull batch has none
        if (n > 0 && !pull_try) k_level_kinds<<<ceil_div((long)n, 256), 256, 0, st>>>(n, in.meta, ls.flags + 5);
    }
    *iters = 0;
    {
        // ---- chain order, segment table, pair -> segment, long-segment positions, (c) constraints
        const int gP = ceil_div((long)std::max<size_t>(P, 1), 256);
        const int gCB = ceil_div((long)std::max<size_t>(P, 1), CB_SPAN);     // k_chain_build without nh
        const int cb_grid = in.sec ? (int)ceil_div((long)std::max<uint32_t>(in.sec_tiles, 1), 4) : in.nh ? gP : gCB;
        const bool has_b = (in.merged_direct && in.merged_direct->ncap > 0) || (in.merged_range && in.merged_range->ncap > 0);
        const bool has_c = (in.n_large > 0 || in.n_special > 0) && nkm > 0 && P > 0;
        PushCtx push{};
        push.key_off = in.key_off; push.pair_seg = ls.pair_seg; push.seg_len = ls.seg_len; push.stamp = ls.stamp;
        push.long_dirty = ls.flags + 2;
        EdgeArgs ea{};
        ea.n = n; ea.meta = in.meta; ea.ex1 = in.ex1; ea.L = in.lvl; ea.changed = ls.flags + 3; ea.work_left = ls.flags + 6;
        const DevCsr* bc[2] = {in.merged_direct, in.merged_range};
        for (int c = 0; c < 2; ++c) {
            if (bc[c] && bc[c]->ncap > 0) { ea.ent_off[c] = bc[c]->ent_off; ea.tcnt[c] = bc[c]->tcnt; ea.txns[c] = bc[c]->txns; }
        }
        if (in.merged_key) {
            ea.mk_key_off = in.merged_key->key_off; ea.mk_keys = in.merged_key->keys; ea.mk_k2t_off = in.merged_key->k2t_off;
            ea.mk_k2t = in.merged_key->k2t; ea.mk_ent_off = in.merged_key->ent_off; ea.mk_txns = in.merged_key->txns;
        }
        ea.cons_pos = ls.cons_pos; ea.pm_all = ls.pm_all; ea.ukey = in.ukey; ea.useg = in.useg; ea.U = in.U;
        ea.c_exec1 = ls.c_exec1; ea.c_txn = ls.c_txn; ea.seg_start = in.seg_start;
        ea.e_txn = in.e_txn; ea.e_meta = in.e_meta; ea.e_exec1 = in.e_exec1;
        uint32_t host[8] = {0};
        // ---- executeAt blocks (block_levels.h): pure key-chain batches whose chains are long (found by the
        // Kahn chain build below), or always when forced
        const bool pure = !has_b && !has_c && in.n_large == 0 && in.n_special == 0;
        auto block_path = [&]() -> int {
            int depth = 0;
            uint32_t rounds = 0;
            int rc;
            {
                KScope ks(K_BLOCK_LEVELS, P);
                rc = run_block_levels(ls, ls.bl, in, st, &depth, &rounds, err);
            }
            if (rc != AD_OK) return rc;
            ls.bl_rounds = rounds;
            ls.bl_used = true;
            ls.chains_ready = false;
            *iters = depth;
            if (want_order && n > 0 && in.order_verify)
                *in.order_pending = order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st, depth - 1, in.order_verify);
            else if (want_order && n > 0)
                order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st);
            return AD_OK;
        };
        if (in.force_blocks && pure && !in.keep_levels && P > 0) {
            if (hipMemcpyAsync(host, ls.flags, 32, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
                err = "exec levels: device error";
                return AD_ERR_DEVICE;
            }
            if (host[5]) {
                err = "exec levels: local-only txns are not part of the batch execution order";
                return AD_ERR_UNSUPPORTED;
            }
            return block_path();
        }
        // a handle whose previous batch had long chains (C3's stream) tests for them with one light kernel and
        // goes straight to the block path, instead of a pull pass that would find them and be discarded
        if (ls.long_hint && pure && !in.keep_levels && P > 0 && in.kahn_ok && !ls.pull_off) {
            k_any_long_seg<<<ceil_div((long)P, 256), 256, 0, st>>>(P, in.seg_start, ls.flags + 7);
            if (hipMemcpyAsync(host, ls.flags, 32, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
                err = "exec levels: device error";
                return AD_ERR_DEVICE;
            }
            if (host[7] && !host[5]) {
                hipMemsetAsync(ls.flags + 7, 0, 4, st);
                if (in.complete && in.complete(in.complete_ctx) != AD_OK) {   // the block path reads every entry
                    err = "exec levels: device error";
                    return AD_ERR_DEVICE;
                }
                return block_path();
            }
            if (host[7]) hipMemsetAsync(ls.flags + 7, 0, 4, st);
            ls.long_hint = false;
        }
        // ---- Kahn wavefront (short-chain key batches): chain build + wavefronts with no decision sync;
        // the first batch's readback also carries the kinds / long-chain flags, and a long chain found by
        // the build sends the batch to the fixpoint below
        // key-domain sync points / ephemeral reads sit in the key segments but not in the execution chains:
        // the chain build of this path treats every key entry as a Read or Write, so such batches resolve on
        // the relaxation path below (its chain scans skip unmanaged entries)
        // ---- one-pass pull levels: pure key batches (no (b)/(c) edges); long chains go to the block path,
        // an abort (a lane waited ~1 s) to the Kahn wavefronts below
        if (in.kahn_ok && !in.keep_levels && P > 0 && pure && !ls.pull_off) {
            ls.chains_ready = false;
            uint32_t lng = 0, res[3] = {0, 0, 0};
            {
                {
                KScope ks(K_KAHN, P);
                const int gn = ceil_div((long)n, 256);
                // predecessor runs zeroed above; ls.flags [16] abort, [17] max level, [18] far pred (zeroed above)
                if (!in.chains_prebuilt)
                    k_chain_build<<<cb_grid, 256, 0, st>>>(P, in.nh, in.prm, in.seg_start, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn,
                                                      ls.c_meta, ls.c_exec1, ls.c_pair, ls.indeg, ls.succ, ls.flags + 7, 0, 1,
                                                      ls.flags + 18, in.sec, in.sec_cnt, in.sec_cap, in.sec_tiles);
                k_level_pull<<<gn, 256, 0, st>>>(n, in.key_off, ls.succ, ls.c_txn, in.lvl, ls.flags + 7, ls.flags + 18, ls.flags + 16,
                                                 ls.sk1, ls.pull_force_abort ? 1 : 0);
                k_level_pull_max<<<1, 1024, 0, st>>>((uint32_t)gn, ls.sk1, ls.flags + 17);
                // the speculative order below clears the levels' LV_FINAL bits in its rank pass (AD_LEVEL_STRIP=1:
                // the separate pass, an A/B switch)
                if (!(want_order && n > 0 && in.order_verify) || level_strip_pass())
                    k_level_strip<<<gn, 256, 0, st>>>(n, in.lvl);
                }
                // the order of the pulled levels, enqueued before the host waits on the pull's flags: one 8-bit
                // level pass (levels up to 255; k_rank_check flags a deeper batch, then finish_order redoes it)
                bool spec_order = false;
                const std::function<void()> spec = [&]() {
                    if (want_order && n > 0 && in.order_verify) {
                        *in.order_pending = order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st, 255, in.order_verify,
                                                       true, !level_strip_pass());
                        spec_order = true;
                    }
                };
                if (!publish_read(ls.pub, st, ls.flags + 7, 1, &lng, ls.flags + 16, 3, res, &spec)) {
                    err = "exec levels: device error";
                    return AD_ERR_DEVICE;
                }
                if (spec_order && !lng && !res[0] && !res[2]) {
                    ls.pull_path = 1;
                    *iters = (int)res[1] + 1;
                    return AD_OK;
                }
            }
            if ((lng || res[0] || res[2]) && in.complete && in.complete(in.complete_ctx) != AD_OK) {
                err = "exec levels: device error";
                return AD_ERR_DEVICE;
            }
            if (lng) {                                                     // deep key chains: executeAt blocks
                ls.long_hint = true;
                return block_path();
            }
            ls.pull_path = res[2] ? 2 : (res[0] ? 3 : 1);                   // 1 pulled, 2 far predecessors, 3 aborted
            if (!res[0] && !res[2]) {
                const int lv = (int)res[1] + 1;
                *iters = lv;
                if (want_order && n > 0 && in.order_verify)
                    *in.order_pending = order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st, lv - 1, in.order_verify);
                else if (want_order && n > 0)
                    order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st);
                return AD_OK;
            }
            hipMemsetAsync(in.lvl, 0, std::max<size_t>(n, 1) * 4, st);     // aborted / far: the wavefronts below
        }
        // ---- one-pass pull levels for mixed key + range batches (k_level_pull_mixed): executeAt order,
        // persistent waves; kinds whose deps may follow them in executeAt, a long chain or a rank miss (a far
        // slow-path bump) skip it, an abort falls through to the Kahn wavefronts
        if (in.kahn_ok && !in.keep_levels && P > 0 && in.n_special == 0 && (has_b || has_c) && !ls.pull_off && !ls.mixpull_off) {
            ls.chains_ready = false;
            uint32_t fl[32] = {0};
            const int gn1 = ceil_div((long)n, 256);
            {
                KScope ks(K_KAHN, P);
                k_mix_kinds<<<gn1, 256, 0, st>>>(n, in.meta, ls.flags + 20);
                hipMemsetAsync(ls.succ, 0, P * 8, st);
                if (has_c) k_chain_copy<<<gP, 256, 0, st>>>(P, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
                k_chain_build<<<cb_grid, 256, 0, st>>>(P, in.nh, in.prm, in.seg_start, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn,
                                                  ls.c_meta, ls.c_exec1, ls.c_pair, ls.indeg, ls.succ, ls.flags + 7, has_c ? 1 : 0, 1,
                                                  nullptr, in.sec, in.sec_cnt, in.sec_cap, in.sec_tiles);
                hipMemsetAsync(ls.sv1, 0xFF, n * 4, st);
                k_window_rank<<<ceil_div((long)n, WR_N), WR_T, 0, st>>>(n, in.ex1, nullptr, in.lvl, ls.key64, ls.sv1, ls.sk1, ls.flags + 21);
                k_perm_check<<<std::min(gn1, 2048), 256, 0, st>>>(n, ls.key64, ls.sv1, ls.flags + 21);
            }
            if (hipMemcpyAsync(fl, ls.flags, sizeof(fl), hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
                err = "exec levels: device error";
                return AD_ERR_DEVICE;
            }
            if (fl[5]) {
                err = "exec levels: local-only txns are not part of the batch execution order";
                return AD_ERR_UNSUPPORTED;
            }
            ls.mixpull_path = fl[7] ? 2 : (fl[20] ? 3 : (fl[21] ? 4 : 0));
            if (!fl[7] && !fl[20] && !fl[21]) {
                uint32_t res[2] = {0, 0};
                {
                    KScope ks(K_KAHN, P);
                    MixPullArgs ma{};
                    ma.n = n; ma.perm = ls.sv1; ma.key_off = in.key_off; ma.pred = ls.succ; ma.c_txn = ls.c_txn; ma.c_meta = ls.c_meta;
                    ma.e = ea; ma.do_b = has_b ? 1 : 0; ma.do_c = has_c ? 1 : 0; ma.L = in.lvl;
                    ma.abort_flag = ls.flags + 23; ma.maxlvl = ls.flags + 24; ma.force_abort = ls.pull_force_abort ? 1 : 0;
                    if (has_c) {
                        // (c) sources per txn: count, offsets, fill (one sync for the total)
                        if (ls.capX < n + 1 || !ls.xcnt) {
                            const size_t c = n + 1;
                            if (!grow((void**)&ls.xcnt, c * 8) || !grow((void**)&ls.xoff, c * 8) || !grow((void**)&ls.xcur, c * 8)) goto oom;
                            ls.capX = c;
                        }
                        k_unmanaged_prep<<<ceil_div((long)n * WAVE, 256), 256, 0, st>>>(ea);
                        const int gw = ceil_div((long)n * WAVE, 256);
                        k_csrc<false><<<gw, 256, 0, st>>>(ma, ls.xcnt, nullptr);
                        device_scan(SumOp<unsigned long long>{ls.xcnt, ls.xoff, n}, n, (unsigned long long*)ls.agg, st);
                        unsigned long long ctot = 0;
                        if (hipMemcpyAsync(&ctot, ls.xoff + n, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
                            hipStreamSynchronize(st) != hipSuccess) {
                            err = "exec levels: device error";
                            return AD_ERR_DEVICE;
                        }
                        if (ls.xs_cap < ctot || !ls.xs) {
                            const size_t c = std::max<size_t>(ctot + ctot / 8, 1);
                            if (!grow((void**)&ls.xs, c * 4)) goto oom;
                            ls.xs_cap = c;
                        }
                        ma.coff = ls.xoff;
                        ma.cs = ls.xs;
                        k_csrc<true><<<gw, 256, 0, st>>>(ma, nullptr, ls.xs);
                    }
                    // every wave must be resident at once (rank-strided waits): the occupancy bound, with margin
                    int occ = 0, dev = 0, cus = 0;
                    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_level_pull_mixed, 256, 0) != hipSuccess || occ < 1) occ = 1;
                    hipGetDevice(&dev);
                    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 1;
                    const int grid = std::max(1, std::min({gn1, MP_GRID, occ * cus * 3 / 4}));
                    k_level_pull_mixed<<<grid, 256, 0, st>>>(ma);
                    k_level_strip<<<gn1, 256, 0, st>>>(n, in.lvl);
                }
                if (hipMemcpyAsync(res, ls.flags + 23, 8, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
                    err = "exec levels: device error";
                    return AD_ERR_DEVICE;
                }
                if (!res[0]) {
                    ls.mixpull_path = 1;
                    const int lv = (int)res[1] + 1;
                    *iters = lv;
                    if (want_order && n > 0 && in.order_verify)
                        *in.order_pending = order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st, lv - 1, in.order_verify);
                    else if (want_order && n > 0)
                        order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st);
                    return AD_OK;
                }
                ls.mixpull_path = 5;                                               // aborted
                hipMemsetAsync(in.lvl, 0, std::max<size_t>(n, 1) * 4, st);
            }
            hipMemsetAsync(ls.flags + 7, 0, 4, st);
        }
        if (in.kahn_ok && !in.keep_levels && P > 0 && in.n_special == 0) {
            ls.chains_ready = false;
            int lv = 0;
            bool fallback = false;
            const bool xedges = has_b || has_c;
            bool go_blocks = false;             // deep key chains found: leave the Kahn region for the block path
            {
                KScope ks(K_KAHN, P);
                hipMemsetAsync(ls.indeg, 0, n * 4, st);
                hipMemsetAsync(ls.succ, 0, P * 8, st);
                // (c) searches every chain in executeAt order, singletons included
                if (has_c) k_chain_copy<<<gP, 256, 0, st>>>(P, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
                k_chain_build<<<cb_grid, 256, 0, st>>>(P, in.nh, in.prm, in.seg_start, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn, ls.c_meta,
                                                  ls.c_exec1, ls.c_pair, ls.indeg, ls.succ, ls.flags + 7, has_c ? 1 : 0, 0,
                                                  nullptr, in.sec, in.sec_cnt, in.sec_cap, in.sec_tiles);
                // long chains found by the build (flags[7]): rebuild every chain with the parallel kernels
                bool long_done = false;
                auto long_build = [&]() -> bool {
                    hipMemsetAsync(ls.indeg, 0, n * 4, st);
                    hipMemsetAsync(ls.succ, 0, P * 8, st);
                    hipMemsetAsync(ls.c_pair, 0xFF, P * 4, st);
                    hipMemsetAsync(ls.flags + 12, 0, 4, st);
                    k_chain_rank<<<ceil_div((long)P, CR_N), CR_T, 0, st>>>(P, in.seg_start, in.e_txn, in.e_meta, in.e_exec1, in.sval,
                                                                           ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
                    k_chain_check<<<std::min(gP, 2048), 256, 0, st>>>(P, in.seg_start, ls.c_exec1, ls.c_pair, ls.flags + 12);
                    uint32_t bad = 0;
                    if (hipMemcpyAsync(&bad, ls.flags + 12, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
                        hipStreamSynchronize(st) != hipSuccess)
                        return false;
                    if (bad) {       // a far slow-path bump: the serial per-segment insertion order
                        k_chain_copy<<<gP, 256, 0, st>>>(P, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
                        k_chain_order<<<gP, 256, 0, st>>>(P, in.seg_start, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
                    }
                    int32_t* last_w = ls.pm_all;
                    int32_t* next_w = ls.pair_seg;
                    device_scan(WriteLinkOp<false>{P, in.seg_start, ls.c_meta, last_w}, P, (WriteLinkOp<false>::S*)ls.agg, st);
                    device_scan(WriteLinkOp<true>{P, in.seg_start, ls.c_meta, next_w}, P, (WriteLinkOp<true>::S*)ls.agg, st);
                    k_chain_links<<<gP, 256, 0, st>>>(P, in.seg_start, ls.c_txn, ls.c_meta, ls.c_pair, last_w, next_w, ls.indeg, ls.succ);
                    hipMemsetAsync(ls.flags + 7, 0, 4, st);
                    long_done = true;
                    return true;
                };
                if (xedges) {
                    // (b)/(c) successor runs: count, offsets (one sync: total + long-chain / kinds flags), fill
                    if (ls.capX < n + 1 || !ls.xcnt) {
                        const size_t c = n + 1;
                        if (!grow((void**)&ls.xcnt, c * 8) || !grow((void**)&ls.xoff, c * 8) || !grow((void**)&ls.xcur, c * 8)) goto oom;
                        ls.capX = c;
                    }
                    const int gn1 = ceil_div((long)n, 256);
                    // long chains first: (c) searches the executeAt-ordered chains, and the rebuild resets indeg
                    if (hipMemcpyAsync(host, ls.flags, 32, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
                        err = "exec levels: device error";
                        return AD_ERR_DEVICE;
                    }
                    if (host[5]) {
                        err = "exec levels: local-only txns are not part of the batch execution order";
                        return AD_ERR_UNSUPPORTED;
                    }
                    if (host[7] && !long_build()) { err = "exec levels: device error"; return AD_ERR_DEVICE; }
                    if (has_c) k_unmanaged_prep<<<ceil_div((long)n * WAVE, 256), 256, 0, st>>>(ea);
                    XEdgeArgs xa{};
                    xa.e = ea; xa.c_meta = ls.c_meta; xa.do_b = has_b ? 1 : 0; xa.do_c = has_c ? 1 : 0;
                    xa.indeg = ls.indeg; xa.outcnt = ls.xcnt; xa.cur = ls.xcur;
                    hipMemsetAsync(ls.xcnt, 0, n * 8, st);
                    k_xedges<false><<<gn1, 256, 0, st>>>(xa);
                    device_scan(SumOp<unsigned long long>{ls.xcnt, ls.xoff, n}, n, (unsigned long long*)ls.agg, st);
                    unsigned long long etot = 0;
                    if (hipMemcpyAsync(&etot, ls.xoff + n, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
                        hipStreamSynchronize(st) != hipSuccess) {
                        err = "exec levels: device error";
                        return AD_ERR_DEVICE;
                    }
                    if (getenv("AD_DEBUG_LEVELS")) fprintf(stderr, "kahn xedges: %llu edges over %zu txns\n", etot, n);
                    {
                        if (ls.xs_cap < etot || !ls.xs) {
                            const size_t c = std::max<size_t>(etot + etot / 8, 1);
                            if (!grow((void**)&ls.xs, c * 4)) goto oom;
                            ls.xs_cap = c;
                        }
                        hipMemcpyAsync(ls.xcur, ls.xoff, n * 8, hipMemcpyDeviceToDevice, st);
                        xa.xs = ls.xs;
                        k_xedges<true><<<gn1, 256, 0, st>>>(xa);
                    }
                }
                if (!fallback) hipMemcpyAsync(ls.rem, ls.indeg, n * 4, hipMemcpyDeviceToDevice, st);
                // wavefronts per launch batch, no host sync inside a batch (a wavefront after the last
                // one exits at once); the first batch covers typical uniform-key depths (C2: 10), later
                // batches double while every wavefront keeps releasing (mixed batches: thousands of levels)
                constexpr int KB_MAX = 64;
                const int gn = std::min(ceil_div((long)n, 256), KAHN_GRID);
                bool more = !fallback;
                // the first batch: the previous batch's depth (+1) on this handle, else 16 (a gated wavefront
                // still costs a ~5 us launch of the whole grid).  (A frontier-list variant that walked only each
                // level's txns measured no faster on C2 and 5x slower on C4's 5650 levels: kept the sweep.)
                int KB = ls.kb_hint > 0 ? ls.kb_hint : 16;
                while (more && lv < (1 << 24)) {
                    hipMemsetAsync(ls.iflags, 0, KB * 4, st);
                    for (int k = 0; k < KB; ++k)
                        k_kahn_step<<<gn, 256, 0, st>>>(n, (uint32_t)(lv + k), ls.indeg, ls.rem, in.lvl, in.key_off, ls.succ, ls.c_txn,
                                                        k == 0 ? ls.flags + 7 : ls.iflags + (k - 1), k == 0, ls.iflags + k,
                                                        xedges ? (const uint64_t*)ls.xoff : nullptr, xedges ? ls.xs : nullptr);
                    uint32_t fh[KB_MAX];
                    if (!publish_read(ls.pub, st, ls.iflags, KB, fh, ls.flags, lv == 0 ? 8 : 0, host)) {
                        err = "exec levels: device error";
                        return AD_ERR_DEVICE;
                    }
                    if (lv == 0) {
                        if (host[5]) {
                            err = "exec levels: local-only txns are not part of the batch execution order";
                            return AD_ERR_UNSUPPORTED;
                        }
                        if (host[7] && !long_done) {      // the batch's wavefronts were gated off: rebuild, restart
                            if (pure) { go_blocks = true; break; }   // deep key chains: executeAt blocks, not wavefronts
                            if (!long_build()) { err = "exec levels: device error"; return AD_ERR_DEVICE; }
                            hipMemcpyAsync(ls.rem, ls.indeg, n * 4, hipMemcpyDeviceToDevice, st);
                            host[7] = 0;
                            KB = 16;
                            continue;
                        }
                    }
                    int k = 0;
                    while (k < KB && fh[k]) ++k;
                    if (k == KB) {                   // all released more: next batch
                        lv += KB;
                        KB = std::min(KB_MAX, 2 * KB);
                        if (!xedges) {
                            // a deep graph: narrow wavefronts run inside one workgroup until one is wide again
                            if (!ls.kfront && !grow((void**)&ls.kfront, (2 * KS_MAX + 4) * 4)) goto oom;
                            uint32_t* kst = ls.kfront + 2 * KS_MAX;
                            hipMemsetAsync(kst, 0, 16, st);
                            k_frontier_collect<<<ceil_div((long)n, 256), 256, 0, st>>>(n, (uint32_t)lv, ls.indeg, in.lvl, ls.kfront, kst);
                            k_kahn_small<<<1, KS_T, 0, st>>>((uint32_t)lv, kst, ls.kfront, ls.kfront + KS_MAX, ls.rem, in.lvl,
                                                              in.key_off, ls.succ, ls.c_txn);
                            uint32_t ks[3] = {0, 0, 0};
                            if (hipMemcpyAsync(ks, kst, 12, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
                                err = "exec levels: device error";
                                return AD_ERR_DEVICE;
                            }
                            if (ks[0] == 0) { lv = (int)ks[1] + 1; more = false; break; }
                            if ((int)ks[1] != lv) KB = 16;     // resumed at a new wide level
                            lv = (int)ks[1];
                        }
                        continue;
                    }
                    lv += k + 1;
                    more = false;
                    ls.kb_hint = std::min(KB_MAX, std::max(4, lv + 1));
                }
            }
            if (go_blocks) return block_path();
            if (!fallback) {
                *iters = lv;
                // the wavefront count gives the level range: the order needs no host sync of its own
                if (want_order && n > 0 && in.order_verify)
                    *in.order_pending = order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st, lv - 1,
                                                   in.order_verify);
                else if (want_order && n > 0)
                    order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st);
                return AD_OK;
            }
            hipMemsetAsync(in.lvl, 0, std::max<size_t>(n, 1) * 4, st);
        }
        // ---- chain fixpoint
        const bool reuse = in.keep_levels && ls.chains_ready;
        if (P > 0 && reuse) {
            k_stamp_reset<<<ceil_div((long)std::max<uint32_t>(ls.nheads, 1), 256), 256, 0, st>>>(ls.heads, ls.nheads, ls.stamp);
        } else if (P > 0) {
            KScope ks(K_CHAIN_PREP);
            k_chain_copy<<<gP, 256, 0, st>>>(P, in.e_txn, in.e_meta, in.e_exec1, in.sval, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
            k_chain_order<<<gP, 256, 0, st>>>(P, in.seg_start, ls.c_txn, ls.c_meta, ls.c_exec1, ls.c_pair);
            k_seg_table<<<gP, 256, 0, st>>>(P, in.seg_start, ls.seg_len, ls.stamp, ls.flags + 7);
        }
        if (P > 0 && !reuse) {
            KScope ks(K_CHAIN_PREP);
            k_pair_seg<<<gP, 256, 0, st>>>(P, ls.c_pair, ls.c_meta, in.seg_start, ls.seg_len, ls.pair_seg, has_c ? 0 : 1);
            device_scan(SegListOp{in.seg_start, ls.seg_len, ls.heads, ls.long_pos, ls.flags, P}, P, (SegListOp::S*)ls.agg, st);
            if (has_c) k_unmanaged_prep<<<ceil_div((long)n * WAVE, 256), 256, 0, st>>>(ea);
        }
        hipMemcpyAsync(host, ls.flags, 32, hipMemcpyDeviceToHost, st);
        if (hipStreamSynchronize(st) != hipSuccess) { err = "exec levels: device error"; return AD_ERR_DEVICE; }
        if (host[5]) {
            err = "exec levels: local-only txns are not part of the batch execution order";
            return AD_ERR_UNSUPPORTED;
        }
        if (!reuse) { ls.nheads = host[0]; ls.nlong = host[1]; ls.chains_ready = true; }
        const uint32_t nheads = ls.nheads, nlong = ls.nlong;
        bool short_work = nheads > 0, long_dirty = nlong > 0;
        ChainOp op{ls.long_pos, ls.c_txn, ls.c_meta, in.seg_start, in.lvl, ls.pm_all, push, ls.flags + 6};
        // Iterations run in launch batches of up to ITB with no host sync inside a batch: every kernel of
        // iteration k reads iteration k-1's flags on the device and exits at once when nothing changed.
        constexpr int ITB = 8;
        int it = 0;
        bool any_work = short_work || long_dirty || has_b || has_c;
        while (any_work && it < (1 << 24)) {
            hipMemsetAsync(ls.iflags, 0, ITB * 4 * 4, st);
            for (int k = 0; k < ITB; ++k) {
                uint32_t* fl = ls.iflags + 4 * k;
                const uint32_t* prev = k == 0 ? nullptr : ls.iflags + 4 * (k - 1);
                push.iter1 = (uint32_t)(it + k) + 1;
                push.long_dirty = fl + 0;
                ea.push = push;
                ea.changed = fl + 1;
                ea.work_left = fl + 2;
                if (short_work || k > 0) {
                    KScope ks(K_SCAN_CHAIN);
                    k_seg_short<<<ceil_div((long)std::max<uint32_t>(nheads, 1), 256), 256, 0, st>>>(
                        ls.heads, nheads, (uint32_t)(it + k), ls.c_txn, ls.c_meta, in.lvl, ls.pm_all, push, fl + 2);
                }
                if (nlong > 0 && (long_dirty || k > 0)) {
                    ChainOp opk = op;
                    opk.push = push;
                    opk.work_left = fl + 2;
                    opk.enable = k == 0 ? nullptr : prev;   // prev[0] = long chains dirtied last iteration
                    KScope ks(K_SCAN_CHAIN);
                    device_scan(opk, nlong, (ChainOp::S*)ls.agg, st);
                }
                if ((has_b || has_c) && n > 0) {
                    KScope ks(K_LEVEL_EDGES);
                    k_level_edges<<<ceil_div((long)n, 256), 256, 0, st>>>(ea, has_b ? 1 : 0, has_c ? 1 : 0, prev);
                }
            }
            uint32_t fh[ITB * 4];
            if (hipMemcpyAsync(fh, ls.iflags, sizeof(fh), hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                err = "exec levels: device error";
                return AD_ERR_DEVICE;
            }
            any_work = false;
            for (int k = 0; k < ITB; ++k) {
                const uint32_t* f = fh + 4 * k;
                *iters = it + k + 1;
                if (!(f[0] | f[1] | f[2])) { any_work = false; break; }
                any_work = true;
                long_dirty = f[0] != 0;
                short_work = f[2] != 0;
            }
            it += ITB;
        }
    }
    if (want_order && n > 0) order_rows(ls, n, nullptr, in.ex1, in.lvl, in.exec_bits, in.order, st);
    return AD_OK;
oom:
    err = "exec levels: out of device memory";
    return AD_ERR_NOMEM;
}

}  // namespace ad
