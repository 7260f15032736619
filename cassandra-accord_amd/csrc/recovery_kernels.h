// recovery_kernels.h — BeginRecovery's CommandStore queries on the device (gfx950).
//
// Replaces, for every recovering txn t of the loaded batch (BeginRecovery.apply, messages/BeginRecovery.java:126-145):
//   earlierCommittedWitness  = stableStartedBeforeAndWitnessed                      :344-352  (STARTED_BEFORE, WITH, IS_STABLE)
//   earlierAcceptedNoWitness = acceptedOrCommittedStartedBeforeWithoutWitnessing     :329-342  (STARTED_BEFORE, WITHOUT, IS_PROPOSED)
//   rejectsFastPath          = hasAcceptedOrCommittedStartedAfterWithoutWitnessing   :354-367  (STARTED_AFTER, WITHOUT, IS_PROPOSED)
//                           || hasStableExecutesAfterWithoutWitnessing               :369-380  (ANY, WITHOUT, IS_STABLE)
// each a SafeCommandStore.mapReduceFull over t's footprint: CommandsForKey.mapReduceFull per key
// (local/cfk/CommandsForKey.java:824-923) and mapReduceRangesInternal over the range commands
// (impl/InMemoryCommandStore.java:884-1017).  The store holds every txn of the batch with its status and
// executeAt, and each txn's Deps are the merged Deps on the handle (what it was accepted / committed with).
//
// WITH / WITHOUT on a CFK entry j: hasAsDep = t not in j.missing().  The CFK invariant (Updating.java:194-287
// builds missing; :340-352 removes a txn from every missing array when it commits or is invalidated) makes
// missing a function of the state: t is missing from j on key k iff j has deps (ACCEPTED..APPLIED),
// t < depsKnownBefore(j) (executeAt once COMMITTED, else TxnId: InternalStatus.depsKnownBefore :561-580),
// t != j, j's kind witnesses t, t is not yet COMMITTED, and t is not in j's Deps.txnIds(k) (keyDeps and
// directKeyDeps of k; rangeDeps only list range-domain TxnIds, Deps.java:80-106, and t is a key txn here).
// A t outside byId (range txn, unmanaged kind) has hasAsDep = false, and WITH visits nothing (loadingFor =
// NO_TXNIDS, nothing pruned).  Range commands: hasAsDep = j.partialDeps().intersects(t, j's ranges)
// (Deps.java:176-186).
//
// Device algorithm: one wave per recovering txn.
//   * CFK part: every footprint element (a key, or a range's CFK keys: a ukey interval) is one contiguous
//     interval of the (key, TxnId)-sorted entries = byId of each key; 64 entries per step, one lane each.
//   * range part: the sorted range entries (start, end, owner) in the merged windows of the footprint
//     (as k_range_deps), each visited once, so every (range, j) is emitted once, in RangeDeps order.
//   * each lane emits at most one entry (the two Deps take disjoint statuses): per output (Deps, class) a
//     ballot, popcounts for the counts, prefix popcounts for the slots.  Entries come out in Deps order:
//     keys ascending (footprint elements ascending, byId within a key), TxnIds ascending within a key.
// Bytes per recovering txn: the visited entries (4 B txn + 1 B meta + 8 B executeAt, + 24 B per range entry);
// a WITH / WITHOUT test binary-searches j's merged Deps (O(log) 4-8 B reads).
#pragma once
#include "range_kernels.h"

namespace ad {

constexpr int RC_OUT = 6;            // [which * 3 + class]; which 0 = earlierCommittedWitness, 1 = earlierAcceptedNoWitness

struct RecoverArgs {
    size_t nq;
    const uint32_t* rows;
    const uint8_t* meta;
    const uint64_t* tx_ts;
    const uint64_t* ex1;
    const uint32_t* key_off;
    const uint64_t* keys;
    const uint32_t* range_off;
    const uint64_t* rs;
    const uint64_t* re;
    // sorted entries (byId of every key)
    const uint64_t* ukey;
    const uint32_t* useg;
    uint32_t U;
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const uint32_t* sval;
    // range entries sorted by (start, end, owner)
    size_t Q;
    const uint64_t* es;
    const uint64_t* ee;
    const uint32_t* eown;
    RangeIndex ix;
    // each txn's Deps (merged), per class
    const uint32_t* m_key_off[3];
    const uint64_t* m_keys[3];
    const uint32_t* m_k2t_off[3];
    const int32_t* m_k2t[3];
    const uint32_t* m_ent_off[3];
    const uint32_t* m_tcnt[3];
    const uint32_t* m_txns[3];
    // outputs
    uint32_t* cnt;                   // count pass: [RC_OUT][nq]
    const uint32_t* off;             // fill pass: [RC_OUT][nq + 1] exclusive offsets
    uint64_t* okeys[RC_OUT];         // key classes: 1 word per entry; range class: start, end
    uint32_t* otxn[RC_OUT];
    uint8_t* reject;                 // [nq]
};

// position of rank t in txn j's class-c TxnId list (sorted ranks), or -1
__device__ inline int32_t rc_txn_index(const RecoverArgs& a, int c, uint32_t j, uint32_t t) {
    if (!a.m_txns[c]) return -1;
    const uint32_t b = a.m_ent_off[c][j], e = b + a.m_tcnt[c][j];
    const uint32_t x = lb_u32(a.m_txns[c], b, e, t);
    return x < e && a.m_txns[c][x] == t ? (int32_t)(x - b) : -1;
}

// is index ti in key ki's list of txn j's class-c CSR (indices ascending)
__device__ inline bool rc_key_lists(const RecoverArgs& a, int c, uint32_t j, uint32_t ki, int32_t ti) {
    const uint32_t nk = a.m_key_off[c][j + 1] - a.m_key_off[c][j];
    const int32_t* m = a.m_k2t[c] + a.m_k2t_off[c][j];
    int32_t lo = ki == 0 ? (int32_t)nk : m[ki - 1], hi = m[ki];
    while (lo < hi) { const int32_t md = (lo + hi) >> 1; if (m[md] < ti) lo = md + 1; else hi = md; }
    return lo < m[ki] && m[lo] == ti;
}

// t in class c's txnIds(key) of txn j (KeyDeps.txnIds(key), KeyDeps.java:540-555)
__device__ inline bool rc_key_has(const RecoverArgs& a, int c, uint32_t j, uint64_t key, uint32_t t) {
    const int32_t ti = rc_txn_index(a, c, j, t);
    if (ti < 0) return false;
    const uint32_t kb = a.m_key_off[c][j], ke = a.m_key_off[c][j + 1];
    const uint32_t k = lb_u64(a.m_keys[c], kb, ke, key);
    return k < ke && a.m_keys[c][k] == key && rc_key_lists(a, c, j, k - kb, ti);
}

// TxnInfo.missing() of CFK entry j (meta mj) on `key` contains the (known, managed) recovering txn t
__device__ inline bool rc_missing(const RecoverArgs& a, uint32_t j, uint32_t mj, uint64_t key, uint32_t t, uint32_t mt) {
    const uint32_t sj = meta_status(mj);
    if (sj < AD_ST_ACCEPTED || sj > AD_ST_APPLIED || j == t) return false;
    const uint64_t tt = a.tx_ts[t];
    const bool before_dkb = sj >= AD_ST_COMMITTED ? tt + 1 < a.ex1[j] : tt < a.tx_ts[j];
    if (!before_dkb || !witnesses(meta_kind(mj), meta_kind(mt)) || meta_status(mt) >= AD_ST_COMMITTED) return false;
    return !rc_key_has(a, AD_CLASS_KEY, j, key, t) && !rc_key_has(a, AD_CLASS_DIRECT_KEY, j, key, t);
}

// Deps.intersects(t, ranges of range txn j) over j's Deps (Deps.java:176-186)
__device__ inline bool rc_intersects(const RecoverArgs& a, uint32_t j, uint32_t t, uint32_t mt) {
    const int c = meta_domain(mt) == AD_DOMAIN_RANGE ? AD_CLASS_RANGE : manages_execution(mt) ? AD_CLASS_KEY : AD_CLASS_DIRECT_KEY;
    const int32_t ti = rc_txn_index(a, c, j, t);
    if (ti < 0) return false;
    const uint32_t kb = a.m_key_off[c][j], ke = a.m_key_off[c][j + 1];
    const uint32_t rb = a.range_off[j], rend = a.range_off[j + 1];
    for (uint32_t k = kb; k < ke; ++k) {
        if (!rc_key_lists(a, c, j, k - kb, ti)) continue;
        for (uint32_t q = rb; q < rend; ++q) {
            const uint64_t s = a.rs[q], e = a.re[q];
            const bool hit = c == AD_CLASS_RANGE ? !(a.m_keys[c][2 * k] >= e) && !(a.m_keys[c][2 * k + 1] <= s)
                                                 : s < a.m_keys[c][k] && a.m_keys[c][k] <= e;
            if (hit) return true;
        }
    }
    return false;
}

template <bool FILL>
struct RcEmit {
    uint32_t n[RC_OUT];
    uint32_t base[RC_OUT];
    __device__ void init(const RecoverArgs& a, size_t q) {
#pragma unroll
        for (int o = 0; o < RC_OUT; ++o) { n[o] = 0; base[o] = FILL ? a.off[(size_t)o * (a.nq + 1) + q] : 0u; }
    }
    // lane emits (k0[, k1], j) into output o (o < 0: nothing)
    __device__ void emit(const RecoverArgs& a, int o, uint64_t k0, uint64_t k1, uint32_t j) {
        const uint64_t below = (1ull << __lane_id()) - 1ull;
#pragma unroll
        for (int x = 0; x < RC_OUT; ++x) {
            const uint64_t mask = __ballot(o == x);
            if (!mask) continue;
            if (FILL && o == x) {
                const uint32_t p = base[x] + n[x] + (uint32_t)__popcll(mask & below);
                a.otxn[x][p] = j;
                if (x % 3 == AD_CLASS_RANGE) { a.okeys[x][2 * (size_t)p] = k0; a.okeys[x][2 * (size_t)p + 1] = k1; }
                else a.okeys[x][p] = k0;
            }
            n[x] += (uint32_t)__popcll(mask);
        }
    }
};

template <bool FILL>
static __global__ __launch_bounds__(256) void k_recover(RecoverArgs a) {
    const size_t q = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (q >= a.nq) return;
    const int lane = __lane_id();
    const uint32_t t = a.rows[q];
    const uint32_t mt = a.meta[t];
    const uint64_t tt = a.tx_ts[t];
    const uint32_t kt = meta_kind(mt);
    const bool key_dom = meta_domain(mt) == AD_DOMAIN_KEY;
    const bool known = manages(mt);                  // t is in byId of each of its keys
    RcEmit<FILL> em;
    em.init(a, q);
    bool reject = false;
    // PreCommitted or later: Deps.NONE, false (BeginRecovery.java:126-130)
    if (meta_status(mt) < AD_ST_COMMITTED) {
        const uint32_t fb = key_dom ? a.key_off[t] : a.range_off[t];
        const uint32_t fe = key_dom ? a.key_off[t + 1] : a.range_off[t + 1];
        // ---- CommandsForKey part ----
        for (uint32_t f = fb; f < fe && a.U > 0; ++f) {
            uint32_t x0, x1;
            if (key_dom) {
                const uint32_t u = lb_u64(a.ukey, 0, a.U, a.keys[f]);
                if (u >= a.U || a.ukey[u] != a.keys[f]) continue;
                x0 = a.useg[u]; x1 = a.useg[u + 1];
            } else {
                x0 = a.useg[ub_u64(a.ukey, 0, a.U, a.rs[f])];               // CFK keys in (start, end]
                x1 = a.useg[ub_u64(a.ukey, 0, a.U, a.re[f])];
            }
            for (uint32_t base = x0; base < x1; base += WAVE) {
                const uint32_t x = base + lane;
                int o = -1;
                uint64_t key = 0;
                uint32_t j = 0;
                if (x < x1) {
                    j = a.e_txn[x];
                    const uint32_t mj = a.e_meta[x];
                    const uint32_t sj = meta_status(mj);
                    const bool proposed = sj == AD_ST_ACCEPTED || sj == AD_ST_COMMITTED;
                    const bool stable = sj == AD_ST_STABLE || sj == AD_ST_APPLIED;
                    // byId entries of a witnessing kind, with deps, executing after t (testDep != ANY_DEPS)
                    if (manages(mj) && j != t && witnesses(meta_kind(mj), kt) && (proposed || stable) && a.e_exec1[x] > tt + 1) {
                        key = a.keys[a.sval[x]];
                        const bool has = known && !rc_missing(a, j, mj, key, t, mt);
                        const int cls = manages_execution(mj) ? AD_CLASS_KEY : AD_CLASS_DIRECT_KEY;
                        if (j < t) {
                            if (stable && has) o = 0 * 3 + cls;                 // earlierCommittedWitness
                            else if (proposed && !has) o = 1 * 3 + cls;         // earlierAcceptedNoWitness
                        }
                        if (!has && ((j > t && proposed) || stable)) reject = true;
                    }
                }
                em.emit(a, o, key, 0, j);
            }
        }
        // ---- range commands ----
        if (a.Q > 0) {
            ri_walk(a.ix, a.es, (uint32_t)a.Q, key_dom, a.keys, a.rs, a.re, fb, fe, [&](uint32_t clo, uint32_t chi) {
                const uint32_t x = clo + lane;
                int o = -1;
                uint64_t s = 0, e = 0;
                uint32_t j = 0;
                if (x < chi) {
                    j = a.eown[x];
                    const uint32_t mj = a.meta[j];
                    const uint32_t sj = meta_status(mj);
                    const bool proposed = sj == AD_ST_ACCEPTED || sj == AD_ST_COMMITTED;
                    const bool stable = sj == AD_ST_STABLE || sj == AD_ST_APPLIED;
                    s = a.es[x]; e = a.ee[x];
                    RangeArgs ra{};
                    ra.keys = a.keys; ra.rs = a.rs; ra.re = a.re;
                    if (j != t && (proposed || stable) && witnesses(meta_kind(mj), kt) &&
                        range_hits(ra, key_dom, fb, fe, s, e)) {
                        const uint64_t ej = a.ex1[j];                   // executeAt + 1
                        const bool exec_ge = ej > tt;                   // executeAt >= t
                        const bool has = rc_intersects(a, j, t, mt);
                        if (j < t && exec_ge) {
                            if (stable && has) o = 0 * 3 + AD_CLASS_RANGE;
                            else if (proposed && !has && ej > tt + 1) o = 1 * 3 + AD_CLASS_RANGE;
                        }
                        if (!has && ((j > t && proposed) || (stable && exec_ge))) reject = true;
                    }
                }
                em.emit(a, o, s, e, j);
            });
        }
    }
    const bool any = __ballot(reject) != 0ull;
    if (lane == 0) {
        if (FILL) a.reject[q] = any ? 1 : 0;
        else {
#pragma unroll
            for (int o = 0; o < RC_OUT; ++o) a.cnt[(size_t)o * a.nq + q] = em.n[o];
        }
    }
}

// exclusive offsets of the six outputs in one scan: off[o * (nq + 1) + q]
struct RecoverOffsetsOp {
    struct S { uint32_t c[RC_OUT]; };
    const uint32_t* cnt;
    uint32_t* off;
    size_t nq;
    __device__ S identity() const { S s; for (int o = 0; o < RC_OUT; ++o) s.c[o] = 0; return s; }
    __device__ S load(size_t i) const { S s; for (int o = 0; o < RC_OUT; ++o) s.c[o] = cnt[(size_t)o * nq + i]; return s; }
    __device__ S combine(const S& x, const S& y) const { S s; for (int o = 0; o < RC_OUT; ++o) s.c[o] = x.c[o] + y.c[o]; return s; }
    __device__ void store(size_t i, const S& ex, const S& inc, const S&) const {
        for (int o = 0; o < RC_OUT; ++o) {
            off[(size_t)o * (nq + 1) + i] = ex.c[o];
            if (i + 1 == nq) off[(size_t)o * (nq + 1) + nq] = inc.c[o];
        }
    }
};

}  // namespace ad
