/*
 * oracle.cpp — CPU restatement of Accord's PreAccept-deps / Deps.merge / execution-order path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker the HIP path is compared against and the
 * "port" CPU baseline that bench.py times; nothing in the product library links, loads or calls
 * it.  It restates the reference algorithms literally (object-free, but loop-for-loop), citing the
 * Java it follows (paths relative to accord-core/src/main/java/accord/):
 *
 *   Timestamp.compareTo ............................ primitives/Timestamp.java:208-217
 *   Txn.Kind.witnesses .............................. primitives/Txn.java:221-245
 *   CommandsForKey.manages / managesExecution ....... local/cfk/CommandsForKey.java:185-199
 *   CommandsForKey.mapReduceActive .................. local/cfk/CommandsForKey.java:925-983
 *   CommandsForKey(...) committedByExecuteAt ........ local/cfk/CommandsForKey.java:642-681
 *   InMemorySafeStore.mapReduceActive ............... impl/InMemoryCommandStore.java:864-871, 272-307
 *   mapReduceRangesInternal ......................... impl/InMemoryCommandStore.java:884-1017
 *   PreAccept.calculatePartialDeps .................. messages/PreAccept.java:245-267
 *   Deps.AbstractBuilder.add ........................ primitives/Deps.java:80-106
 *   RelationMultiMap.AbstractBuilder ................ utils/RelationMultiMap.java:88-271
 *   RelationMultiMap.linearUnion .................... utils/RelationMultiMap.java:562-816
 *   RelationMultiMap.LinearMerger / KeyDeps.merge ... utils/RelationMultiMap.java:284-406, primitives/KeyDeps.java:115-135
 *   Pruning (steady-state CFK trimming, baseline) ... local/cfk/Pruning.java:164-233
 *   Execution order (WaitingOn / notifyManaged) ..... local/Commands.java:617-821,
 *                                                      local/cfk/CommandsForKey.java:1208-1330,
 *                                                      local/cfk/Updating.java:715-800 (Unmanaged)
 *
 * Parity pins: see tests/test_oracle_*.py (restated KeyDepsTest / SortedArraysTest properties,
 * PreAcceptTest known answers, CommandsForKeyTest.Canon execution invariant) — the reference itself
 * is Java and cannot be compiled or run in this image (no JVM), see DESIGN.md §Oracle.
 */
#include "../include/accord_deps.h"
/* The query model the tests hand the oracle in one struct: ad_config's replicas + ad_replica_model's window,
 * drop_p and seed (the engine takes them through ad_open and ad_set_replica_model). */
typedef struct oracle_config {
    uint32_t window, replicas;
    float drop_p;
    uint32_t pad_;
    uint64_t seed;
} oracle_config;

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <iterator>
#include <map>
#include <stdexcept>
#include <string>
#include <memory>
#include <thread>
#include <vector>

namespace {

struct Ts { uint64_t msb, lsb; int32_t node; };

static inline int cmpu(uint64_t a, uint64_t b) { return a < b ? -1 : a > b ? 1 : 0; }

// Timestamp.compareTo — primitives/Timestamp.java:208-217
static inline int ts_cmp(const Ts& a, const Ts& b) {
    int c = cmpu(a.msb, b.msb);                                   // Long.compareUnsigned(msb)
    if (c == 0) c = cmpu(a.lsb >> 16, b.lsb >> 16);               // Long.compare(lowHlc) (non-negative)
    if (c == 0) c = cmpu(a.lsb & 0x1E, b.lsb & 0x1E);             // IDENTITY_FLAGS
    if (c == 0) c = a.node < b.node ? -1 : a.node > b.node ? 1 : 0; // Id.compareTo (signed int)
    return c;
}

static inline int kind_of(const Ts& t) { return (int)((t.lsb >> 1) & 7); }   // TxnId.java:157-160
static inline int domain_of(const Ts& t) { return (int)(t.lsb & 1); }        // TxnId.java:162-165

// Txn.Kind.witnesses — primitives/Txn.java:221-245 (+ Kinds.test :140-152)
static inline bool witnesses(int q, int d) {
    switch (q) {
        case AD_KIND_EPHEMERAL_READ:
        case AD_KIND_READ: return d == AD_KIND_WRITE;                                      // Ws
        case AD_KIND_WRITE:
        case AD_KIND_SYNC_POINT: return d == AD_KIND_READ || d == AD_KIND_WRITE;          // RsOrWs
        case AD_KIND_EXCLUSIVE_SYNC_POINT:                                                 // AnyGloballyVisible
            return d == AD_KIND_READ || d == AD_KIND_WRITE || d == AD_KIND_SYNC_POINT || d == AD_KIND_EXCLUSIVE_SYNC_POINT;
        default: return false;
    }
}
static inline bool globally_visible(int k) {   // Txn.Kind.isGloballyVisible :187-201
    return k == AD_KIND_READ || k == AD_KIND_WRITE || k == AD_KIND_SYNC_POINT || k == AD_KIND_EXCLUSIVE_SYNC_POINT;
}
// CommandsForKey.manages :185-188
static inline bool manages(const Ts& t) { return domain_of(t) == AD_DOMAIN_KEY && globally_visible(kind_of(t)); }
// CommandsForKey.managesExecution :196-199 (Write.witnesses(kind) && key)
static inline bool manages_execution(const Ts& t) {
    return domain_of(t) == AD_DOMAIN_KEY && witnesses(AD_KIND_WRITE, kind_of(t));
}
// Txn.Kind.awaitsOnlyDeps :211-214
static inline bool awaits_only_deps(int k) { return k == AD_KIND_EXCLUSIVE_SYNC_POINT || k == AD_KIND_EPHEMERAL_READ; }

// InternalStatus.isCommitted-and-visible-in-committedByExecuteAt (CommandsForKey.java:659,667)
static inline bool in_committed_by_execute_at(int st) {
    return st >= AD_ST_COMMITTED && st != AD_ST_INVALID;
}

struct RangeK { uint64_t s, e; };   // Range.EndInclusive (start, end]
static inline int range_cmp(const RangeK& a, const RangeK& b) {  // Range.compare — Range.java:310-317
    int c = cmpu(a.s, b.s);
    if (c == 0) c = cmpu(a.e, b.e);
    return c;
}
static inline bool range_contains(const RangeK& r, uint64_t k) { return r.s < k && k <= r.e; }   // EndInclusive.compareTo :48-55
static inline bool ranges_intersect(const RangeK& a, const RangeK& b) {                           // compareIntersecting :296-305
    return !(a.s >= b.e) && !(a.e <= b.s);
}

/* ---------------------------------------------------------------------------------------------- */
/* Canonical relation map (one per txn per class): KeyDeps / RangeDeps raw layout.                 */
/* ---------------------------------------------------------------------------------------------- */
template <class K>
struct Csr {
    std::vector<K> keys;          // sorted unique
    std::vector<uint32_t> vals;   // sorted unique txn ranks
    std::vector<int32_t> k2t;     // keys.size() end offsets, then value indices
    bool empty() const { return k2t.size() == keys.size(); }
};

template <class K> struct KeyOps;
template <> struct KeyOps<uint64_t> {
    static int cmp(uint64_t a, uint64_t b) { return cmpu(a, b); }
};
template <> struct KeyOps<RangeK> {
    static int cmp(const RangeK& a, const RangeK& b) { return range_cmp(a, b); }
};

// RelationMultiMap.AbstractBuilder — utils/RelationMultiMap.java:88-271 (restated on value ranks,
// which order exactly as TxnId.compareTo because the batch is TxnId-sorted).
template <class K>
struct Builder {
    std::vector<K> keys;
    std::vector<int> keyLimits;
    std::vector<uint32_t> kv;     // keysToValues
    int keyOffset = 0;
    bool hasOrderedKeys = true, hasOrderedValues = true;

    int totalCount() const { return (int)kv.size(); }

    void nextKey(const K& key) {                                           // :125-145
        if (!keys.empty() && KeyOps<K>::cmp(keys.back(), key) >= 0) hasOrderedKeys = false;
        finishKey();
        keys.push_back(key);
        keyLimits.push_back(0);
        hasOrderedValues = true;
    }
    void finishKey() {                                                     // :147-173
        if (totalCount() == keyOffset && !keys.empty()) { keys.pop_back(); keyLimits.pop_back(); return; }
        if (keys.empty()) return;
        if (!hasOrderedValues) {
            std::sort(kv.begin() + keyOffset, kv.end());
            kv.erase(std::unique(kv.begin() + keyOffset, kv.end()), kv.end());
        }
        keyLimits.back() = totalCount();
        keyOffset = totalCount();
    }
    void add(const K& key, uint32_t v) {                                   // :175-180
        if (keys.empty() || KeyOps<K>::cmp(keys.back(), key) != 0) nextKey(key);
        add(v);
    }
    void add(uint32_t v) {                                                 // :185-199
        if (hasOrderedValues && totalCount() > keyOffset && kv.back() >= v) hasOrderedValues = false;
        kv.push_back(v);
    }
    Csr<K> build() {                                                       // :201-260
        Csr<K> out;
        if (totalCount() == 0) return out;                                 // none()
        finishKey();
        std::vector<uint32_t> uniq(kv);
        std::sort(uniq.begin(), uniq.end());
        uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
        const int keyCount = (int)keys.size();
        std::vector<int> order(keyCount);
        for (int i = 0; i < keyCount; ++i) order[i] = i;
        if (!hasOrderedKeys) {
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return KeyOps<K>::cmp(keys[a], keys[b]) < 0; });
            for (int i = 1; i < keyCount; ++i)
                if (KeyOps<K>::cmp(keys[order[i - 1]], keys[order[i]]) == 0)
                    throw std::invalid_argument("Key has been visited more than once");   // :234-239
        }
        out.keys.resize(keyCount);
        out.k2t.assign(keyCount + totalCount(), 0);
        int offset = keyCount;
        for (int ki = 0; ki < keyCount; ++ki) {
            int k = order[ki];
            out.keys[ki] = keys[k];
            int from = k == 0 ? 0 : keyLimits[k - 1];
            int to = keyLimits[k];
            // foldlIntersection(values, keysToValues[from..to)) -> index of each value (:252-255)
            size_t li = 0;
            for (int ri = from; ri < to; ++ri) {
                while (uniq[li] < kv[ri]) ++li;
                out.k2t[offset++] = (int32_t)li;
            }
            out.k2t[ki] = offset;
        }
        out.k2t.resize(offset);
        out.vals = std::move(uniq);
        return out;
    }
};

// RelationMultiMap.linearUnion — utils/RelationMultiMap.java:562-816 (general branch; the two
// pass-through branches :583-730 return an input that equals the union, so the result is identical).
template <class K>
static Csr<K> linear_union(const Csr<K>& L, const Csr<K>& R) {
    if (L.empty()) return R;                               // KeyDeps.with :252-253
    if (R.empty()) return L;
    Csr<K> out;
    // SortedArrays.linearUnion on keys and values (SortedArrays.java:198-333)
    {
        size_t i = 0, j = 0;
        while (i < L.keys.size() || j < R.keys.size()) {
            int c = i == L.keys.size() ? 1 : j == R.keys.size() ? -1 : KeyOps<K>::cmp(L.keys[i], R.keys[j]);
            if (c <= 0) { out.keys.push_back(L.keys[i]); ++i; if (c == 0) ++j; }
            else { out.keys.push_back(R.keys[j]); ++j; }
        }
        std::set_union(L.vals.begin(), L.vals.end(), R.vals.begin(), R.vals.end(), std::back_inserter(out.vals));
    }
    // remapToSuperset (SortedArrays.java:1249-1275)
    auto remap = [&](const std::vector<uint32_t>& v) {
        std::vector<int32_t> m(v.size());
        size_t o = 0;
        for (size_t x = 0; x < v.size(); ++x) { while (out.vals[o] < v[x]) ++o; m[x] = (int32_t)o; }
        return m;
    };
    std::vector<int32_t> remapL = remap(L.vals), remapR = remap(R.vals);
    const int nk = (int)out.keys.size();
    out.k2t.assign(nk, 0);
    int lk = 0, rk = 0, ok = 0;
    int l = (int)L.keys.size(), r = (int)R.keys.size();
    const int lkn = (int)L.keys.size(), rkn = (int)R.keys.size();
    while (lk < lkn && rk < rkn) {                                      // :736-783
        int ck = KeyOps<K>::cmp(L.keys[lk], R.keys[rk]);
        if (ck < 0) {
            while (l < L.k2t[lk]) out.k2t.push_back(remapL[L.k2t[l++]]);
            out.k2t[ok++] = (int32_t)out.k2t.size(); lk++;
        } else if (ck > 0) {
            while (r < R.k2t[rk]) out.k2t.push_back(remapR[R.k2t[r++]]);
            out.k2t[ok++] = (int32_t)out.k2t.size(); rk++;
        } else {
            while (l < L.k2t[lk] && r < R.k2t[rk]) {
                int nl = remapL[L.k2t[l]], nr = remapR[R.k2t[r]];
                if (nl <= nr) { out.k2t.push_back(nl); l += 1; r += nl == nr ? 1 : 0; }
                else { out.k2t.push_back(nr); ++r; }
            }
            while (l < L.k2t[lk]) out.k2t.push_back(remapL[L.k2t[l++]]);
            while (r < R.k2t[rk]) out.k2t.push_back(remapR[R.k2t[r++]]);
            out.k2t[ok++] = (int32_t)out.k2t.size(); rk++; lk++;
        }
    }
    while (lk < lkn) { while (l < L.k2t[lk]) out.k2t.push_back(remapL[L.k2t[l++]]); out.k2t[ok++] = (int32_t)out.k2t.size(); lk++; }
    while (rk < rkn) { while (r < R.k2t[rk]) out.k2t.push_back(remapR[R.k2t[r++]]); out.k2t[ok++] = (int32_t)out.k2t.size(); rk++; }
    return out;
}

/* ---------------------------------------------------------------------------------------------- */
/* The batch                                                                                       */
/* ---------------------------------------------------------------------------------------------- */
struct Batch {
    size_t n = 0;
    std::vector<Ts> tx, ex;
    std::vector<uint8_t> st;
    std::vector<uint32_t> key_off, range_off;
    std::vector<uint64_t> keys;
    std::vector<RangeK> ranges;

    explicit Batch(const ad_batch* b) {
        n = b->n;
        tx.resize(n); ex.resize(n); st.assign(b->status, b->status + n);
        for (size_t i = 0; i < n; ++i) {
            tx[i] = Ts{b->txn_msb[i], b->txn_lsb[i], b->txn_node[i]};
            ex[i] = Ts{b->exec_msb[i], b->exec_lsb[i], b->exec_node[i]};
        }
        key_off.assign(b->key_off, b->key_off + n + 1);
        keys.assign(b->keys, b->keys + key_off[n]);
        range_off.assign(n + 1, 0);
        if (b->range_off) {
            range_off.assign(b->range_off, b->range_off + n + 1);
            ranges.resize(range_off[n]);
            for (size_t q = 0; q < ranges.size(); ++q) ranges[q] = RangeK{b->range_start[q], b->range_end[q]};
        }
        for (size_t i = 1; i < n; ++i)
            if (ts_cmp(tx[i - 1], tx[i]) >= 0) throw std::invalid_argument("batch TxnIds must be strictly ascending");
        // Keys / Ranges are sorted sets (primitives/Keys.java, AbstractRanges): the ABI requires them so
        for (size_t i = 0; i < n; ++i) {
            for (uint32_t p = key_off[i] + 1; p < key_off[i + 1]; ++p)
                if (keys[p - 1] >= keys[p]) throw std::invalid_argument("a txn's keys must be strictly ascending");
            for (uint32_t q = range_off[i]; q < range_off[i + 1]; ++q)
                if (ranges[q].s >= ranges[q].e || (q > range_off[i] && ranges[q].s < ranges[q - 1].e))
                    throw std::invalid_argument("a txn's ranges must be sorted, disjoint, start < end");
            if (domain_of(tx[i]) == AD_DOMAIN_RANGE && key_off[i + 1] != key_off[i])
                throw std::invalid_argument("range txns carry no keys");
            if (domain_of(tx[i]) == AD_DOMAIN_KEY && range_off[i + 1] != range_off[i])
                throw std::invalid_argument("key txns carry no ranges");
        }
    }
};

struct TxnDeps { Csr<uint64_t> key, direct; Csr<RangeK> range; };

struct Config {
    uint32_t window = 32, replicas = 1; uint64_t seed = 0; uint32_t drop_thresh = 0;
};

/* CommandsForKey for one key: byId = ranks of managed txns touching the key, ascending. */
struct Cfk {
    uint64_t key;
    std::vector<uint32_t> byId;
};
// baseline pruning state of one CFK (Pruning.java:164-233): a prefix of byId that can never again be emitted
// (committed, executeAt below the running maxCommittedWriteBefore) is dropped.  Kept apart from the CFK so
// threads answering disjoint TxnId ranges share one immutable byId index, each with its own pruning state.
struct CfkPrune {
    size_t prunedBefore = 0;
    bool hasPrunedMaxWrite = false;
    Ts prunedMaxWrite{0, 0, 0};
};
struct CfkIndex {
    std::vector<Cfk> cfks;              // sorted by key
    std::vector<uint32_t> rangeTxns;    // ranks of range-domain txns (rangeCommands registry)
};

struct Oracle {
    const Batch& B;
    Config cfg;
    bool prune;
    bool accept;                        // bound = executeAt (Accept / GetDeps) instead of TxnId (PreAccept)
    bool bound_max = false;             // bound = Timestamp.MAX (GetEphemeralReadDeps.java:76)
    std::shared_ptr<const CfkIndex> index;
    const std::vector<Cfk>& cfks;
    const std::vector<uint32_t>& rangeTxns;
    std::vector<CfkPrune> pst;          // per CFK (this Oracle's queries only)

    static std::shared_ptr<const CfkIndex> build_index(const Batch& B) {
        auto ix = std::make_shared<CfkIndex>();
        std::map<uint64_t, std::vector<uint32_t>> m;
        for (uint32_t i = 0; i < B.n; ++i) {
            if (domain_of(B.tx[i]) == AD_DOMAIN_RANGE) { ix->rangeTxns.push_back(i); continue; }
            if (!manages(B.tx[i])) continue;   // EphemeralRead etc: never registered in CFK
            for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1]; ++p) m[B.keys[p]].push_back(i);
        }
        for (auto& e : m) { Cfk c2; c2.key = e.first; c2.byId = std::move(e.second); ix->cfks.push_back(std::move(c2)); }
        return ix;
    }
    Oracle(const Batch& b, const Config& c, bool prune_, bool accept_ = false, std::shared_ptr<const CfkIndex> shared = nullptr)
        : B(b), cfg(c), prune(prune_ && !accept_), accept(accept_), index(shared ? shared : build_index(b)),
          cfks(index->cfks), rangeTxns(index->rangeTxns), pst(index->cfks.size()) {}
    CfkPrune& prune_of(const Cfk& c) { return pst[&c - cfks.data()]; }

    // rows -> global arrival ranks (a batch that carries earlier batches' kept rows first; nullptr = identity)
    const uint32_t* gid = nullptr;
    uint32_t g(uint32_t x) const { return gid ? gid[x] : x; }
    bool in_window(uint32_t i, uint32_t j) const { return cfg.window > 0 && (uint64_t)g(j) + cfg.window >= g(i); }
    // status of j as seen when i is PreAccepted (SURVEY §8d status model)
    int seen_status(uint32_t i, uint32_t j) const { return in_window(i, j) ? (int)AD_ST_PREACCEPTED : (int)B.st[j]; }
    bool dropped(uint32_t view, uint32_t i, uint32_t j) const {
        return in_window(i, j) && cfg.drop_thresh && ad_drop_hash(cfg.seed, view, g(i), g(j)) < cfg.drop_thresh;
    }
    // The query of txn i: its bound (startedBefore) and the arrival position it is answered at.  PreAccept:
    // TxnId_i at position i.  Accept / GetDeps (Accept.calculatePartialDeps :113-116, GetDeps.apply :76 ->
    // PreAccept.calculatePartialDeps with executeAt): executeAt_i, answered once every txn with a smaller
    // TxnId has arrived — position q = #{j : TxnId_j < executeAt_i}; the status model and window apply from q.
    Ts ts_max{~0ull, ~0ull, INT32_MAX};  // Timestamp.MAX
    const Ts& bound_of(uint32_t i) const { return bound_max ? ts_max : (accept ? B.ex[i] : B.tx[i]); }
    uint32_t query_pos(uint32_t i) const {
        if (bound_max) return (uint32_t)B.n;     // answered after every arrival
        if (!accept) return i;
        const Ts& b = B.ex[i];
        return (uint32_t)(std::lower_bound(B.tx.begin(), B.tx.end(), b, [](const Ts& x, const Ts& y) { return ts_cmp(x, y) < 0; }) - B.tx.begin());
    }
    int seen_status_q(uint32_t q, uint32_t j) const { return in_window(q, j) ? (int)AD_ST_PREACCEPTED : (int)B.st[j]; }
    bool dropped_q(uint32_t view, uint32_t q, uint32_t i, uint32_t j) const {
        return in_window(q, j) && cfg.drop_thresh && ad_drop_hash(cfg.seed, view, g(i), g(j)) < cfg.drop_thresh;
    }

    // CommandsForKey.mapReduceActive(startedBefore = bound, testKind = kind_i.witnesses()) — CommandsForKey.java:925-983;
    // PreAccept.calculatePartialDeps' fn leaves out the txn itself (:258-260: p1 = txnId when executeAt != txnId)
    template <class F>
    void map_reduce_active(const Cfk& cfk, uint32_t i, uint32_t view, F&& emit) {
        CfkPrune& ps = prune_of(cfk);
        const Ts& bound = bound_of(i);
        const uint32_t qp = query_pos(i);
        const int qkind = kind_of(B.tx[i]);
        // int end = insertPos(startedBefore)  (:929, :1373-1378); byId is rank-ordered
        size_t end = std::lower_bound(cfk.byId.begin(), cfk.byId.end(), qp) - cfk.byId.begin();
        // maxCommittedWriteBefore (:930-943): the greatest executeAt of a committed Write in
        // committedByExecuteAt with executeAt < startedBefore.  committedByExecuteAt holds the byId
        // entries (all have TxnId < bound here) whose status >= COMMITTED and != INVALID.
        bool hasM = ps.hasPrunedMaxWrite;
        Ts M = ps.prunedMaxWrite;
        for (size_t x = ps.prunedBefore; x < end; ++x) {
            uint32_t j = cfk.byId[x];
            if (j == i) continue;
            if (!in_committed_by_execute_at(seen_status_q(qp, j))) continue;
            if (kind_of(B.tx[j]) != AD_KIND_WRITE) continue;
            if (ts_cmp(B.ex[j], bound) >= 0) continue;
            if (!hasM || ts_cmp(B.ex[j], M) > 0) { M = B.ex[j]; hasM = true; }
        }
        for (size_t x = ps.prunedBefore; x < end; ++x) {                        // :945-965
            uint32_t j = cfk.byId[x];
            if (j == i) continue;
            const Ts& txn = B.tx[j];
            if (!witnesses(qkind, kind_of(txn))) continue;
            switch (seen_status_q(qp, j)) {
                case AD_ST_COMMITTED: case AD_ST_STABLE: case AD_ST_APPLIED:
                    if (!hasM || ts_cmp(B.ex[j], M) >= 0 || !witnesses(AD_KIND_WRITE, kind_of(txn))) break;
                    continue;                                                    // elided (falls into :959-961)
                case AD_ST_TRANSITIVELY_KNOWN: case AD_ST_INVALID:
                    continue;
                default: break;
            }
            if (dropped_q(view, qp, i, j)) continue;
            emit(cfk.key, j);
        }
        // prunedBefore future-dependency branch (:967-980) never fires: queries arrive in TxnId
        // order, so startedBefore > prunedBefore always.
        if (prune && hasM) {
            // Pruning.maybePrune restated for the steady state: later queries have a larger bound and
            // a larger-or-equal M, so committed entries (seen committed by every later query) with
            // executeAt < M, before any non-prunable entry, are never emitted again.
            size_t x = ps.prunedBefore;
            while (x < end) {
                uint32_t j = cfk.byId[x];
                if (in_window(i + 1, j)) break;                 // still in flight for the next query
                int st = B.st[j];
                bool committed = in_committed_by_execute_at(st);
                bool skip = st == AD_ST_TRANSITIVELY_KNOWN || st == AD_ST_INVALID;
                if (!skip && !(committed && ts_cmp(B.ex[j], M) < 0 && witnesses(AD_KIND_WRITE, kind_of(B.tx[j])))) break;
                if (committed && kind_of(B.tx[j]) == AD_KIND_WRITE && ts_cmp(B.ex[j], bound) < 0) {
                    if (!ps.hasPrunedMaxWrite || ts_cmp(B.ex[j], ps.prunedMaxWrite) > 0) { ps.prunedMaxWrite = B.ex[j]; ps.hasPrunedMaxWrite = true; }
                }
                ++x;
            }
            ps.prunedBefore = x;
        }
    }

    const Cfk* find_cfk(uint64_t key) const {
        auto it = std::lower_bound(cfks.begin(), cfks.end(), key, [](const Cfk& c, uint64_t k) { return c.key < k; });
        return it != cfks.end() && it->key == key ? &*it : nullptr;
    }

    // PreAccept.calculatePartialDeps (PreAccept.java:245-267) via InMemorySafeStore.mapReduceActive
    TxnDeps preaccept(uint32_t i, uint32_t view) {
        Builder<uint64_t> kb, db;
        Builder<RangeK> rb;
        const Ts& me = B.tx[i];
        const int qkind = kind_of(me);
        // Deps.AbstractBuilder.add — Deps.java:80-106
        auto emit_key = [&](uint64_t key, uint32_t j) {
            if (manages_execution(B.tx[j])) kb.add(key, j); else db.add(key, j);
        };
        // mapReduceForKey — InMemoryCommandStore.java:272-307
        if (domain_of(me) == AD_DOMAIN_KEY) {
            std::vector<uint64_t> ks(B.keys.begin() + B.key_off[i], B.keys.begin() + B.key_off[i + 1]);
            std::sort(ks.begin(), ks.end());                     // Keys are sorted
            for (uint64_t k : ks) { const Cfk* c = find_cfk(k); if (c) map_reduce_active(*c, i, view, emit_key); }
        } else {
            for (uint32_t q = B.range_off[i]; q < B.range_off[i + 1]; ++q) {
                const RangeK& r = B.ranges[q];
                // commandsForKey.subMap(start, false, end, true)
                auto it = std::upper_bound(cfks.begin(), cfks.end(), r.s, [](uint64_t k, const Cfk& c) { return k < c.key; });
                for (; it != cfks.end() && it->key <= r.e; ++it) map_reduce_active(*it, i, view, emit_key);
            }
        }
        // mapReduceRangesInternal(STARTED_BEFORE, ANY_DEPS, ANY_STATUS) — InMemoryCommandStore.java:884-1017
        std::vector<std::pair<RangeK, std::vector<uint32_t>>> collect;   // TreeMap<Range, List> by Range::compare
        const uint32_t qp = query_pos(i);
        for (uint32_t j : rangeTxns) {
            if (j >= qp) break;                                      // txnId.compareTo(testTimestamp) >= 0 -> return
            if (j == i) continue;
            if (seen_status_q(qp, j) == AD_ST_INVALID) continue;     // saveStatus >= Erased
            if (!witnesses(qkind, kind_of(B.tx[j]))) continue;
            if (dropped_q(view, qp, i, j)) continue;
            for (uint32_t q = B.range_off[j]; q < B.range_off[j + 1]; ++q) {
                const RangeK& r = B.ranges[q];
                bool hit = false;
                if (domain_of(me) == AD_DOMAIN_KEY) {
                    for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1] && !hit; ++p) hit = range_contains(r, B.keys[p]);
                } else {
                    for (uint32_t p = B.range_off[i]; p < B.range_off[i + 1] && !hit; ++p) hit = ranges_intersect(r, B.ranges[p]);
                }
                if (!hit) continue;
                auto it = std::lower_bound(collect.begin(), collect.end(), r, [](const std::pair<RangeK, std::vector<uint32_t>>& e, const RangeK& x) { return range_cmp(e.first, x) < 0; });
                if (it == collect.end() || range_cmp(it->first, r) != 0) it = collect.insert(it, {r, {}});
                if (it->second.empty() || it->second.back() != j) it->second.push_back(j);
            }
        }
        for (auto& e : collect) for (uint32_t j : e.second) rb.add(e.first, j);
        TxnDeps d;
        d.key = kb.build(); d.direct = db.build(); d.range = rb.build();
        return d;
    }

    // CommandStore.preaccept's maxConflicts.get(keysOrRanges) (local/CommandStore.java:342) as replica view `view`
    // holds it when txn i arrives: MaxConflicts.update (local/MaxConflicts.java:56-59) has folded in the
    // executeAt of every globally visible txn the store holds over its keys or ranges (CommandStore.
    // updateMaxConflicts :282-291; MaxConflicts is a ReducingRangeMap: a key is a point, get() folds every
    // interval intersecting the query) — txns j < i that are not TRANSITIVELY_KNOWN/INVALID, in-flight ones
    // unless the view dropped them: the key txns on i's keys (CFK byId) or on keys inside i's ranges, and the
    // range txns whose ranges contain one of i's keys / intersect one of i's ranges.  Returns the rank of the
    // greatest executeAt (Timestamp::max, ties to the larger rank) or UINT32_MAX for Timestamp.NONE.
    uint32_t max_conflict(uint32_t i, uint32_t view) {
        uint32_t best = UINT32_MAX;
        auto consider = [&](uint32_t j) {
            int st = seen_status(i, j);
            if (st == AD_ST_TRANSITIVELY_KNOWN || st == AD_ST_INVALID) return;
            if (dropped(view, i, j)) return;
            int cmp = best == UINT32_MAX ? 1 : ts_cmp(B.ex[j], B.ex[best]);
            if (cmp > 0 || (cmp == 0 && j > best)) best = j;
        };
        auto cfk_prefix = [&](const Cfk& c) {
            for (uint32_t j : c.byId) {
                if (j >= i) break;
                consider(j);
            }
        };
        const bool key_dom = domain_of(B.tx[i]) == AD_DOMAIN_KEY;
        if (key_dom) {
            for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1]; ++p) {
                const Cfk* c = find_cfk(B.keys[p]);
                if (c) cfk_prefix(*c);
            }
        } else {
            for (uint32_t q = B.range_off[i]; q < B.range_off[i + 1]; ++q) {
                const RangeK& r = B.ranges[q];
                auto it = std::upper_bound(cfks.begin(), cfks.end(), r.s, [](uint64_t k, const Cfk& c) { return k < c.key; });
                for (; it != cfks.end() && it->key <= r.e; ++it) cfk_prefix(*it);
            }
        }
        for (uint32_t j : rangeTxns) {
            if (j >= i) break;
            if (!globally_visible(kind_of(B.tx[j]))) continue;
            bool hit = false;
            for (uint32_t q = B.range_off[j]; q < B.range_off[j + 1] && !hit; ++q) {
                const RangeK& r = B.ranges[q];
                if (key_dom) {
                    for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1] && !hit; ++p) hit = range_contains(r, B.keys[p]);
                } else {
                    for (uint32_t x = B.range_off[i]; x < B.range_off[i + 1] && !hit; ++x) hit = ranges_intersect(r, B.ranges[x]);
                }
            }
            if (hit) consider(j);
        }
        return best;
    }
};

/* Flattened batched CSR (ad_csr_out layout, compacted txn lists). */
struct Flat {
    std::vector<uint32_t> key_off{0}, k2t_off{0}, txn_off{0}, txns;
    std::vector<uint64_t> keys;
    std::vector<int32_t> k2t;
    void push(const Csr<uint64_t>& c) {
        keys.insert(keys.end(), c.keys.begin(), c.keys.end());
        key_off.push_back((uint32_t)(key_off.back() + c.keys.size()));
        k2t.insert(k2t.end(), c.k2t.begin(), c.k2t.end());
        k2t_off.push_back((uint32_t)k2t.size());
        txns.insert(txns.end(), c.vals.begin(), c.vals.end());
        txn_off.push_back((uint32_t)txns.size());
    }
    void push(const Csr<RangeK>& c) {
        for (auto& r : c.keys) { keys.push_back(r.s); keys.push_back(r.e); }
        key_off.push_back((uint32_t)(key_off.back() + c.keys.size()));
        k2t.insert(k2t.end(), c.k2t.begin(), c.k2t.end());
        k2t_off.push_back((uint32_t)k2t.size());
        txns.insert(txns.end(), c.vals.begin(), c.vals.end());
        txn_off.push_back((uint32_t)txns.size());
    }
};

}  // namespace

/* ---------------------------------------------------------------------------------------------- */
/* Execution levels                                                                                 */
/* ---------------------------------------------------------------------------------------------- */
namespace {

// Execution order over the committed batch.  level[T] = 1 + max level over T's predecessors (0 if none):
//  * managed T (key Read/Write): per key, every earlier-executeAt managed txn T witnesses
//    (CommandsForKey.notifyManaged :1208-1289 with unappliedCounters :1291-1330: a Write waits for
//    all earlier Reads+Writes, a Read for earlier Writes; CommandsForKeyTest.Canon.readyToExecute :169-174),
//  * every T: direct-key and range deps with executeAt < T's (Commands.updateWaitingOn :749-755 drops a
//    dependency that executes later) — all of them when T.kind.awaitsOnlyDeps (ExclusiveSyncPoint,
//    EphemeralRead: Commands.initialiseWaitingOn :690-691 waits at maxForEpoch, Txn.java:211-214),
//  * unmanaged T (range domain; key-domain SyncPoint / ExclusiveSyncPoint / EphemeralRead): per key of its
//    keyDeps, every managed txn with executeAt <= the bound = greatest executeAt among its qualifying deps
//    there (Updating.updateUnmanaged :740-792 -> Unmanaged APPLY "wait for it and all earlier txn to
//    Apply", CommandsForKey.java:437-445).  Qualifying: executeAt below T's own; any for EphemeralRead;
//    TxnId below T's for ExclusiveSyncPoint.  Sync points (SyncPoint, ExclusiveSyncPoint) also fold every
//    managed-execution txn of the key's byId between their first and last dependency (:760-777).
// Every edge into a txn that does not await only its deps increases executeAt, so those are resolved in
// executeAt order (phase 1).  Only ExclusiveSyncPoints witness ExclusiveSyncPoints and nothing witnesses an
// EphemeralRead, and their deps precede them in TxnId order: phase 2 resolves them in TxnId order.
// done_aware (a batch carrying CFK history, statuses current): an APPLIED or INVALID txn is done — it waits for
// nothing and nothing waits for it (Commands.updateWaitingOn drops applied / invalidated deps, Commands.java:
// 700-775; CommandsForKey's unapplied counters skip them, :1291-1330): its level is -1 inside the recurrence,
// AD_LEVEL_DONE outside, and the order lists the done txns first (executeAt order), then the rest by (level,
// executeAt).
static std::vector<uint32_t> exec_levels(const Batch& B, const std::vector<TxnDeps>& merged, std::vector<uint32_t>& order,
                                         bool done_aware = false) {
    const uint32_t n = (uint32_t)B.n;
    auto done = [&](uint32_t t) { return done_aware && (B.st[t] == AD_ST_APPLIED || B.st[t] == AD_ST_INVALID); };
    for (uint32_t i = 0; i < n; ++i)
        if (kind_of(B.tx[i]) == AD_KIND_LOCAL_ONLY)
            throw std::invalid_argument("exec levels: local-only txns are not part of the batch execution order");
    std::vector<uint32_t> byExec(n);
    for (uint32_t i = 0; i < n; ++i) byExec[i] = i;
    std::sort(byExec.begin(), byExec.end(), [&](uint32_t a, uint32_t b) { return ts_cmp(B.ex[a], B.ex[b]) < 0; });
    std::vector<int64_t> level(n, -1);
    struct Chain { std::vector<Ts> exec; std::vector<int64_t> pmAll; int64_t maxAll = -1, maxW = -1; };
    // keys as dense ids (sorted distinct keys): chains and byId in flat vectors instead of ordered maps
    std::vector<uint64_t> uk(B.keys.begin(), B.keys.end());
    std::sort(uk.begin(), uk.end());
    uk.erase(std::unique(uk.begin(), uk.end()), uk.end());
    auto kid_of = [&](uint64_t k) -> int64_t {
        auto it = std::lower_bound(uk.begin(), uk.end(), k);
        return it != uk.end() && *it == k ? (int64_t)(it - uk.begin()) : -1;
    };
    std::vector<uint32_t> pkid(B.keys.size());
    for (size_t p = 0; p < B.keys.size(); ++p) pkid[p] = (uint32_t)kid_of(B.keys[p]);
    std::vector<Chain> chains(uk.size());
    // per key: the managed-execution txns in TxnId (= batch) order (CommandsForKey.byId restricted to them)
    std::vector<std::vector<uint32_t>> byId(uk.size());
    for (uint32_t t = 0; t < n; ++t)
        if (manages_execution(B.tx[t]))
            for (uint32_t p = B.key_off[t]; p < B.key_off[t + 1]; ++p) byId[pkid[p]].push_back(t);
    auto resolve = [&](uint32_t t) {
        int64_t lv = -1;
        const Ts& me = B.tx[t];
        const Ts& myExec = B.ex[t];
        const int kind = kind_of(me);
        const bool awaits = awaits_only_deps(kind);
        const bool sync_point = kind == AD_KIND_SYNC_POINT || kind == AD_KIND_EXCLUSIVE_SYNC_POINT;
        const TxnDeps& d = merged[t];
        auto dep_pred = [&](uint32_t dep) {
            if (awaits || ts_cmp(B.ex[dep], myExec) < 0) lv = std::max(lv, level[dep]);
        };
        for (uint32_t v : d.direct.vals) dep_pred(v);
        for (uint32_t v : d.range.vals) dep_pred(v);
        // updateUnmanaged's qualification of a committed managed txn j as one T waits for
        auto qualifies = [&](uint32_t j) {
            return ts_cmp(B.ex[j], myExec) < 0 || kind == AD_KIND_EPHEMERAL_READ ||
                   (kind == AD_KIND_EXCLUSIVE_SYNC_POINT && j < t);
        };
        if (manages_execution(me)) {
            bool w = kind == AD_KIND_WRITE;
            for (uint32_t p = B.key_off[t]; p < B.key_off[t + 1]; ++p) {
                const Chain& c = chains[pkid[p]];             // an empty chain: maxAll = maxW = -1
                lv = std::max(lv, w ? c.maxAll : c.maxW);
            }
        } else {
            // unmanaged: per key of keyDeps, bound = max executeAt of its qualifying deps (+ byId between them)
            const Csr<uint64_t>& kd = d.key;
            for (size_t ki = 0; ki < kd.keys.size(); ++ki) {
                int from = ki == 0 ? (int)kd.keys.size() : kd.k2t[ki - 1];
                bool has = false; Ts bnd{0, 0, 0};
                auto fold = [&](uint32_t j) {
                    if (qualifies(j) && (!has || ts_cmp(B.ex[j], bnd) > 0)) { bnd = B.ex[j]; has = true; }
                };
                uint32_t first = UINT32_MAX, last = 0;
                for (int x = from; x < kd.k2t[ki]; ++x) {
                    uint32_t dep = kd.vals[kd.k2t[x]];
                    fold(dep);
                    first = std::min(first, dep); last = std::max(last, dep);
                }
                const int64_t kk = kid_of(kd.keys[ki]);
                if (sync_point && first != UINT32_MAX && kk >= 0) {
                    const std::vector<uint32_t>& ids = byId[kk];
                    for (auto q = std::lower_bound(ids.begin(), ids.end(), first); q != ids.end() && *q <= last; ++q) fold(*q);
                }
                if (!has || kk < 0) continue;
                Chain& c = chains[kk];
                size_t pos = std::upper_bound(c.exec.begin(), c.exec.end(), bnd, [](const Ts& a, const Ts& b) { return ts_cmp(a, b) < 0; }) - c.exec.begin();
                if (pos > 0) lv = std::max(lv, c.pmAll[pos - 1]);
            }
        }
        level[t] = done(t) ? -1 : lv + 1;
        if (manages_execution(me)) {
            bool w = kind == AD_KIND_WRITE;
            for (uint32_t p = B.key_off[t]; p < B.key_off[t + 1]; ++p) {
                Chain& c = chains[pkid[p]];
                c.maxAll = std::max(c.maxAll, level[t]);
                if (w) c.maxW = std::max(c.maxW, level[t]);
                c.exec.push_back(myExec);
                c.pmAll.push_back(c.maxAll);
            }
        }
    };
    for (uint32_t t : byExec)                       // phase 1
        if (!awaits_only_deps(kind_of(B.tx[t]))) resolve(t);
    for (uint32_t t = 0; t < n; ++t)                // phase 2
        if (awaits_only_deps(kind_of(B.tx[t]))) resolve(t);
    std::vector<uint32_t> out(n);
    for (uint32_t i = 0; i < n; ++i) out[i] = done(i) ? AD_LEVEL_DONE : (uint32_t)level[i];
    order = byExec;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return out[a] + 1u < out[b] + 1u; });
    return out;
}

}  // namespace

/* ---------------------------------------------------------------------------------------------- */
/* C API for tests / bench (ctypes)                                                                 */
/* ---------------------------------------------------------------------------------------------- */
struct oracle_result {
    uint32_t replicas = 0;
    std::vector<Flat> deps;      // [view * 3 + class]
    std::vector<Flat> merged;    // [class]
    std::vector<uint32_t> level, order;
    double t_deps = 0, t_merge = 0, t_levels = 0;
    uint64_t deps_entries = 0, merged_entries = 0;
    std::string error;
};

extern "C" {

/* flags: bit0 = pruning (baseline mode), bit1 = merge, bit2 = levels, bit3 = executeAt-bound deps (Accept /
 * GetDeps; no pruning), bit4 = levels with APPLIED / INVALID txns done (CFK history batches), bit5 = bound
 * Timestamp.MAX (GetEphemeralReadDeps); threads: key-range shards
 * for the deps stage (InMemoryCommandStore.SingleThread per shard + PreAccept.reduce). */
oracle_result* oracle_run_masked(const ad_batch* b, const oracle_config* c, uint32_t flags, uint32_t threads,
                                 const uint8_t* view_mask);
oracle_result* oracle_run(const ad_batch* b, const oracle_config* c, uint32_t flags, uint32_t threads) {
    return oracle_run_masked(b, c, flags, threads, nullptr);
}

/* As oracle_run; view_mask (nullable, [replicas * n]) selects, per txn, the replies the merge folds: the
 * coordinator's fast-path merge takes only the replies whose witnessedAt == TxnId
 * (CoordinateTransaction.onPreAccepted, coordinate/CoordinateTransaction.java:71-101, :75). */
static oracle_result* oracle_run_impl(const ad_batch* b, const oracle_config* c, uint32_t flags, uint32_t threads,
                                      const uint8_t* view_mask, const uint32_t* gid);
oracle_result* oracle_run_masked(const ad_batch* b, const oracle_config* c, uint32_t flags, uint32_t threads,
                                 const uint8_t* view_mask) {
    return oracle_run_impl(b, c, flags, threads, view_mask, nullptr);
}
/* As oracle_run over a batch whose rows carry global arrival ranks gid[n] (the engine's CFK history layout:
 * kept rows of earlier batches, then the new txns); window and drop decisions use gid.  Single-threaded,
 * PreAccept bound. */
oracle_result* oracle_run_gid(const ad_batch* b, const oracle_config* c, uint32_t flags, const uint32_t* gid) {
    return oracle_run_impl(b, c, flags & ~8u, 1, nullptr, gid);
}
static oracle_result* oracle_run_impl(const ad_batch* b, const oracle_config* c, uint32_t flags, uint32_t threads,
                                      const uint8_t* view_mask, const uint32_t* gid) {
    oracle_result* res = new oracle_result();
    try {
        Batch B(b);
        Config cfg;
        cfg.window = c->window; cfg.replicas = c->replicas ? c->replicas : 1; cfg.seed = c->seed;
        cfg.drop_thresh = ad_drop_threshold(c->drop_p);
        res->replicas = cfg.replicas;
        const uint32_t R = cfg.replicas;
        const uint32_t n = (uint32_t)B.n;
        std::vector<std::vector<TxnDeps>> all(R, std::vector<TxnDeps>(n));
        auto t0 = std::chrono::steady_clock::now();
        if (threads <= 1) {
            for (uint32_t v = 0; v < R; ++v) {
                Oracle o(B, cfg, (flags & 1) && !gid, (flags & 40) != 0);
                o.bound_max = (flags & 32) != 0;
                o.gid = gid;
                for (uint32_t i = 0; i < n; ++i) all[v][i] = o.preaccept(i, v);
            }
        } else if (!(flags & 64)) {
            // T threads over contiguous TxnId ranges of the batch, one shared immutable CFK index: every query
            // only reads it (each thread keeps its own pruning state; a range's first query on a key scans the
            // key's whole prefix once, then pruning keeps it short), so the answers equal the serial run's
            auto ix = Oracle::build_index(B);
            std::vector<std::thread> pool;
            for (uint32_t s = 0; s < threads; ++s) {
                pool.emplace_back([&, s]() {
                    const uint32_t i0 = (uint32_t)((uint64_t)n * s / threads), i1 = (uint32_t)((uint64_t)n * (s + 1) / threads);
                    for (uint32_t v = 0; v < R; ++v) {
                        Oracle o(B, cfg, (flags & 1) && !gid, (flags & 40) != 0, ix);
                        o.bound_max = (flags & 32) != 0;
                        o.gid = gid;
                        for (uint32_t i = i0; i < i1; ++i) all[v][i] = o.preaccept(i, v);
                    }
                });
            }
            for (auto& th : pool) th.join();
        } else {
            if (flags & 40) throw std::invalid_argument("key-sharded oracle: executeAt / MAX-bound deps unsupported");
            // Shard the key space into `threads` contiguous ranges of the batch's distinct keys
            // (ShardDistributor.EvenSplit, local/ShardDistributor.java:32-80), one single-threaded
            // store per shard; each store answers the part of every query that falls in its range;
            // PreAccept.reduce (PreAccept.java:141-156) then combines per txn with Deps.with.
            // Range txns / range deps are kept on shard 0 only (single-store semantics).
            std::vector<uint64_t> uk(B.keys);
            std::sort(uk.begin(), uk.end()); uk.erase(std::unique(uk.begin(), uk.end()), uk.end());
            std::vector<uint64_t> bounds;  // shard s owns keys < bounds[s]
            for (uint32_t s = 1; s < threads; ++s) bounds.push_back(uk.empty() ? 0 : uk[std::min(uk.size() - 1, uk.size() * s / threads)]);
            bounds.push_back(UINT64_MAX);
            if (B.range_off[n] > 0) throw std::invalid_argument("threaded oracle: range txns unsupported");
            std::vector<std::vector<std::vector<TxnDeps>>> part(threads, std::vector<std::vector<TxnDeps>>(R, std::vector<TxnDeps>(n)));
            std::vector<std::thread> pool;
            for (uint32_t s = 0; s < threads; ++s) {
                pool.emplace_back([&, s]() {
                    uint64_t lo = s == 0 ? 0 : bounds[s - 1], hi = bounds[s];
                    // a batch view containing only this shard's keys
                    ad_batch sb = *b;
                    std::vector<uint32_t> off(n + 1, 0); std::vector<uint64_t> ks;
                    for (uint32_t i = 0; i < n; ++i) {
                        for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1]; ++p)
                            if (B.keys[p] >= lo && (B.keys[p] < hi || (hi == UINT64_MAX))) ks.push_back(B.keys[p]);
                        off[i + 1] = (uint32_t)ks.size();
                    }
                    sb.key_off = off.data(); sb.keys = ks.data();
                    Batch SB(&sb);
                    for (uint32_t v = 0; v < R; ++v) {
                        Oracle o(SB, cfg, flags & 1);
                        for (uint32_t i = 0; i < n; ++i) part[s][v][i] = o.preaccept(i, v);
                    }
                });
            }
            for (auto& th : pool) th.join();
            for (uint32_t v = 0; v < R; ++v)
                for (uint32_t i = 0; i < n; ++i) {
                    TxnDeps acc = part[0][v][i];
                    for (uint32_t s = 1; s < threads; ++s) {
                        acc.key = linear_union(acc.key, part[s][v][i].key);
                        acc.direct = linear_union(acc.direct, part[s][v][i].direct);
                    }
                    all[v][i] = std::move(acc);
                }
        }
        auto t1 = std::chrono::steady_clock::now();
        res->t_deps = std::chrono::duration<double>(t1 - t0).count();
        res->deps.resize(R * AD_NUM_CLASSES);
        for (uint32_t v = 0; v < R; ++v)
            for (uint32_t i = 0; i < n; ++i) {
                res->deps[v * 3 + 0].push(all[v][i].key);
                res->deps[v * 3 + 1].push(all[v][i].direct);
                res->deps[v * 3 + 2].push(all[v][i].range);
                res->deps_entries += all[v][i].key.k2t.size() - all[v][i].key.keys.size()
                                   + all[v][i].direct.k2t.size() - all[v][i].direct.keys.size()
                                   + all[v][i].range.k2t.size() - all[v][i].range.keys.size();
            }
        std::vector<TxnDeps> merged;
        if (flags & 6) {
            auto t2 = std::chrono::steady_clock::now();
            // Deps.merge(list) = per class LinearMerger over the replies in order (Deps.java:281-286); txns are
            // independent: T threads over contiguous ranges
            merged.resize(n);
            auto merge_range = [&](uint32_t i0, uint32_t i1) {
                for (uint32_t i = i0; i < i1; ++i) {
                    TxnDeps acc;
                    for (uint32_t v = 0; v < R; ++v) {
                        if (view_mask && !view_mask[(size_t)v * n + i]) continue;
                        acc.key = linear_union(acc.key, all[v][i].key);
                        acc.direct = linear_union(acc.direct, all[v][i].direct);
                        acc.range = linear_union(acc.range, all[v][i].range);
                    }
                    merged[i] = std::move(acc);
                }
            };
            if (threads <= 1) {
                merge_range(0, n);
            } else {
                std::vector<std::thread> pool;
                for (uint32_t s = 0; s < threads; ++s)
                    pool.emplace_back(merge_range, (uint32_t)((uint64_t)n * s / threads), (uint32_t)((uint64_t)n * (s + 1) / threads));
                for (auto& th : pool) th.join();
            }
            auto t3 = std::chrono::steady_clock::now();
            res->t_merge = std::chrono::duration<double>(t3 - t2).count();
            res->merged.resize(AD_NUM_CLASSES);
            for (uint32_t i = 0; i < n; ++i) {
                res->merged[0].push(merged[i].key);
                res->merged[1].push(merged[i].direct);
                res->merged[2].push(merged[i].range);
                res->merged_entries += merged[i].key.k2t.size() - merged[i].key.keys.size()
                                     + merged[i].direct.k2t.size() - merged[i].direct.keys.size()
                                     + merged[i].range.k2t.size() - merged[i].range.keys.size();
            }
        }
        if (flags & 4) {
            auto t4 = std::chrono::steady_clock::now();
            res->level = exec_levels(B, merged, res->order, (flags & 16) != 0);
            auto t5 = std::chrono::steady_clock::now();
            res->t_levels = std::chrono::duration<double>(t5 - t4).count();
        }
    } catch (const std::exception& e) {
        res->error = e.what();
    }
    return res;
}

const char* oracle_error(const oracle_result* r) { return r->error.empty() ? nullptr : r->error.c_str(); }

/* The rest of CommandStore.preaccept (local/CommandStore.java:322-347) around the maxConflicts test, restated
 * literally; the state is set by oracle_set_preaccept_expiry (test infrastructure: one global store state):
 *   boolean isExpired = time.now() - txnId.hlc() >= preAcceptTimeout && !txnId.kind().isSyncPoint();        :326
 *   if (rejectBefore != null && !isExpired)
 *       isExpired = null == rejectBefore.foldl(keys, (rejectIfBefore, test) -> rejectIfBefore.compareTo(test) > 0
 *                                                                                ? null : test, txnId, Objects::isNull);
 *   if (isExpired) return time.uniqueNow(txnId).asRejected();           -> fast = AD_FAST_REJECTED (2)     :330-331
 *   if (txnId.kind() == ExclusiveSyncPoint) { markExclusiveSyncPoint(..); return txnId; }   -> fast = 1    :333-337
 * rejectBefore is a ReducingRangeMap<Timestamp>: intervals (s, e]; a key k meets (s < k <= e), a range (qs, qe]
 * meets s < qe && e > qs. */
static struct {
    bool clock = false;
    uint64_t now = 0, timeout = 0;
    std::vector<uint64_t> s, e, msb, lsb;
    std::vector<int32_t> node;
} g_expiry;

int oracle_set_preaccept_expiry(uint64_t now, uint64_t timeout, size_t m, const uint64_t* s, const uint64_t* e,
                                const uint64_t* msb, const uint64_t* lsb, const int32_t* node) {
    g_expiry.clock = timeout != AD_NO_TIMEOUT;
    g_expiry.now = now; g_expiry.timeout = timeout;
    g_expiry.s.assign(s, s + m); g_expiry.e.assign(e, e + m);
    g_expiry.msb.assign(msb, msb + m); g_expiry.lsb.assign(lsb, lsb + m); g_expiry.node.assign(node, node + m);
    return AD_OK;
}

static void preaccept_rules(const Batch& B, uint32_t i, uint32_t replicas, uint8_t* fast) {
    const Ts& t = B.tx[i];
    const uint32_t kind = kind_of(t);
    const uint64_t hlc = ((t.msb & 0x7FFFull) << 48) | (t.lsb >> 16);
    const bool sync_point = kind == AD_KIND_SYNC_POINT || kind == AD_KIND_EXCLUSIVE_SYNC_POINT;
    bool expired = g_expiry.clock && (int64_t)(g_expiry.now - hlc) >= (int64_t)g_expiry.timeout && !sync_point;
    if (!expired && !g_expiry.s.empty()) {
        bool rejected = false;                 // the foldl turned null: some rejectIfBefore > txnId
        auto test = [&](size_t x) {
            if (ts_cmp(Ts{g_expiry.msb[x], g_expiry.lsb[x], g_expiry.node[x]}, t) > 0) rejected = true;
        };
        for (size_t x = 0; x < g_expiry.s.size() && !rejected; ++x) {
            if (domain_of(t) == AD_DOMAIN_KEY) {
                for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1]; ++p)
                    if (g_expiry.s[x] < B.keys[p] && B.keys[p] <= g_expiry.e[x]) { test(x); break; }
            } else {
                for (uint32_t q = B.range_off[i]; q < B.range_off[i + 1]; ++q)
                    if (g_expiry.s[x] < B.ranges[q].e && g_expiry.e[x] > B.ranges[q].s) { test(x); break; }
            }
        }
        expired = rejected;
    }
    if (!expired && kind != AD_KIND_EXCLUSIVE_SYNC_POINT) return;
    for (uint32_t v = 0; v < replicas; ++v) fast[(size_t)v * B.n + i] = expired ? AD_FAST_REJECTED : 1;
}

/* witnessedAt proposal per view (CommandStore.preaccept, local/CommandStore.java:322-347): max_rank[v*n+i] =
 * Oracle::max_conflict (key and range footprints), fast[v*n+i] = TxnId_i >= that executeAt (or none) — the
 * fast-path test :343.  -1 on invalid input. */
int oracle_max_conflicts(const ad_batch* b, const oracle_config* c, uint32_t* max_rank, uint8_t* fast) {
    try {
        Batch B(b);
        Config cfg;
        cfg.window = c->window; cfg.replicas = c->replicas ? c->replicas : 1; cfg.seed = c->seed;
        cfg.drop_thresh = ad_drop_threshold(c->drop_p);
        Oracle o(B, cfg, false);
        const uint32_t n = (uint32_t)B.n;
        for (uint32_t v = 0; v < cfg.replicas; ++v)
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t m = o.max_conflict(i, v);
                max_rank[(size_t)v * n + i] = m;
                fast[(size_t)v * n + i] = (m == UINT32_MAX || ts_cmp(B.tx[i], B.ex[m]) >= 0) ? 1 : 0;
            }
        for (uint32_t i = 0; i < n; ++i) preaccept_rules(B, i, cfg.replicas, fast);
        return AD_OK;
    } catch (const std::exception&) {
        return AD_ERR_ARGUMENT;
    }
}

/* MaxConflicts carried across batches (ad_max_conflicts_carry / _ts / _export): the carry is the store's
 * MaxConflicts map from earlier batches (local/MaxConflicts.java:32-96), held as two tables — points (a key k is
 * the interval (k - 1, k]) and sorted disjoint intervals (s, e] from range txns — that together are the
 * reference's ReducingRangeMap<Timestamp>.  maxConflicts.get(keysOrRanges) of a batch txn is the greatest of the
 * carried values its footprint meets (foldl Timestamp::max, :46-54) and the batch answer above.  Among carried
 * values that compare equal the larger raw lsb is kept (a deterministic tie rule; the reference's Timestamp::max
 * keeps whichever its merge order meets first). */
static bool carry_lookup(size_t m, const uint64_t* ck, const uint64_t* cm, const uint64_t* cl, const int32_t* cn,
                         uint64_t k, Ts* out) {
    const uint64_t* it = std::lower_bound(ck, ck + m, k);
    if (it == ck + m || *it != k) return false;
    const size_t x = (size_t)(it - ck);
    *out = Ts{cm[x], cl[x], cn[x]};
    return true;
}
static inline void carry_fold(const Ts& t, Ts& cb, bool& has) {
    const int c = has ? ts_cmp(t, cb) : 1;
    if (c > 0 || (c == 0 && t.lsb > cb.lsb)) { cb = t; has = true; }
}

int oracle_max_conflicts_ts_ranges(const ad_batch* b, const oracle_config* c, size_t m, const uint64_t* ck, const uint64_t* cm,
                                   const uint64_t* cl, const int32_t* cn, size_t mi, const uint64_t* is, const uint64_t* ie,
                                   const uint64_t* im, const uint64_t* il, const int32_t* in, uint64_t* om, uint64_t* ol,
                                   int32_t* on, uint8_t* fast) {
    try {
        Batch B(b);
        Config cfg;
        cfg.window = c->window; cfg.replicas = c->replicas ? c->replicas : 1; cfg.seed = c->seed;
        cfg.drop_thresh = ad_drop_threshold(c->drop_p);
        Oracle o(B, cfg, false);
        const uint32_t n = (uint32_t)B.n;
        for (uint32_t i = 0; i < n; ++i) {
            bool has = false;
            Ts cb{0, 0, 0};
            auto meet = [&](uint64_t qs, uint64_t qe) {         // every carried point / interval meeting (qs, qe]
                for (size_t x = 0; x < m; ++x) if (qs < ck[x] && ck[x] <= qe) carry_fold(Ts{cm[x], cl[x], cn[x]}, cb, has);
                for (size_t x = 0; x < mi; ++x) if (is[x] < qe && ie[x] > qs) carry_fold(Ts{im[x], il[x], in[x]}, cb, has);
            };
            if (domain_of(B.tx[i]) == AD_DOMAIN_KEY) {
                for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1]; ++p) {
                    const uint64_t k = B.keys[p];
                    Ts t;
                    if (carry_lookup(m, ck, cm, cl, cn, k, &t)) carry_fold(t, cb, has);
                    for (size_t x = 0; x < mi; ++x) if (is[x] < k && k <= ie[x]) carry_fold(Ts{im[x], il[x], in[x]}, cb, has);
                }
            } else {
                for (uint32_t q = B.range_off[i]; q < B.range_off[i + 1]; ++q) meet(B.ranges[q].s, B.ranges[q].e);
            }
            for (uint32_t v = 0; v < cfg.replicas; ++v) {
                const uint32_t r = o.max_conflict(i, v);
                Ts best = cb;
                bool any = has;
                if (r != UINT32_MAX && (!any || ts_cmp(B.ex[r], best) > 0)) { best = B.ex[r]; any = true; }
                const size_t x = (size_t)v * n + i;
                om[x] = any ? best.msb : 0; ol[x] = any ? best.lsb : 0; on[x] = any ? best.node : 0;
                fast[x] = (!any || ts_cmp(B.tx[i], best) >= 0) ? 1 : 0;
            }
            preaccept_rules(B, i, cfg.replicas, fast);
        }
        return AD_OK;
    } catch (const std::exception&) {
        return AD_ERR_ARGUMENT;
    }
}

int oracle_max_conflicts_ts(const ad_batch* b, const oracle_config* c, size_t m, const uint64_t* ck, const uint64_t* cm,
                            const uint64_t* cl, const int32_t* cn, uint64_t* om, uint64_t* ol, int32_t* on, uint8_t* fast) {
    return oracle_max_conflicts_ts_ranges(b, c, m, ck, cm, cl, cn, 0, nullptr, nullptr, nullptr, nullptr, nullptr, om, ol,
                                          on, fast);
}

/* The interval part of the map after the batch: ReducingIntervalMap as boundaries + a value (or none) per gap,
 * updated txn by txn in TxnId order with every range of each range txn the store records (globally visible, not
 * TRANSITIVELY_KNOWN / INVALID): MaxConflicts.update = merge(this, create(ranges, executeAt)) (:56-59), merge =
 * ReducingIntervalMap.merge with Timestamp::max; adjacent gaps of one value coalesce (the builder's normal form).
 * Output: the valued pieces (s, e] in order.  out == NULL: size only. */
struct IntervalMap {
    std::vector<uint64_t> b;            // boundaries, ascending; gap x = (b[x], b[x + 1]]
    std::vector<int> has;               // [b.size() - 1]
    std::vector<Ts> v;
    void merge_range(uint64_t s, uint64_t e, const Ts& t) {
        if (!(s < e)) return;
        std::vector<uint64_t> nb;
        std::merge(b.begin(), b.end(), &s, &s + 1, std::back_inserter(nb));
        std::vector<uint64_t> tmp;
        std::merge(nb.begin(), nb.end(), &e, &e + 1, std::back_inserter(tmp));
        tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
        std::vector<int> nh(tmp.size() ? tmp.size() - 1 : 0, 0);
        std::vector<Ts> nv(nh.size(), Ts{0, 0, 0});
        size_t x = 0;                    // the old gap holding the new gap g
        for (size_t g = 0; g + 1 < tmp.size(); ++g) {
            const uint64_t y = tmp[g + 1];
            while (x + 1 < b.size() && b[x + 1] < y) ++x;
            bool h = false;
            Ts cur{0, 0, 0};
            if (x + 1 < b.size() && b[x] < y && y <= b[x + 1] && has[x]) { h = true; cur = v[x]; }
            if (s < y && y <= e) carry_fold(t, cur, h);
            nh[g] = h ? 1 : 0;
            nv[g] = cur;
        }
        b.swap(tmp); has.swap(nh); v.swap(nv);
    }
};
/* The MaxConflicts table after the batch: carry merged with, per key, the greatest executeAt of the batch txns
 * the store recorded there (globally visible, not TRANSITIVELY_KNOWN / INVALID).  out == NULL: size only. */
int oracle_max_conflicts_export(const ad_batch* b, size_t m, const uint64_t* ck, const uint64_t* cm, const uint64_t* cl,
                                const int32_t* cn, size_t* count, uint64_t* ok, uint64_t* om, uint64_t* ol, int32_t* on) {
    try {
        Batch B(b);
        std::map<uint64_t, Ts> t;
        for (size_t x = 0; x < m; ++x) t[ck[x]] = Ts{cm[x], cl[x], cn[x]};
        for (uint32_t i = 0; i < (uint32_t)B.n; ++i) {
            if (!manages(B.tx[i]) || B.st[i] == AD_ST_TRANSITIVELY_KNOWN || B.st[i] == AD_ST_INVALID) continue;
            for (uint32_t p = B.key_off[i]; p < B.key_off[i + 1]; ++p) {
                auto it = t.find(B.keys[p]);
                if (it == t.end()) t[B.keys[p]] = B.ex[i];
                else if (ts_cmp(B.ex[i], it->second) > 0) it->second = B.ex[i];
            }
        }
        *count = t.size();
        if (!ok) return AD_OK;
        size_t x = 0;
        for (auto& e : t) { ok[x] = e.first; om[x] = e.second.msb; ol[x] = e.second.lsb; on[x] = e.second.node; ++x; }
        return AD_OK;
    } catch (const std::exception&) {
        return AD_ERR_ARGUMENT;
    }
}

int oracle_max_conflicts_export_ranges(const ad_batch* b, size_t mi, const uint64_t* is, const uint64_t* ie, const uint64_t* im,
                                       const uint64_t* il, const int32_t* in, size_t* count, uint64_t* os, uint64_t* oe,
                                       uint64_t* om, uint64_t* ol, int32_t* on) {
    try {
        Batch B(b);
        IntervalMap map;
        for (size_t x = 0; x < mi; ++x) map.merge_range(is[x], ie[x], Ts{im[x], il[x], in[x]});
        for (uint32_t i = 0; i < (uint32_t)B.n; ++i) {
            if (domain_of(B.tx[i]) != AD_DOMAIN_RANGE || !globally_visible(kind_of(B.tx[i]))) continue;
            if (B.st[i] == AD_ST_TRANSITIVELY_KNOWN || B.st[i] == AD_ST_INVALID) continue;
            for (uint32_t q = B.range_off[i]; q < B.range_off[i + 1]; ++q) map.merge_range(B.ranges[q].s, B.ranges[q].e, B.ex[i]);
        }
        std::vector<size_t> st, en;     // valued runs of one raw value
        for (size_t g = 0; g < map.has.size(); ++g) {
            if (!map.has[g]) continue;
            const Ts& t = map.v[g];
            const bool same = g > 0 && map.has[g - 1] && map.v[g - 1].msb == t.msb && map.v[g - 1].lsb == t.lsb &&
                              map.v[g - 1].node == t.node;
            if (same) en.back() = g;
            else { st.push_back(g); en.push_back(g); }
        }
        *count = st.size();
        if (!os) return AD_OK;
        for (size_t k = 0; k < st.size(); ++k) {
            const Ts& t = map.v[st[k]];
            os[k] = map.b[st[k]]; oe[k] = map.b[en[k] + 1]; om[k] = t.msb; ol[k] = t.lsb; on[k] = t.node;
        }
        return AD_OK;
    } catch (const std::exception&) {
        return AD_ERR_ARGUMENT;
    }
}

static const Flat* pick(const oracle_result* r, int stage, uint32_t view, uint32_t cls) {
    if (cls >= AD_NUM_CLASSES) return nullptr;
    if (stage == 0) { if (view >= r->replicas || r->deps.empty()) return nullptr; return &r->deps[view * 3 + cls]; }
    if (r->merged.empty()) return nullptr;
    return &r->merged[cls];
}

int oracle_sizes(const oracle_result* r, int stage, uint32_t view, uint32_t cls, ad_csr_sizes* out) {
    const Flat* f = pick(r, stage, view, cls);
    if (!f) return AD_ERR_ARGUMENT;
    out->n = f->key_off.size() - 1;
    out->keys = f->key_off.back();
    out->k2t = f->k2t.size();
    out->txn_cap = f->txns.size();
    out->txns = f->txns.size();
    return AD_OK;
}

int oracle_fetch(const oracle_result* r, int stage, uint32_t view, uint32_t cls, ad_csr_out* out) {
    const Flat* f = pick(r, stage, view, cls);
    if (!f) return AD_ERR_ARGUMENT;
    // (memcpy of an empty vector's null data() is undefined even for 0 bytes: UBSan, tests/native/oracle_asan.cpp)
    auto cp = [](void* dst, const void* src, size_t bytes) { if (bytes) std::memcpy(dst, src, bytes); };
    cp(out->key_off, f->key_off.data(), f->key_off.size() * 4);
    cp(out->keys, f->keys.data(), f->keys.size() * 8);
    cp(out->k2t_off, f->k2t_off.data(), f->k2t_off.size() * 4);
    cp(out->k2t, f->k2t.data(), f->k2t.size() * 4);
    cp(out->txn_off, f->txn_off.data(), f->txn_off.size() * 4);
    cp(out->txns, f->txns.data(), f->txns.size() * 4);
    return AD_OK;
}

int oracle_levels(const oracle_result* r, uint32_t* level, uint32_t* order) {
    if (r->level.empty()) return AD_ERR_STATE;
    if (level) std::memcpy(level, r->level.data(), r->level.size() * 4);
    if (order) std::memcpy(order, r->order.data(), r->order.size() * 4);
    return AD_OK;
}

void oracle_stats(const oracle_result* r, double* times3, uint64_t* entries2) {
    times3[0] = r->t_deps; times3[1] = r->t_merge; times3[2] = r->t_levels;
    entries2[0] = r->deps_entries; entries2[1] = r->merged_entries;
}

void oracle_free(oracle_result* r) { delete r; }

/* --- primitive entry points for the restated KeyDepsTest / SortedArraysTest properties --------- */

/* RelationMultiMap.AbstractBuilder over (key, value) pairs in the given add order. Returns the
 * canonical CSR in caller buffers sized n_keys+n_pairs (k2t), n_pairs (keys), n_pairs (vals). */
int oracle_build(const uint64_t* keys, const uint32_t* vals, size_t n, uint64_t* out_keys, size_t* n_keys,
                 uint32_t* out_vals, size_t* n_vals, int32_t* out_k2t, size_t* n_k2t) {
    try {
        Builder<uint64_t> bld;
        for (size_t x = 0; x < n; ++x) bld.add(keys[x], vals[x]);
        Csr<uint64_t> c = bld.build();
        std::copy(c.keys.begin(), c.keys.end(), out_keys); *n_keys = c.keys.size();
        std::copy(c.vals.begin(), c.vals.end(), out_vals); *n_vals = c.vals.size();
        std::copy(c.k2t.begin(), c.k2t.end(), out_k2t); *n_k2t = c.k2t.size();
        return AD_OK;
    } catch (const std::invalid_argument&) { return AD_ERR_ARGUMENT; }
}

/* RelationMultiMap.linearUnion of two canonical CSRs. */
int oracle_union(const uint64_t* lk, size_t nlk, const uint32_t* lv, size_t nlv, const int32_t* lm, size_t nlm,
                 const uint64_t* rk, size_t nrk, const uint32_t* rv, size_t nrv, const int32_t* rm, size_t nrm,
                 uint64_t* ok, size_t* nok, uint32_t* ov, size_t* nov, int32_t* om, size_t* nom) {
    Csr<uint64_t> L, R;
    L.keys.assign(lk, lk + nlk); L.vals.assign(lv, lv + nlv); L.k2t.assign(lm, lm + nlm);
    R.keys.assign(rk, rk + nrk); R.vals.assign(rv, rv + nrv); R.k2t.assign(rm, rm + nrm);
    Csr<uint64_t> o = linear_union(L, R);
    std::copy(o.keys.begin(), o.keys.end(), ok); *nok = o.keys.size();
    std::copy(o.vals.begin(), o.vals.end(), ov); *nov = o.vals.size();
    std::copy(o.k2t.begin(), o.k2t.end(), om); *nom = o.k2t.size();
    return AD_OK;
}

/* RelationMultiMap.invert — utils/RelationMultiMap.java:907-938, as KeyDeps.txnIdsToKeys (primitives/KeyDeps.java
 * :362-367) and RangeDeps.txnIdsToRanges (primitives/RangeDeps.java:576-582) call it: src = keysToTxnIds
 * (srcKeyCount end offsets, then value indices), trg = trgKeyCount end offsets (base trgKeyCount), then per value
 * index its key indices ascending.  trg must hold trgKeyCount + srcLength - srcKeyCount ints. */
int oracle_invert(const int32_t* src, size_t src_len, size_t src_keys, size_t trg_keys, int32_t* trg) {
    if (src_len < src_keys) return AD_ERR_ARGUMENT;
    const size_t len = trg_keys + src_len - src_keys;
    std::fill(trg, trg + len, 0);
    if (len == 0) return AD_OK;
    // first pass: count per value
    for (size_t i = src_keys; i < src_len; ++i) {
        if (src[i] < 0 || (size_t)src[i] >= trg_keys) return AD_ERR_ARGUMENT;
        trg[src[i]]++;
    }
    // into offsets (base trgKeyCount), then shifted forward one so trg[v] is v's start
    trg[0] += (int32_t)trg_keys;
    for (size_t i = 1; i < trg_keys; ++i) trg[i] += trg[i - 1];
    for (size_t i = trg_keys; i-- > 1;) trg[i] = trg[i - 1];
    trg[0] = (int32_t)trg_keys;
    // place each key at its value's cursor (the cursor ends as the value's end offset)
    size_t k = 0;
    for (size_t i = src_keys; i < src_len; ++i) {
        while (k < src_keys && i == (size_t)src[k]) ++k;
        trg[trg[src[i]]++] = (int32_t)k;
    }
    return AD_OK;
}

}  // extern "C"

/* ---------------------------------------------------------------------------------------------- */
/* BeginRecovery's store queries                                                */
/*                                                                                                 */
/*   BeginRecovery.apply .............................. messages/BeginRecovery.java:126-145         */
/*   acceptedOrCommittedStartedBeforeWithoutWitnessing  :329-342  (STARTED_BEFORE, WITHOUT, IS_PROPOSED) */
/*   stableStartedBeforeAndWitnessed .................. :344-352  (STARTED_BEFORE, WITH, IS_STABLE)   */
/*   hasAcceptedOrCommittedStartedAfterWithout... ..... :354-367  (STARTED_AFTER, WITHOUT, IS_PROPOSED) */
/*   hasStableExecutesAfterWithoutWitnessing .......... :369-380  (ANY, WITHOUT, IS_STABLE)           */
/*   CommandsForKey.mapReduceFull ..................... local/cfk/CommandsForKey.java:824-923        */
/*   InMemorySafeStore.mapReduceFull / RangesInternal . impl/InMemoryCommandStore.java:875-1017     */
/*   TxnInfo.missing (the CFK invariant) .............. Updating.computeInfoAndAdditions :194-287,   */
/*                                                      Updating.java:340-352 (remove/addToMissingArrays) */
/*                                                                                                 */
/* The store: every txn of the batch with its status and executeAt; each txn's deps = `merged` (the */
/* Deps it was accepted / committed with); nothing pruned (prunedBefore = none).  A managed txn j's   */
/* missing() on key k holds the TxnIds t of byId_k with t < depsKnownBefore(j) (executeAt when       */
/* COMMITTED/STABLE/APPLIED, else TxnId, InternalStatus.depsKnownBefore :561-580), t != j, witnessed */
/* by j's kind, not yet COMMITTED (committed / invalidated txns leave every missing array), and not */
/* in j's Deps.txnIds(k) (Deps.java:188-203: keyDeps, covering rangeDeps, directKeyDeps).            */
/* ---------------------------------------------------------------------------------------------- */
namespace {

struct DepsIn {
    const ad_csr_in* c;      // [3]
    bool key_list_has(int cls, uint32_t j, uint64_t key, uint32_t t) const {   // t in class cls's txnIds(key) of j
        const ad_csr_in& x = c[cls];
        const uint32_t kb = x.key_off[j], ke = x.key_off[j + 1];
        const uint64_t* it = std::lower_bound(x.keys + kb, x.keys + ke, key);
        if (it == x.keys + ke || *it != key) return false;
        return list_has(x, j, (uint32_t)(it - (x.keys + kb)), t);
    }
    static bool list_has(const ad_csr_in& x, uint32_t j, uint32_t ki, uint32_t t) {
        const uint32_t nk = x.key_off[j + 1] - x.key_off[j];
        const int32_t* m = x.k2t + x.k2t_off[j];
        const uint32_t* v = x.txns + x.txn_off[j];
        for (int32_t p = ki == 0 ? (int32_t)nk : m[ki - 1]; p < m[ki]; ++p)
            if (v[m[p]] == t) return true;
        return false;
    }
    // Deps.txnIds(key) contains t (Deps.java:188-203)
    bool txn_ids_has(uint32_t j, uint64_t key, uint32_t t) const {
        if (key_list_has(AD_CLASS_KEY, j, key, t) || key_list_has(AD_CLASS_DIRECT_KEY, j, key, t)) return true;
        const ad_csr_in& r = c[AD_CLASS_RANGE];
        if (!r.key_off) return false;
        for (uint32_t q = r.key_off[j]; q < r.key_off[j + 1]; ++q)
            if (range_contains(RangeK{r.keys[2 * q], r.keys[2 * q + 1]}, key) && list_has(r, j, q - r.key_off[j], t)) return true;
        return false;
    }
    // Deps.intersects(txnId, ranges) (Deps.java:176-186, KeyDeps.java:278-300, RangeDeps.java:507-534)
    bool intersects(uint32_t j, const Ts& tid, uint32_t t, const std::vector<RangeK>& ranges) const {
        const int cls = domain_of(tid) == AD_DOMAIN_RANGE ? AD_CLASS_RANGE : manages_execution(tid) ? AD_CLASS_KEY : AD_CLASS_DIRECT_KEY;
        const ad_csr_in& x = c[cls];
        if (!x.key_off) return false;
        const uint32_t kb = x.key_off[j], ke = x.key_off[j + 1];
        for (uint32_t q = kb; q < ke; ++q) {
            if (!list_has(x, j, q - kb, t)) continue;
            for (const RangeK& r : ranges) {
                if (cls == AD_CLASS_RANGE ? ranges_intersect(RangeK{x.keys[2 * q], x.keys[2 * q + 1]}, r) : range_contains(r, x.keys[q]))
                    return true;
            }
        }
        return false;
    }
};

enum TestStartedAt { STARTED_BEFORE, STARTED_AFTER, ANY };
enum TestDep { WITH, WITHOUT, ANY_DEPS };
enum TestStatus { IS_PROPOSED, IS_STABLE, ANY_STATUS };

struct Recovery {
    const Batch& B;
    const Oracle& O;
    DepsIn deps;

    static bool has_execute_at_or_deps(int st) { return st == AD_ST_ACCEPTED || st == AD_ST_COMMITTED || st == AD_ST_STABLE || st == AD_ST_APPLIED; }

    bool missing_has(uint32_t j, uint64_t key, uint32_t t) const {       // TxnInfo.missing() of j on key contains t
        const int sj = B.st[j];
        if (!has_execute_at_or_deps(sj) || t == j) return false;
        const Ts& dkb = (sj >= AD_ST_COMMITTED) ? B.ex[j] : B.tx[j];
        if (ts_cmp(B.tx[t], dkb) >= 0) return false;
        if (!witnesses(kind_of(B.tx[j]), kind_of(B.tx[t]))) return false;
        if (B.st[t] >= AD_ST_COMMITTED) return false;
        return !deps.txn_ids_has(j, key, t);
    }

    // CommandsForKey.mapReduceFull (CommandsForKey.java:824-923); fn(j) per visited entry
    template <class F>
    void cfk_full(const Cfk& c, uint32_t t, TestStartedAt sa, TestDep td, TestStatus ts, F fn) const {
        const Ts& tid = B.tx[t];
        auto it = std::lower_bound(c.byId.begin(), c.byId.end(), t);
        const bool known = it != c.byId.end() && *it == t;
        const size_t insertPos = (size_t)(it - c.byId.begin());
        // loadingFor: known -> null; unknown -> NO_TXNIDS (nothing is pruned: WITH returns the initial value)
        if (!known && td == WITH) return;
        size_t start = 0, end = c.byId.size();
        if (sa == STARTED_BEFORE) end = insertPos;
        else if (sa == STARTED_AFTER) start = known ? insertPos + 1 : insertPos;   // byId order: known t sits at insertPos
        for (size_t i = start; i < end; ++i) {
            const uint32_t j = c.byId[i];
            if (sa == STARTED_AFTER && j == t) continue;
            if (!witnesses(kind_of(B.tx[j]), kind_of(tid))) continue;      // testKind = kind.witnessedBy()
            const int st = B.st[j];
            if (ts == IS_PROPOSED && !(st == AD_ST_ACCEPTED || st == AD_ST_COMMITTED)) continue;
            if (ts == IS_STABLE && !(st == AD_ST_STABLE || st == AD_ST_APPLIED)) continue;
            if (ts == ANY_STATUS && st == AD_ST_TRANSITIVELY_KNOWN) continue;
            if (td != ANY_DEPS) {
                if (!has_execute_at_or_deps(st)) continue;
                if (ts_cmp(B.ex[j], tid) <= 0) continue;
                const bool hasAsDep = known ? !missing_has(j, c.key, t) : false;
                if (hasAsDep != (td == WITH)) continue;
            }
            fn(c.key, j);
        }
    }

    // the store's CFKs the footprint of t visits (mapReduceForKey: its keys, or every CFK key in its ranges)
    template <class F>
    void for_cfks(uint32_t t, F fn) const {
        if (domain_of(B.tx[t]) == AD_DOMAIN_KEY) {
            for (uint32_t p = B.key_off[t]; p < B.key_off[t + 1]; ++p) {
                auto it = std::lower_bound(O.cfks.begin(), O.cfks.end(), B.keys[p], [](const Cfk& c, uint64_t k) { return c.key < k; });
                if (it != O.cfks.end() && it->key == B.keys[p]) fn(*it);
            }
        } else {
            for (const Cfk& c : O.cfks) {
                bool in = false;
                for (uint32_t q = B.range_off[t]; q < B.range_off[t + 1] && !in; ++q) in = range_contains(B.ranges[q], c.key);
                if (in) fn(c);
            }
        }
    }

    // mapReduceRangesInternal (InMemoryCommandStore.java:884-1017) over the range commands
    template <class F>
    void ranges_full(uint32_t t, TestStartedAt sa, TestDep td, TestStatus ts, F fn) const {
        const Ts& tid = B.tx[t];
        const bool key_dom = domain_of(tid) == AD_DOMAIN_KEY;
        for (uint32_t j : O.rangeTxns) {
            if (sa == STARTED_AFTER && ts_cmp(B.tx[j], tid) <= 0) continue;
            if (sa == STARTED_BEFORE && ts_cmp(B.tx[j], tid) >= 0) continue;
            if (sa != STARTED_AFTER && td != ANY_DEPS && ts_cmp(B.ex[j], tid) < 0) continue;
            const int st = B.st[j];
            if (ts == IS_PROPOSED && !(st == AD_ST_ACCEPTED || st == AD_ST_COMMITTED)) continue;
            if (ts == IS_STABLE && !(st == AD_ST_STABLE || st == AD_ST_APPLIED)) continue;
            if (!witnesses(kind_of(B.tx[j]), kind_of(tid))) continue;
            std::vector<RangeK> jr(B.ranges.begin() + B.range_off[j], B.ranges.begin() + B.range_off[j + 1]);
            if (td != ANY_DEPS) {
                if (!has_execute_at_or_deps(st)) continue;
                if ((td == WITH) == !deps.intersects(j, tid, t, jr)) continue;
            }
            for (const RangeK& r : jr) {        // Routables.foldl(rangeCommand.ranges, sliced): ranges meeting t's footprint
                bool hit = false;
                if (key_dom) for (uint32_t p = B.key_off[t]; p < B.key_off[t + 1] && !hit; ++p) hit = range_contains(r, B.keys[p]);
                else for (uint32_t q = B.range_off[t]; q < B.range_off[t + 1] && !hit; ++q) hit = ranges_intersect(r, B.ranges[q]);
                if (hit) fn(r, j);
            }
        }
    }
};

struct RecoveryDeps {             // Deps.Builder: key, direct, range builders (Deps.java:80-106)
    Builder<uint64_t> key, direct;
    Builder<RangeK> range;
};

}  // namespace

struct oracle_recovery {
    std::vector<uint32_t> off[2][3];
    std::vector<uint64_t> keys[2][3];
    std::vector<uint32_t> txns[2][3];
    std::vector<uint8_t> reject;
    std::string error;
};

extern "C" {

/* rows[nq]: the recovering txns (batch rows).  merged[3]: each txn's Deps (ad_csr_in per class; range may have
 * NULL arrays for key batches).  Outputs per which (0 = earlierCommittedWitness, 1 = earlierAcceptedNoWitness)
 * and class: the built Deps flattened to its (key or range, TxnId) entries in Deps order; reject[q] =
 * rejectsFastPath.  Txns already PreCommitted (status COMMITTED / STABLE / APPLIED / INVALID) answer
 * Deps.NONE and false (:126-130). */
oracle_recovery* oracle_recover(const ad_batch* b, const ad_csr_in* merged, const uint32_t* rows, size_t nq) {
    oracle_recovery* res = new oracle_recovery();
    try {
        Batch B(b);
        Config cfg;
        cfg.window = 0; cfg.replicas = 1;
        Oracle O(B, cfg, false);
        Recovery R{B, O, DepsIn{merged}};
        for (int w = 0; w < 2; ++w)
            for (int c = 0; c < 3; ++c) res->off[w][c].assign(1, 0);
        res->reject.assign(nq, 0);
        for (size_t q = 0; q < nq; ++q) {
            const uint32_t t = rows[q];
            if (t >= B.n) throw std::invalid_argument("recovery row out of range");
            RecoveryDeps out[2];
            if (B.st[t] < AD_ST_COMMITTED) {
                bool reject = false;
                auto any = [&](uint64_t, uint32_t) { reject = true; };
                auto anyr = [&](const RangeK&, uint32_t) { reject = true; };
                R.for_cfks(t, [&](const Cfk& c) { R.cfk_full(c, t, STARTED_AFTER, WITHOUT, IS_PROPOSED, any); });
                R.ranges_full(t, STARTED_AFTER, WITHOUT, IS_PROPOSED, anyr);
                if (!reject) {
                    R.for_cfks(t, [&](const Cfk& c) { R.cfk_full(c, t, ANY, WITHOUT, IS_STABLE, any); });
                    R.ranges_full(t, ANY, WITHOUT, IS_STABLE, anyr);
                }
                res->reject[q] = reject ? 1 : 0;
                auto add_key = [&](RecoveryDeps& d, uint64_t k, uint32_t j) {
                    if (manages_execution(B.tx[j])) d.key.add(k, j); else d.direct.add(k, j);
                };
                // stableStartedBeforeAndWitnessed
                R.for_cfks(t, [&](const Cfk& c) { R.cfk_full(c, t, STARTED_BEFORE, WITH, IS_STABLE,
                                                             [&](uint64_t k, uint32_t j) { add_key(out[0], k, j); }); });
                R.ranges_full(t, STARTED_BEFORE, WITH, IS_STABLE, [&](const RangeK& r, uint32_t j) { out[0].range.add(r, j); });
                // acceptedOrCommittedStartedBeforeWithoutWitnessing (the map adds only executeAt > startedBefore)
                R.for_cfks(t, [&](const Cfk& c) { R.cfk_full(c, t, STARTED_BEFORE, WITHOUT, IS_PROPOSED, [&](uint64_t k, uint32_t j) {
                    if (ts_cmp(B.ex[j], B.tx[t]) > 0) add_key(out[1], k, j); }); });
                R.ranges_full(t, STARTED_BEFORE, WITHOUT, IS_PROPOSED, [&](const RangeK& r, uint32_t j) {
                    if (ts_cmp(B.ex[j], B.tx[t]) > 0) out[1].range.add(r, j); });
            }
            for (int w = 0; w < 2; ++w) {
                auto flat_key = [&](Csr<uint64_t> c, int cls) {
                    for (size_t k = 0; k < c.keys.size(); ++k)
                        for (int32_t p = k == 0 ? (int32_t)c.keys.size() : c.k2t[k - 1]; p < c.k2t[k]; ++p) {
                            res->keys[w][cls].push_back(c.keys[k]);
                            res->txns[w][cls].push_back(c.vals[c.k2t[p]]);
                        }
                    res->off[w][cls].push_back((uint32_t)res->txns[w][cls].size());
                };
                flat_key(out[w].key.build(), AD_CLASS_KEY);
                flat_key(out[w].direct.build(), AD_CLASS_DIRECT_KEY);
                Csr<RangeK> rc = out[w].range.build();
                for (size_t k = 0; k < rc.keys.size(); ++k)
                    for (int32_t p = k == 0 ? (int32_t)rc.keys.size() : rc.k2t[k - 1]; p < rc.k2t[k]; ++p) {
                        res->keys[w][AD_CLASS_RANGE].push_back(rc.keys[k].s);
                        res->keys[w][AD_CLASS_RANGE].push_back(rc.keys[k].e);
                        res->txns[w][AD_CLASS_RANGE].push_back(rc.vals[rc.k2t[p]]);
                    }
                res->off[w][AD_CLASS_RANGE].push_back((uint32_t)res->txns[w][AD_CLASS_RANGE].size());
            }
        }
    } catch (const std::exception& e) {
        res->error = e.what();
    }
    return res;
}

const char* oracle_recovery_error(const oracle_recovery* r) { return r->error.empty() ? nullptr : r->error.c_str(); }

size_t oracle_recovery_entries(const oracle_recovery* r, uint32_t which, uint32_t cls) {
    return which < 2 && cls < 3 ? r->txns[which][cls].size() : 0;
}

int oracle_recovery_fetch(const oracle_recovery* r, uint32_t which, uint32_t cls, uint32_t* off, uint64_t* keys, uint32_t* txns) {
    if (which >= 2 || cls >= 3) return AD_ERR_ARGUMENT;
    auto cp = [](void* dst, const void* src, size_t bytes) { if (bytes) std::memcpy(dst, src, bytes); };
    cp(off, r->off[which][cls].data(), r->off[which][cls].size() * 4);
    cp(keys, r->keys[which][cls].data(), r->keys[which][cls].size() * 8);
    cp(txns, r->txns[which][cls].data(), r->txns[which][cls].size() * 4);
    return AD_OK;
}

int oracle_recovery_flags(const oracle_recovery* r, uint8_t* reject) {
    if (!r->reject.empty()) std::memcpy(reject, r->reject.data(), r->reject.size());
    return AD_OK;
}

void oracle_recovery_free(oracle_recovery* r) { delete r; }

}  // extern "C"
