// cfk_query_kernels.h — CommandsForKey.mapReduceActive over the device-resident CFK rows (ad_cfk_store_query).
//
// The PreAccept / Accept / GetDeps query of local/cfk/CommandsForKey.java:925-983 as PreAccept.calculatePartialDeps
// (messages/PreAccept.java:245-267) asks it, per (query txn, store key) item, one wave per item:
//   end = insertPos(startedBefore)                                        (rows are byId: TxnId ascending)
//   maxCommittedWriteBefore = the greatest executeAt < startedBefore of a committed Write (:930-943; committedByExecuteAt
//     holds the COMMITTED / STABLE / APPLIED rows, :660-667)
//   emit byId[i < end] whose kind the query witnesses, skipping TRANSITIVELY_KNOWN / INVALID rows and eliding committed
//     Reads / Writes executing before maxCommittedWriteBefore (:945-962)
//   startedBefore <= prunedBefore: also the earliest committed Write executing at or after startedBefore, or the last
//     Applied Write when none precedes it in committedByExecuteAt (:967-980) — the future dependency that takes the place
//     of pruned txns that may execute after the query (ExclusiveSyncPoints: their bound is their TxnId)
//   the query's own TxnId is left out (the map function of calculatePartialDeps, :256-261).
// Each item's emissions are byId ordered (TxnId ascending), split by Deps.Builder's routing (primitives/Deps.java:80-106):
// Read / Write deps to keyDeps, sync points to directKeyDeps.  Then one thread per query unions its items' lists into
// Deps.Builder's canonical CSR (RelationMultiMap.AbstractBuilder.build, utils/RelationMultiMap.java:201-260) in capacity
// regions (one per item / entry), the exact counts beside them; ad_cfk_store_query_fetch compacts.
#pragma once
#include "cfk_store_kernels.h"

namespace ad {

struct CfkQueryArgs {
    CfkStoreArgs s;                          // the resident rows (cnt, tm/tl/tn, em/el/en, st, pbm/pbl/pbn)
    uint32_t nq, items;
    const uint32_t* qoff;                    // [nq + 1] items of query q
    const uint32_t* qkey;                    // [items] store key of each item
    const uint32_t* iq;                      // [items] the item's query
    const uint64_t *qtm, *qtl, *qbm, *qbl;   // [nq] query TxnId, bound
    const int32_t *qtn, *qbn;
    uint32_t* icnt;                          // [items * 2] per item and class: emitted entries (count pass)
    const uint32_t* ioff;                    // [items * 2] their offsets into the per-class lists (fill pass)
    uint64_t *lm[2], *ll[2];                 // per class: the items' lists (TxnIds), byId order
    int32_t* ln[2];
    // per-query output, capacity regions per class: keys at qoff (one slot per item), keysToTxnIds at qoff + entries
    // offset, TxnIds at the entries offset (qeoff: exclusive per-query entry sums per class)
    const uint32_t* qeoff;                   // [2 * (nq + 1)]
    uint64_t* okeys[2];
    int32_t* ok2t[2];
    uint64_t *otm[2], *otl[2];
    int32_t* otn[2];
    uint32_t* okc[2];                        // [nq] keys / entries / TxnIds per query
    uint32_t* oen[2];
    uint32_t* otc[2];
    uint32_t* icur;                          // [items] union cursors
};

__device__ inline void wave_ts3_fold(Ts3& v, bool& has, bool want_max) {
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        Ts3 o{(uint64_t)__shfl_xor((long long)v.msb, d), (uint64_t)__shfl_xor((long long)v.lsb, d), __shfl_xor(v.node, d)};
        const bool oh = __shfl_xor(has ? 1 : 0, d) != 0;
        if (oh && (!has || (want_max ? ts3_cmp(o, v) > 0 : ts3_cmp(o, v) < 0))) { v = o; has = true; }
    }
}

struct CsqItem {
    size_t base;
    uint32_t n, end, qkind;
    int fd;                                  // the future dependency's row, or -1
    Ts3 mcwb, x;
    bool has_mcwb, has_x;
};

__device__ inline CsqItem csq_setup(const CfkQueryArgs& a, uint32_t it) {
    const CfkStoreArgs& s = a.s;
    const uint32_t q = a.iq[it], key = a.qkey[it];
    CsqItem c;
    c.base = cs_tier(key, s.K, s.cap, s.words, s.kslot, s.capB, s.wordsB).rbase;
    c.n = s.cnt[key];
    const Ts3 B{a.qbm[q], a.qbl[q], a.qbn[q]};
    c.x = Ts3{a.qtm[q], a.qtl[q], a.qtn[q]};
    c.has_x = ts3_cmp(c.x, B) != 0;           // executeAt.equals(txnId) ? null : txnId
    c.qkind = cs_kind(c.x.lsb);
    bool found;
    c.end = cs_find(s, c.base, c.n, B, found);  // insertPos (every lane: uniform)
    // maxCommittedWriteBefore and the last Applied Write by executeAt
    Ts3 mc{0, 0, 0}, aw{0, 0, 0};
    bool hmc = false, haw = false;
    for (uint32_t r = __lane_id(); r < c.n; r += WAVE) {
        const size_t x = c.base + r;
        const uint32_t st = s.st[x];
        if (!cs_decided(st) || cs_kind(s.tl[x]) != AD_KIND_WRITE) continue;
        const Ts3 e{s.em[x], s.el[x], s.en[x]};
        if (ts3_cmp(e, B) < 0 && (!hmc || ts3_cmp(e, mc) > 0)) { mc = e; hmc = true; }
        if (st == AD_ST_APPLIED && (!haw || ts3_cmp(e, aw) > 0)) { aw = e; haw = true; }
    }
    wave_ts3_fold(mc, hmc, true);
    wave_ts3_fold(aw, haw, true);
    c.mcwb = mc; c.has_mcwb = hmc;
    c.fd = -1;
    const Ts3 pb{s.pbm[key], s.pbl[key], s.pbn[key]};
    const bool pruned = pb.msb != 0 || pb.lsb != 0 || pb.node != 0;       // TxnId.NONE: nothing pruned
    if (pruned && haw && ts3_cmp(B, pb) <= 0) {
        // the committed Write executing first at or after min(startedBefore, maxAppliedWrite's executeAt)
        const Ts3 lo = ts3_cmp(B, aw) < 0 ? B : aw;
        Ts3 f{0, 0, 0};
        bool hf = false;
        int fr = -1;
        for (uint32_t r = __lane_id(); r < c.n; r += WAVE) {
            const size_t x = c.base + r;
            if (!cs_decided(s.st[x]) || cs_kind(s.tl[x]) != AD_KIND_WRITE) continue;
            const Ts3 e{s.em[x], s.el[x], s.en[x]};
            if (ts3_cmp(e, lo) >= 0 && (!hf || ts3_cmp(e, f) < 0)) { f = e; hf = true; fr = (int)r; }
        }
        // the row with the least executeAt (executeAts are unique): fold (executeAt, row) pairs
#pragma unroll
        for (int d = 1; d < WAVE; d <<= 1) {
            Ts3 o{(uint64_t)__shfl_xor((long long)f.msb, d), (uint64_t)__shfl_xor((long long)f.lsb, d), __shfl_xor(f.node, d)};
            const bool oh = __shfl_xor(hf ? 1 : 0, d) != 0;
            const int orow = __shfl_xor(fr, d);
            if (oh && (!hf || ts3_cmp(o, f) < 0 || (ts3_cmp(o, f) == 0 && orow < fr))) { f = o; hf = true; fr = orow; }
        }
        c.fd = hf ? fr : -1;
    }
    return c;
}

// row r of the item: emitted?  (class: 0 keyDeps, 1 directKeyDeps)
__device__ inline bool csq_emit(const CfkQueryArgs& a, const CsqItem& c, uint32_t r, int* cls) {
    const CfkStoreArgs& s = a.s;
    const size_t x = c.base + r;
    const uint32_t st = s.st[x], k = cs_kind(s.tl[x]);
    *cls = (k == AD_KIND_READ || k == AD_KIND_WRITE) ? 0 : 1;
    bool e = false;
    if (r < c.end && witnesses(c.qkind, k) && st != AD_ST_TRANSITIVELY_KNOWN && st != AD_ST_INVALID) {
        e = true;
        if (cs_decided(st) && c.has_mcwb && (k == AD_KIND_READ || k == AD_KIND_WRITE) &&
            ts3_cmp(Ts3{s.em[x], s.el[x], s.en[x]}, c.mcwb) < 0)
            e = false;                                                          // elided (:951-959)
    }
    if ((int)r == c.fd) e = true;
    if (e && c.has_x && ts3_cmp(Ts3{s.tm[x], s.tl[x], s.tn[x]}, c.x) == 0) e = false;
    return e;
}

template <bool FILL>
static __global__ __launch_bounds__(256) void k_csq_items(CfkQueryArgs a) {
    const uint32_t it = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    if (it >= a.items) return;
    const CsqItem c = csq_setup(a, it);
    const uint32_t lim = max(c.end, c.fd >= 0 ? (uint32_t)c.fd + 1 : 0u);
    uint32_t tot[2] = {0, 0};
    const uint32_t o0 = FILL ? a.ioff[2 * it] : 0, o1 = FILL ? a.ioff[2 * it + 1] : 0;
    for (uint32_t r0 = 0; r0 < lim; r0 += WAVE) {
        const uint32_t r = r0 + __lane_id();
        int cls = 0;
        const bool e = r < lim && csq_emit(a, c, r, &cls);
        const uint64_t m0 = __ballot(e && cls == 0), m1 = __ballot(e && cls == 1);
        if (FILL && e) {
            const uint64_t m = cls == 0 ? m0 : m1;
            const uint32_t pos = (cls == 0 ? o0 + tot[0] : o1 + tot[1]) + (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull));
            const size_t x = c.base + r;
            a.lm[cls][pos] = a.s.tm[x]; a.ll[cls][pos] = a.s.tl[x]; a.ln[cls][pos] = a.s.tn[x];
        }
        tot[0] += (uint32_t)__popcll(m0);
        tot[1] += (uint32_t)__popcll(m1);
    }
    if (!FILL && __lane_id() == 0) { a.icnt[2 * it] = tot[0]; a.icnt[2 * it + 1] = tot[1]; }
}

// One thread per (query, class): the union of its items' sorted lists (RelationMultiMap builder), keys with entries in
// item (key) order, keysToTxnIds = key ends (header) then the per-key indices into the union.
static __global__ __launch_bounds__(256) void k_csq_union(CfkQueryArgs a) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= 2 * a.nq) return;
    const uint32_t q = x >> 1, c = x & 1;
    const uint32_t i0 = a.qoff[q], i1 = a.qoff[q + 1];
    const uint32_t eb = a.qeoff[c * (a.nq + 1) + q];                 // this query's entries (and TxnId capacity) start
    uint64_t* tm = a.otm[c] + eb;
    uint64_t* tl = a.otl[c] + eb;
    int32_t* tn = a.otn[c] + eb;
    for (uint32_t i = i0; i < i1; ++i) a.icur[2 * i + c] = a.ioff[2 * i + c];
    uint32_t u = 0;
    while (true) {                                                 // repeated minimum over the item heads
        bool any = false;
        Ts3 mn{0, 0, 0};
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t p = a.icur[2 * i + c];
            if (p == a.ioff[2 * i + c] + a.icnt[2 * i + c]) continue;
            const Ts3 h{a.lm[c][p], a.ll[c][p], a.ln[c][p]};
            if (!any || ts3_cmp(h, mn) < 0) { mn = h; any = true; }
        }
        if (!any) break;
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t p = a.icur[2 * i + c];
            if (p == a.ioff[2 * i + c] + a.icnt[2 * i + c]) continue;
            if (ts3_cmp(Ts3{a.lm[c][p], a.ll[c][p], a.ln[c][p]}, mn) == 0) a.icur[2 * i + c] = p + 1;
        }
        tm[u] = mn.msb; tl[u] = mn.lsb; tn[u] = mn.node;
        ++u;
    }
    // keys (capacity: one slot per item at i0) and keysToTxnIds (capacity: items + entries at i0 + eb)
    uint64_t* ok = a.okeys[c] + i0;
    int32_t* om = a.ok2t[c] + i0 + eb;
    uint32_t nk = 0;
    for (uint32_t i = i0; i < i1; ++i) nk += a.icnt[2 * i + c] ? 1u : 0u;
    uint32_t run = nk, k = 0;
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t cnt = a.icnt[2 * i + c];
        if (!cnt) continue;
        const uint32_t p0 = a.ioff[2 * i + c];
        uint32_t y = 0;                                            // monotone position in the union
        for (uint32_t j = 0; j < cnt; ++j) {
            const Ts3 v{a.lm[c][p0 + j], a.ll[c][p0 + j], a.ln[c][p0 + j]};
            while (ts3_cmp(Ts3{tm[y], tl[y], tn[y]}, v) < 0) ++y;
            om[run++] = (int32_t)y;
        }
        ok[k] = a.qkey[i];
        om[k] = (int32_t)run;
        ++k;
    }
    a.okc[c][q] = nk; a.oen[c][q] = run - nk; a.otc[c][q] = u;
}

}  // namespace ad
