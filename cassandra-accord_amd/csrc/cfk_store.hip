// cfk_store.hip — ad_cfk_store_*: device-resident CommandsForKey states driven by CommandsForKey.update events
// (cfk_store_kernels.h), with CommandsForKey.notifyManaged's release rule over the resident rows (notify_kernels.h).
#include "engine_internal.h"
#include "cfk_query_kernels.h"

// Timestamp.compareTo on the host (Timestamp.java:208-217; the device's ts3_cmp)
static int host_ts_cmp(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn) {
    if (am != bm) return am < bm ? -1 : 1;
    if ((al >> 16) != (bl >> 16)) return (al >> 16) < (bl >> 16) ? -1 : 1;
    if ((al & 0x1E) != (bl & 0x1E)) return (al & 0x1E) < (bl & 0x1E) ? -1 : 1;
    return an < bn ? -1 : (an > bn ? 1 : 0);
}

int ad_cfk_store_open(ad_handle* h, uint32_t keys, uint32_t capacity) {
    return ad_cfk_store_open_tiered(h, keys, capacity, 0, 0);
}

int ad_cfk_store_open_tiered(ad_handle* h, uint32_t keys, uint32_t capacity, uint32_t big_capacity, uint32_t big_keys) {
    if (!h) return AD_ERR_ARGUMENT;
    if (keys == 0 || capacity == 0 || capacity > 8192)
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_open: keys >= 1 and 1 <= capacity <= 8192");
    if (big_keys && (big_capacity <= capacity || big_capacity > 64 * NF_MAX_WORDS || big_keys > keys))
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_open_tiered: capacity < big_capacity <= 16384 and big_keys <= keys");
    hipSetDevice(h->device);
    auto& c = h->cs;
    c.K = keys;
    c.ucap = capacity;
    c.cap = (capacity + 63) & ~63u;
    c.words = c.cap / 64;
    c.nbig = big_keys;
    c.ucapB = big_keys ? big_capacity : 0;
    c.capB = big_keys ? (big_capacity + 63) & ~63u : 0;
    c.wordsB = c.capB / 64;
    c.kslot_host.assign(big_keys ? keys : 0, ~0u);
    c.big_keys.clear();
    // regular tier: keys x cap rows; large tier after it: nbig x capB rows (bitmaps: a row of the tier's words per slot)
    const size_t rows = (size_t)c.K * c.cap + (size_t)c.nbig * c.capB;
    const size_t bw = (size_t)c.K * c.cap * c.words + (size_t)c.nbig * c.capB * c.wordsB;
    CK(dalloc(h, S_CS0 + 0, &c.cnt, c.K)); CK(dalloc(h, S_CS0 + 1, &c.tm, rows)); CK(dalloc(h, S_CS0 + 2, &c.tl, rows));
    CK(dalloc(h, S_CS0 + 3, &c.tn, rows)); CK(dalloc(h, S_CS0 + 4, &c.em, rows)); CK(dalloc(h, S_CS0 + 5, &c.el, rows));
    CK(dalloc(h, S_CS0 + 6, &c.en, rows)); CK(dalloc(h, S_CS0 + 7, &c.st, rows)); CK(dalloc(h, S_CS0 + 8, &c.slot, rows));
    CK(dalloc(h, S_CS0 + 9, &c.bits, bw)); CK(dalloc(h, S_CS0 + 10, &c.out, rows));
    CK(dalloc(h, S_CS0 + 11, &c.pre, 2 * rows)); CK(dalloc(h, S_CS0 + 12, &c.flags, 4));
    CK(dalloc(h, S_CS0 + 13, &c.pbm, c.K)); CK(dalloc(h, S_CS0 + 14, &c.pbl, c.K)); CK(dalloc(h, S_CS0 + 15, &c.pbn, c.K));
    CK(dalloc(h, S_CS0 + 16, &c.lp_cnt, c.K)); CK(dalloc(h, S_CS0 + 17, &c.lpm, rows));
    CK(dalloc(h, S_CS0 + 18, &c.lpl, rows)); CK(dalloc(h, S_CS0 + 19, &c.lpn, rows));
    CK(dalloc(h, S_CS0 + 20, &c.lp_bits, bw));
    CK(dalloc(h, S_CSU0 + 0, &c.lp_xm, rows)); CK(dalloc(h, S_CSU0 + 1, &c.lp_xl, rows)); CK(dalloc(h, S_CSU0 + 2, &c.lp_xn, rows));
    CK(dalloc(h, S_CSU0 + 3, &c.lp_xh, rows)); CK(dalloc(h, S_CSU0 + 4, &c.um_cnt, c.K)); CK(dalloc(h, S_CSU0 + 5, &c.um_p, rows));
    CK(dalloc(h, S_CSU0 + 6, &c.um_wm, rows)); CK(dalloc(h, S_CSU0 + 7, &c.um_wl, rows)); CK(dalloc(h, S_CSU0 + 8, &c.um_wn, rows));
    CK(dalloc(h, S_CSU0 + 9, &c.um_tm, rows)); CK(dalloc(h, S_CSU0 + 10, &c.um_tl, rows)); CK(dalloc(h, S_CSU0 + 11, &c.um_tn, rows));
    CK(dalloc(h, S_CSU0 + 12, &c.nt_cnt, c.K));
    c.kslot = c.kres = nullptr;
    if (c.nbig) {
        CK(dalloc(h, S_CSKSLOT, &c.kslot, c.K)); CK(dalloc(h, S_CSKRES, &c.kres, c.K));
        HIPCHK(h, hipMemsetAsync(c.kslot, 0xFF, (size_t)c.K * 4, h->st));
        HIPCHK(h, hipMemsetAsync(c.kres, 0xFF, (size_t)c.K * 4, h->st));
    }
    HIPCHK(h, hipMemsetAsync(c.um_cnt, 0, (size_t)c.K * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.nt_cnt, 0, (size_t)c.K * 4, h->st));
    c.nt_total = 0;
    HIPCHK(h, hipMemsetAsync(c.pbm, 0, (size_t)c.K * 8, h->st));
    HIPCHK(h, hipMemsetAsync(c.pbl, 0, (size_t)c.K * 8, h->st));
    HIPCHK(h, hipMemsetAsync(c.pbn, 0, (size_t)c.K * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.lp_cnt, 0, (size_t)c.K * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.cnt, 0, (size_t)c.K * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.flags, 0, 16, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

// the store's tier fields of a kernel's args
static void cs_tier_args(const ad_handle::CfkStore& c, CfkStoreArgs& a) {
    a.K = c.K; a.cap = c.cap; a.words = c.words;
    a.kslot = c.kslot; a.capB = c.capB; a.wordsB = c.wordsB; a.nbig = c.nbig;
}

int ad_cfk_store_apply(ad_handle* h, const ad_cfk_events* ev) {
    if (!h || !ev) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_apply before ad_cfk_store_open");
    const size_t m = ev->m;
    if (!ev->ev_off || !ev->deps_off) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: ev_off / deps_off missing");
    if (ev->ev_off[0] != 0 || ev->ev_off[c.K] != m || ev->deps_off[0] != 0)
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: ev_off must span [0, m] and deps_off start at 0");
    for (uint32_t k = 0; k < c.K; ++k)
        if (ev->ev_off[k + 1] < ev->ev_off[k]) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: ev_off not monotone");
    for (size_t e = 0; e < m; ++e)
        if (ev->deps_off[e + 1] < ev->deps_off[e]) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: deps_off not monotone");
    if (m == 0) {
        hipSetDevice(h->device);
        HIPCHK(h, hipMemsetAsync(c.nt_cnt, 0, (size_t)c.K * 4, h->st));   // this call notified nothing
        c.ev_off_host.assign(ev->ev_off, ev->ev_off + c.K + 1);
        c.nt_base_host.assign(c.K + 1, 0);
        HIPCHK(h, hipStreamSynchronize(h->st));
        return AD_OK;
    }
    if (!ev->txn_msb || !ev->txn_lsb || !ev->txn_node || !ev->status || !ev->exec_msb || !ev->exec_lsb || !ev->exec_node)
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: an event array is missing");
    for (size_t e = 0; e < m; ++e)
        if (ev->status[e] > AD_ST_INVALID) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: status out of range");
    if (ev->op)
        for (size_t e = 0; e < m; ++e) {
            if (ev->op[e] > AD_CFK_OP_UNMANAGED_RECHECK) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: op out of range");
            if (ev->op[e] == AD_CFK_OP_PRUNE && ev->exec_node[e] < 0)
                return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: a PRUNE event's interval (exec_node) is negative");
            if (ev->op[e] == AD_CFK_OP_LOADING && ev->deps_off[e + 1] - ev->deps_off[e] > 1)
                return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: a LOADING event names at most one witness");
        }
    const size_t nd = ev->deps_off[m];
    if (nd && (!ev->deps_msb || !ev->deps_lsb || !ev->deps_node))
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: deps without arrays");
    // every event's deps strictly ascending (a Deps' TxnIds), checked before anything reaches the device: the kernel
    // would otherwise have half-applied the key's events when it met them (the store stays as it was on an error)
    for (size_t e = 0; e < m; ++e)
        for (uint32_t j = ev->deps_off[e] + 1; j < ev->deps_off[e + 1]; ++j)
            if (host_ts_cmp(ev->deps_msb[j - 1], ev->deps_lsb[j - 1], ev->deps_node[j - 1], ev->deps_msb[j], ev->deps_lsb[j],
                            ev->deps_node[j]) >= 0)
                return set_err(h, AD_ERR_UNSORTED, "ad_cfk_store_apply: event " + std::to_string(e) +
                                                       "'s deps are not strictly ascending");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    uint32_t *eo, *doff;
    uint64_t *etm, *etl, *eem, *eel, *dtm, *dtl;
    int32_t *etn, *een, *dtn;
    uint8_t* est;
    const size_t dn = std::max<size_t>(nd, 1);
    CK(dalloc(h, S_CSE0 + 0, &eo, c.K + 1)); CK(dalloc(h, S_CSE0 + 1, &etm, m)); CK(dalloc(h, S_CSE0 + 2, &etl, m));
    CK(dalloc(h, S_CSE0 + 3, &etn, m)); CK(dalloc(h, S_CSE0 + 4, &est, m)); CK(dalloc(h, S_CSE0 + 5, &eem, m));
    CK(dalloc(h, S_CSE0 + 6, &eel, m)); CK(dalloc(h, S_CSE0 + 7, &een, m)); CK(dalloc(h, S_CSE0 + 8, &doff, m + 1));
    CK(dalloc(h, S_CSE0 + 9, &dtm, dn)); CK(dalloc(h, S_CSE0 + 10, &dtl, dn)); CK(dalloc(h, S_CSE0 + 11, &dtn, dn));
    uint8_t* eop = nullptr;
    if (ev->op) {
        CK(dalloc(h, S_CSE0 + 12, &eop, m));
        HIPCHK(h, hipMemcpyAsync(eop, ev->op, m, hipMemcpyHostToDevice, st));
    }
    HIPCHK(h, hipMemcpyAsync(eo, ev->ev_off, (c.K + 1) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(etm, ev->txn_msb, m * 8, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(etl, ev->txn_lsb, m * 8, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(etn, ev->txn_node, m * 4, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(est, ev->status, m, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(eem, ev->exec_msb, m * 8, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(eel, ev->exec_lsb, m * 8, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(een, ev->exec_node, m * 4, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(doff, ev->deps_off, (m + 1) * 4, hipMemcpyHostToDevice, st));
    if (nd) {
        HIPCHK(h, hipMemcpyAsync(dtm, ev->deps_msb, nd * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(dtl, ev->deps_lsb, nd * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(dtn, ev->deps_node, nd * 4, hipMemcpyHostToDevice, st));
    }
    CfkStoreArgs a{};
    cs_tier_args(c, a);
    a.cnt = c.cnt;
    a.tm = c.tm; a.tl = c.tl; a.tn = c.tn; a.em = c.em; a.el = c.el; a.en = c.en; a.st = c.st; a.slot = c.slot; a.bits = c.bits;
    a.ev_off = eo; a.etm = etm; a.etl = etl; a.etn = etn; a.est = est; a.eem = eem; a.eel = eel; a.een = een;
    a.dep_off = doff; a.dtm = dtm; a.dtl = dtl; a.dtn = dtn;
    a.overflow = c.flags; a.bad = c.flags + 1;
    a.pbm = c.pbm; a.pbl = c.pbl; a.pbn = c.pbn; a.lp_cnt = c.lp_cnt; a.lpm = c.lpm; a.lpl = c.lpl; a.lpn = c.lpn;
    a.lp_bits = c.lp_bits; a.eop = eop;
    a.lp_xm = c.lp_xm; a.lp_xl = c.lp_xl; a.lp_xn = c.lp_xn; a.lp_xh = c.lp_xh;
    a.um_cnt = c.um_cnt; a.um_p = c.um_p; a.um_wm = c.um_wm; a.um_wl = c.um_wl; a.um_wn = c.um_wn;
    a.um_tm = c.um_tm; a.um_tl = c.um_tl; a.um_tn = c.um_tn;
    // notifications: per key a region of (its events + the registry's capacity) entries
    {
        std::vector<uint32_t> nb(c.K + 1, 0);
        for (uint32_t k = 0; k < c.K; ++k) nb[k + 1] = nb[k] + (ev->ev_off[k + 1] - ev->ev_off[k]) + std::max(c.cap, c.capB);
        c.nt_base_host = nb;
        const size_t tot = std::max<size_t>(nb[c.K], 1);
        CK(dalloc(h, S_CSU0 + 13, &c.nt_base, c.K + 1)); CK(dalloc(h, S_CSU0 + 14, &c.nt_ev, tot));
        CK(dalloc(h, S_CSU0 + 15, &c.nt_tag, tot)); CK(dalloc(h, S_CSU0 + 16, &c.nt_tm, tot));
        CK(dalloc(h, S_CSU0 + 17, &c.nt_tl, tot)); CK(dalloc(h, S_CSU0 + 18, &c.nt_tn, tot));
        HIPCHK(h, hipMemcpyAsync(c.nt_base, nb.data(), (c.K + 1) * 4, hipMemcpyHostToDevice, st));
        c.ev_off_host.assign(ev->ev_off, ev->ev_off + c.K + 1);
    }
    a.nt_base = c.nt_base; a.nt_cnt = c.nt_cnt; a.nt_ev = c.nt_ev; a.nt_tag = c.nt_tag;
    a.nt_tm = c.nt_tm; a.nt_tl = c.nt_tl; a.nt_tn = c.nt_tn;
    HIPCHK(h, hipMemsetAsync(c.flags, 0, 8, st));          // this call's overflow / order flags
    const char* tmr = getenv("AD_CS_TIMERS");
    uint64_t* dbg = nullptr;
    if (tmr && tmr[0] == '1') {
        HIPCHK(h, hipMalloc(&dbg, 8 * 128));
        HIPCHK(h, hipMemsetAsync(dbg, 0, 8 * 128, st));
    }
    a.dbg = dbg;
    // rows in LDS while the key's events apply when they fit (AD_CFK_STORE_HBM=1: the HBM-resident kernel, for tests)
    const char* hbm = getenv("AD_CFK_STORE_HBM");
    const bool lds_ok = !(hbm && hbm[0] == '1');
    a.kres = c.kres;
    // one pass over the keys (klist: nullptr) or over a list of them; the large-tier keys that do not fit LDS take the
    // HBM kernel
    auto launch = [&](const uint32_t* klist, uint32_t nk, const uint32_t* big_list, uint32_t nbl) {
        CfkStoreArgs x = a;
        x.klist = klist;
        if (lds_ok && c.cap <= CS_LDS_CAP) {
            k_cfk_apply<true><<<nk, CS_T, 0, st>>>(x);
            if (nbl && c.capB > CS_LDS_CAP) {
                x.klist = big_list;
                k_cfk_apply<false><<<nbl, CS_T, 0, st>>>(x);
            }
        } else {
            k_cfk_apply<false><<<nk, CS_T, 0, st>>>(x);
        }
    };
    uint32_t* bl = nullptr;
    if (!c.big_keys.empty()) {
        CK(dalloc(h, S_CSKLIST, &bl, c.big_keys.size()));
        HIPCHK(h, hipMemcpyAsync(bl, c.big_keys.data(), c.big_keys.size() * 4, hipMemcpyHostToDevice, st));
    }
    launch(nullptr, c.K, bl, (uint32_t)c.big_keys.size());
    HIPCHK(h, hipGetLastError());
    // keys that ran out of rows stopped before the event (kres): they move to the large tier and resume from it
    for (int round = 0; c.nbig && round < 2; ++round) {
        uint32_t f0 = 0;
        HIPCHK(h, hipMemcpyAsync(&f0, c.flags, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        if (!f0) break;
        std::vector<uint32_t> kres(c.K);
        HIPCHK(h, hipMemcpy(kres.data(), c.kres, (size_t)c.K * 4, hipMemcpyDeviceToHost));
        std::vector<uint32_t> moved, slots, resumed;
        for (uint32_t k = 0; k < c.K; ++k) {
            if (kres[k] == ~0u) continue;
            if (c.kslot_host[k] != ~0u || c.big_keys.size() >= c.nbig) {
                HIPCHK(h, hipMemsetAsync(c.kres, 0xFF, (size_t)c.K * 4, st));
                HIPCHK(h, hipStreamSynchronize(st));
                return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_store_apply: a key outgrew the store's large tier (rows or "
                                                      "loadingPruned entries, or no large-tier slot left); the key keeps "
                                                      "its state up to the event before");
            }
            c.kslot_host[k] = (uint32_t)c.big_keys.size();
            slots.push_back(c.kslot_host[k]);
            c.big_keys.push_back(k);
            moved.push_back(k);
        }
        const uint32_t nm = (uint32_t)moved.size();
        uint32_t *ml = nullptr, *ms = nullptr;
        CK(dalloc(h, S_CSKLIST, &ml, std::max<size_t>(c.big_keys.size(), nm)));
        CK(dalloc(h, S_CSKNEW, &ms, nm));
        HIPCHK(h, hipMemcpyAsync(ml, moved.data(), nm * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(ms, slots.data(), nm * 4, hipMemcpyHostToDevice, st));
        CfkStoreArgs pa = a;
        pa.klist = ml;
        k_cfk_promote<<<nm, 256, 0, st>>>(pa, ms);
        // resume: each moved key from the event it stopped at (the others skip: ev_start ~0u)
        uint32_t* ks = nullptr;
        CK(dalloc(h, S_CSKSTART, &ks, c.K));
        HIPCHK(h, hipMemcpyAsync(ks, c.kres, (size_t)c.K * 4, hipMemcpyDeviceToDevice, st));
        HIPCHK(h, hipMemsetAsync(c.kres, 0xFF, (size_t)c.K * 4, st));
        HIPCHK(h, hipMemsetAsync(c.flags, 0, 4, st));
        a.ev_start = ks;
        launch(ml, nm, ml, nm);
        a.ev_start = nullptr;
        HIPCHK(h, hipGetLastError());
    }
    uint32_t f[2] = {0, 0};
    HIPCHK(h, hipMemcpyAsync(f, c.flags, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (dbg) {                                   // per key % 8 group: op class (cycles, events)
        uint64_t d[128];
        HIPCHK(h, hipMemcpy(d, dbg, sizeof d, hipMemcpyDeviceToHost));
        hipFree(dbg);
        for (int g = 0; g < 8; ++g) {
            fprintf(stderr, "cs_timers g%d", g);
            for (int k = 0; k < 8; ++k) fprintf(stderr, " %d:%llu/%llu", k, (unsigned long long)d[16 * g + 2 * k], (unsigned long long)d[16 * g + 2 * k + 1]);
            fprintf(stderr, "\n");
        }
    }
    if (f[1]) return set_err(h, AD_ERR_UNSORTED, "ad_cfk_store_apply: an event's deps are not strictly ascending");
    // (the key that ran out is left as far as its last complete event: reopen the store, or fetch it and replay)
    if (f[0]) return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_store_apply: a key outgrew the store's capacity (rows or "
                                                    "loadingPruned entries); the key keeps its state up to the event before");
    return AD_OK;
}

int ad_cfk_store_notify(ad_handle* h, uint32_t* rows, uint8_t* not_waiting) {
    if (!h) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_notify before ad_cfk_store_open");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    HIPCHK(h, hipMemsetAsync(c.flags + 2, 0, 8, st));
    NotifyArgs a{};
    a.K = c.K; a.row_off = nullptr; a.cnt = c.cnt; a.cap = c.cap; a.words = c.words; a.slot = c.slot; a.bits = c.bits;
    a.kslot = c.kslot; a.capB = c.capB; a.wordsB = c.wordsB;
    a.tm = c.tm; a.tl = c.tl; a.tn = c.tn; a.em = c.em; a.el = c.el; a.en = c.en; a.st = c.st;
    a.pre = c.pre; a.out = c.out; a.bad_order = c.flags + 2; a.bad_miss = c.flags + 3;
    a.lp_cnt = c.lp_cnt; a.lpm = c.lpm; a.lpl = c.lpl; a.lpn = c.lpn; a.lp_bits = c.lp_bits;
    k_cfk_notify<<<c.K, NF_T, 0, st>>>(a);
    HIPCHK(h, hipGetLastError());
    if (rows) HIPCHK(h, hipMemcpyAsync(rows, c.cnt, (size_t)c.K * 4, hipMemcpyDeviceToHost, st));
    // not_waiting is [keys * capacity] at the caller's (unrounded) capacity: a 2D copy out of the 64-row-aligned rows
    if (not_waiting)
    {
        HIPCHK(h, hipMemcpy2DAsync(not_waiting, c.ucap, c.out, c.cap, c.ucap, c.K, hipMemcpyDeviceToHost, st));
        // large-tier keys: their first `capacity` rows (ad_cfk_store_notify_key has them all)
        for (uint32_t k : c.big_keys)
            HIPCHK(h, hipMemcpyAsync(not_waiting + (size_t)k * c.ucap, c.out + c.rbase(k), c.ucap, hipMemcpyDeviceToHost, st));
    }
    uint32_t f[2] = {0, 0};
    HIPCHK(h, hipMemcpyAsync(f, c.flags + 2, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (f[0]) return set_err(h, AD_ERR_STATE, "ad_cfk_store_notify: a key's rows are not in byId order");
    return AD_OK;
}

int ad_cfk_store_fetch(ad_handle* h, uint32_t key, size_t* rows, size_t* missing_total, uint64_t* txn_msb,
                       uint64_t* txn_lsb, int32_t* txn_node, uint64_t* exec_msb, uint64_t* exec_lsb, int32_t* exec_node,
                       uint8_t* status, uint32_t* miss_off, uint32_t* missing) {
    if (!h || !rows) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_fetch before ad_cfk_store_open");
    if (key >= c.K) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_fetch: key out of range");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    uint32_t n = 0;
    HIPCHK(h, hipMemcpyAsync(&n, c.cnt + key, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    const size_t base = c.rbase(key);
    const uint32_t words = c.words_of(key);
    std::vector<uint32_t> slot(n);
    std::vector<uint64_t> bits((size_t)n * words);
    if (n) {
        HIPCHK(h, hipMemcpyAsync(slot.data(), c.slot + base, (size_t)n * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(bits.data(), c.bits + c.bbase(key), (size_t)n * words * 8, hipMemcpyDeviceToHost, st));
        if (txn_msb) HIPCHK(h, hipMemcpyAsync(txn_msb, c.tm + base, (size_t)n * 8, hipMemcpyDeviceToHost, st));
        if (txn_lsb) HIPCHK(h, hipMemcpyAsync(txn_lsb, c.tl + base, (size_t)n * 8, hipMemcpyDeviceToHost, st));
        if (txn_node) HIPCHK(h, hipMemcpyAsync(txn_node, c.tn + base, (size_t)n * 4, hipMemcpyDeviceToHost, st));
        if (exec_msb) HIPCHK(h, hipMemcpyAsync(exec_msb, c.em + base, (size_t)n * 8, hipMemcpyDeviceToHost, st));
        if (exec_lsb) HIPCHK(h, hipMemcpyAsync(exec_lsb, c.el + base, (size_t)n * 8, hipMemcpyDeviceToHost, st));
        if (exec_node) HIPCHK(h, hipMemcpyAsync(exec_node, c.en + base, (size_t)n * 4, hipMemcpyDeviceToHost, st));
        if (status) HIPCHK(h, hipMemcpyAsync(status, c.st + base, n, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    // missing() as byId row indices: slot -> row, then each row's bitmap in row order
    std::vector<uint32_t> row_of(n);
    for (uint32_t r = 0; r < n; ++r) {
        if (slot[r] >= n) return set_err(h, AD_ERR_DEVICE, "ad_cfk_store_fetch: slot out of range");
        row_of[slot[r]] = r;
    }
    size_t tot = 0;
    std::vector<uint32_t> tmp;
    for (uint32_t r = 0; r < n; ++r) {
        tmp.clear();
        const uint64_t* b = bits.data() + (size_t)slot[r] * words;
        for (uint32_t w = 0; w < words; ++w)
            for (uint64_t x = b[w]; x; x &= x - 1) {
                const uint32_t s = w * 64 + (uint32_t)__builtin_ctzll(x);
                if (s >= n) return set_err(h, AD_ERR_DEVICE, "ad_cfk_store_fetch: a missing bit beyond the rows");
                tmp.push_back(row_of[s]);
            }
        std::sort(tmp.begin(), tmp.end());
        if (miss_off) miss_off[r] = (uint32_t)tot;
        if (missing) std::copy(tmp.begin(), tmp.end(), missing + tot);
        tot += tmp.size();
    }
    if (miss_off) miss_off[n] = (uint32_t)tot;
    *rows = n;
    if (missing_total) *missing_total = tot;
    return AD_OK;
}

int ad_cfk_store_pruning(ad_handle* h, uint32_t key, uint64_t* pruned_msb, uint64_t* pruned_lsb, int32_t* pruned_node,
                         size_t* loading, size_t* witness_total, uint64_t* lp_msb, uint64_t* lp_lsb, int32_t* lp_node,
                         uint32_t* lp_off, uint32_t* lp_rows) {
    if (!h || !loading) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_pruning before ad_cfk_store_open");
    if (key >= c.K) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_pruning: key out of range");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    uint32_t L = 0, n = 0;
    uint64_t pm = 0, pl = 0;
    int32_t pn = 0;
    HIPCHK(h, hipMemcpyAsync(&L, c.lp_cnt + key, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(&n, c.cnt + key, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(&pm, c.pbm + key, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(&pl, c.pbl + key, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(&pn, c.pbn + key, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (pruned_msb) *pruned_msb = pm;
    if (pruned_lsb) *pruned_lsb = pl;
    if (pruned_node) *pruned_node = pn;
    const size_t base = c.rbase(key);
    const uint32_t words = c.words_of(key);
    std::vector<uint32_t> slot(n);
    std::vector<uint64_t> bits((size_t)L * words);
    if (n) HIPCHK(h, hipMemcpyAsync(slot.data(), c.slot + base, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    if (L) {
        HIPCHK(h, hipMemcpyAsync(bits.data(), c.lp_bits + c.bbase(key), (size_t)L * words * 8, hipMemcpyDeviceToHost, st));
        if (lp_msb) HIPCHK(h, hipMemcpyAsync(lp_msb, c.lpm + base, (size_t)L * 8, hipMemcpyDeviceToHost, st));
        if (lp_lsb) HIPCHK(h, hipMemcpyAsync(lp_lsb, c.lpl + base, (size_t)L * 8, hipMemcpyDeviceToHost, st));
        if (lp_node) HIPCHK(h, hipMemcpyAsync(lp_node, c.lpn + base, (size_t)L * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    std::vector<uint32_t> row_of(c.rows_cap(key), 0xFFFFFFFFu);
    for (uint32_t r = 0; r < n; ++r) {
        if (slot[r] >= n) return set_err(h, AD_ERR_DEVICE, "ad_cfk_store_pruning: slot out of range");
        row_of[slot[r]] = r;
    }
    size_t tot = 0;
    std::vector<uint32_t> tmp;
    for (uint32_t j = 0; j < L; ++j) {
        tmp.clear();
        const uint64_t* b = bits.data() + (size_t)j * words;
        for (uint32_t w = 0; w < words; ++w)
            for (uint64_t x = b[w]; x; x &= x - 1) {
                const uint32_t s = w * 64 + (uint32_t)__builtin_ctzll(x);
                if (s >= n) return set_err(h, AD_ERR_DEVICE, "ad_cfk_store_pruning: a witness bit beyond the rows");
                tmp.push_back(row_of[s]);
            }
        std::sort(tmp.begin(), tmp.end());
        if (lp_off) lp_off[j] = (uint32_t)tot;
        if (lp_rows) std::copy(tmp.begin(), tmp.end(), lp_rows + tot);
        tot += tmp.size();
    }
    if (lp_off) lp_off[L] = (uint32_t)tot;
    *loading = L;
    if (witness_total) *witness_total = tot;
    return AD_OK;
}

// ---- mapReduceActive over the resident rows (cfk_query_kernels.h) ---------------------------------------------------
int ad_cfk_store_query(ad_handle* h, const ad_cfk_queries* q, ad_csr_sizes* sizes) {
    if (!h || !q) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_query before ad_cfk_store_open");
    const size_t nq = q->nq;
    if (nq && (!q->key_off || !q->txn_msb || !q->txn_lsb || !q->txn_node || !q->bound_msb || !q->bound_lsb || !q->bound_node))
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_query: an array is missing");
    if (nq && q->key_off[0] != 0) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_query: key_off must start at 0");
    const size_t items = nq ? q->key_off[nq] : 0;
    if (items && !q->keys) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_query: keys missing");
    std::vector<uint32_t> iq(items);
    for (size_t x = 0; x < nq; ++x) {
        if (q->key_off[x + 1] < q->key_off[x]) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_query: key_off not monotone");
        for (uint32_t j = q->key_off[x]; j < q->key_off[x + 1]; ++j) {
            if (q->keys[j] >= c.K) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_query: key out of range");
            if (j > q->key_off[x] && q->keys[j] <= q->keys[j - 1])
                return set_err(h, AD_ERR_UNSORTED, "ad_cfk_store_query: a query's keys are not strictly ascending");
            iq[j] = (uint32_t)x;
        }
    }
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    auto& r = h->csq;
    r.nq = nq; r.items = items;
    const size_t nq1 = std::max<size_t>(nq, 1), it1 = std::max<size_t>(items, 1);
    CfkQueryArgs a{};
    cs_tier_args(c, a.s);
    a.s.cnt = c.cnt;
    a.s.tm = c.tm; a.s.tl = c.tl; a.s.tn = c.tn; a.s.em = c.em; a.s.el = c.el; a.s.en = c.en; a.s.st = c.st;
    a.s.pbm = c.pbm; a.s.pbl = c.pbl; a.s.pbn = c.pbn;
    a.nq = (uint32_t)nq; a.items = (uint32_t)items;
    uint32_t *qoff, *qkey, *diq, *icnt, *ioff, *qeoff, *icur;
    uint64_t *qtm, *qtl, *qbm, *qbl;
    int32_t *qtn, *qbn;
    CK(dalloc(h, S_CSQ0 + 0, &qoff, nq + 1)); CK(dalloc(h, S_CSQ0 + 1, &qkey, it1)); CK(dalloc(h, S_CSQ0 + 2, &diq, it1));
    CK(dalloc(h, S_CSQ0 + 3, &qtm, nq1)); CK(dalloc(h, S_CSQ0 + 4, &qtl, nq1)); CK(dalloc(h, S_CSQ0 + 5, &qtn, nq1));
    CK(dalloc(h, S_CSQ0 + 6, &qbm, nq1)); CK(dalloc(h, S_CSQ0 + 7, &qbl, nq1)); CK(dalloc(h, S_CSQ0 + 8, &qbn, nq1));
    CK(dalloc(h, S_CSQ0 + 9, &icnt, 2 * it1)); CK(dalloc(h, S_CSQ0 + 10, &ioff, 2 * it1));
    CK(dalloc(h, S_CSQ0 + 11, &qeoff, 2 * (nq + 1))); CK(dalloc(h, S_CSQ0 + 12, &icur, 2 * it1));
    if (nq) {
        HIPCHK(h, hipMemcpyAsync(qoff, q->key_off, (nq + 1) * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(qtm, q->txn_msb, nq * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(qtl, q->txn_lsb, nq * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(qtn, q->txn_node, nq * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(qbm, q->bound_msb, nq * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(qbl, q->bound_lsb, nq * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(qbn, q->bound_node, nq * 4, hipMemcpyHostToDevice, st));
    }
    if (items) {
        HIPCHK(h, hipMemcpyAsync(qkey, q->keys, items * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(diq, iq.data(), items * 4, hipMemcpyHostToDevice, st));
    }
    a.qoff = qoff; a.qkey = qkey; a.iq = diq; a.qtm = qtm; a.qtl = qtl; a.qtn = qtn; a.qbm = qbm; a.qbl = qbl; a.qbn = qbn;
    a.icnt = icnt; a.ioff = ioff; a.qeoff = qeoff; a.icur = icur;
    // count pass -> per (item, class) offsets and per-query entry bases (host: this is the store's query API, not the
    // batch pipeline), then fill and union
    std::vector<uint32_t> cnt(2 * items), off(2 * items), qe(2 * (nq + 1), 0);
    if (items) {
        k_csq_items<false><<<ceil_div((long)items * WAVE, 256), 256, 0, st>>>(a);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipMemcpyAsync(cnt.data(), icnt, items * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    uint64_t tot[2] = {0, 0};
    for (size_t x = 0; x < nq; ++x) {
        for (int cl = 0; cl < 2; ++cl) qe[cl * (nq + 1) + x] = (uint32_t)tot[cl];
        for (uint32_t j = q->key_off[x]; j < q->key_off[x + 1]; ++j)
            for (int cl = 0; cl < 2; ++cl) { off[2 * j + cl] = (uint32_t)tot[cl]; tot[cl] += cnt[2 * j + cl]; }
    }
    for (int cl = 0; cl < 2; ++cl) qe[cl * (nq + 1) + nq] = (uint32_t)tot[cl];
    if (tot[0] + items > 0xFFFFFFFFull || tot[1] + items > 0xFFFFFFFFull)
        return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_store_query: more than 2^32 entries");
    if (items) HIPCHK(h, hipMemcpyAsync(ioff, off.data(), items * 8, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(qeoff, qe.data(), qe.size() * 4, hipMemcpyHostToDevice, st));
    for (int cl = 0; cl < 2; ++cl) {
        const size_t e1 = std::max<size_t>(tot[cl], 1);
        CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 0, &a.lm[cl], e1)); CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 1, &a.ll[cl], e1));
        CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 2, &a.ln[cl], e1)); CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 3, &a.okeys[cl], it1));
        CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 4, &a.ok2t[cl], items + tot[cl] + 1));
        CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 5, &a.otm[cl], e1)); CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 6, &a.otl[cl], e1));
        CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 7, &a.otn[cl], e1));
        CK(dalloc(h, S_CSQ0 + 13 + 10 * cl + 8, &a.okc[cl], 3 * nq1));
        a.oen[cl] = a.okc[cl] + nq1; a.otc[cl] = a.okc[cl] + 2 * nq1;
        r.lists[cl] = tot[cl];
        r.okeys[cl] = a.okeys[cl]; r.ok2t[cl] = a.ok2t[cl]; r.otm[cl] = a.otm[cl]; r.otl[cl] = a.otl[cl]; r.otn[cl] = a.otn[cl];
        r.okc[cl] = a.okc[cl]; r.oen[cl] = a.oen[cl]; r.otc[cl] = a.otc[cl];
    }
    r.qe = qe;
    r.qoff.assign(q->key_off, q->key_off + nq + 1);
    if (items) k_csq_items<true><<<ceil_div((long)items * WAVE, 256), 256, 0, st>>>(a);
    if (nq) k_csq_union<<<ceil_div((long)nq * 2, 256), 256, 0, st>>>(a);
    HIPCHK(h, hipGetLastError());
    std::vector<uint32_t> counts[2];
    for (int cl = 0; cl < 2; ++cl) {
        counts[cl].resize(3 * nq1);
        if (nq) HIPCHK(h, hipMemcpyAsync(counts[cl].data(), a.okc[cl], 3 * nq1 * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    for (int cl = 0; cl < 2; ++cl) {
        r.kc[cl].assign(counts[cl].begin(), counts[cl].begin() + nq);
        r.en[cl].assign(counts[cl].begin() + nq1, counts[cl].begin() + nq1 + nq);
        r.tc[cl].assign(counts[cl].begin() + 2 * nq1, counts[cl].begin() + 2 * nq1 + nq);
        size_t k = 0, m = 0, t = 0;
        for (size_t x = 0; x < nq; ++x) { k += r.kc[cl][x]; m += r.kc[cl][x] + r.en[cl][x]; t += r.tc[cl][x]; }
        if (sizes) sizes[cl] = ad_csr_sizes{nq, k, m, t, t};
    }
    r.ready = true;
    return AD_OK;
}

int ad_cfk_store_query_fetch(ad_handle* h, uint32_t cls, ad_csr_out* out, uint64_t* txn_msb, uint64_t* txn_lsb, int32_t* txn_node) {
    if (!h || !out || cls > 1) return AD_ERR_ARGUMENT;
    auto& r = h->csq;
    if (!r.ready) return set_err(h, AD_ERR_STATE, "ad_cfk_store_query_fetch before ad_cfk_store_query");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const size_t nq = r.nq, items = r.items, e = r.lists[cls];
    std::vector<uint64_t> keys(std::max<size_t>(items, 1)), tm(std::max<size_t>(e, 1)), tl(std::max<size_t>(e, 1));
    std::vector<int32_t> k2t(items + e + 1), tn(std::max<size_t>(e, 1));
    if (items) HIPCHK(h, hipMemcpyAsync(keys.data(), r.okeys[cls], items * 8, hipMemcpyDeviceToHost, st));
    if (items + e) HIPCHK(h, hipMemcpyAsync(k2t.data(), r.ok2t[cls], (items + e) * 4, hipMemcpyDeviceToHost, st));
    if (e) {
        HIPCHK(h, hipMemcpyAsync(tm.data(), r.otm[cls], e * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(tl.data(), r.otl[cls], e * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(tn.data(), r.otn[cls], e * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    size_t ko = 0, mo = 0, to = 0;
    out->key_off[0] = 0; out->k2t_off[0] = 0; out->txn_off[0] = 0;
    for (size_t x = 0; x < nq; ++x) {
        const uint32_t i0 = r.qoff[x], eb = r.qe[cls * (nq + 1) + x];
        const uint32_t nk = r.kc[cls][x], nm = nk + r.en[cls][x], nt = r.tc[cls][x];
        for (uint32_t j = 0; j < nk; ++j) out->keys[ko + j] = keys[i0 + j];
        for (uint32_t j = 0; j < nm; ++j) out->k2t[mo + j] = k2t[i0 + eb + j];
        for (uint32_t j = 0; j < nt; ++j) {
            if (txn_msb) txn_msb[to + j] = tm[eb + j];
            if (txn_lsb) txn_lsb[to + j] = tl[eb + j];
            if (txn_node) txn_node[to + j] = tn[eb + j];
            if (out->txns) out->txns[to + j] = (uint32_t)(to + j);
        }
        ko += nk; mo += nm; to += nt;
        out->key_off[x + 1] = (uint32_t)ko; out->k2t_off[x + 1] = (uint32_t)mo; out->txn_off[x + 1] = (uint32_t)to;
    }
    return AD_OK;
}

// ---- the unmanaged registry and the last apply's unmanaged notifications -----------------------------------------
int ad_cfk_store_unmanaged(ad_handle* h, uint32_t key, size_t* count, uint8_t* pending, uint64_t* wait_msb,
                           uint64_t* wait_lsb, int32_t* wait_node, uint64_t* txn_msb, uint64_t* txn_lsb, int32_t* txn_node) {
    if (!h || !count) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_unmanaged before ad_cfk_store_open");
    if (key >= c.K) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_unmanaged: key out of range");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    uint32_t U = 0;
    HIPCHK(h, hipMemcpyAsync(&U, c.um_cnt + key, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    *count = U;
    const size_t b = c.rbase(key);
    if (U) {
        if (pending) HIPCHK(h, hipMemcpyAsync(pending, c.um_p + b, U, hipMemcpyDeviceToHost, st));
        if (wait_msb) HIPCHK(h, hipMemcpyAsync(wait_msb, c.um_wm + b, U * 8, hipMemcpyDeviceToHost, st));
        if (wait_lsb) HIPCHK(h, hipMemcpyAsync(wait_lsb, c.um_wl + b, U * 8, hipMemcpyDeviceToHost, st));
        if (wait_node) HIPCHK(h, hipMemcpyAsync(wait_node, c.um_wn + b, U * 4, hipMemcpyDeviceToHost, st));
        if (txn_msb) HIPCHK(h, hipMemcpyAsync(txn_msb, c.um_tm + b, U * 8, hipMemcpyDeviceToHost, st));
        if (txn_lsb) HIPCHK(h, hipMemcpyAsync(txn_lsb, c.um_tl + b, U * 8, hipMemcpyDeviceToHost, st));
        if (txn_node) HIPCHK(h, hipMemcpyAsync(txn_node, c.um_tn + b, U * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    return AD_OK;
}

int ad_cfk_store_notified(ad_handle* h, uint32_t* counts, size_t* total, uint32_t* event, uint8_t* tag, uint64_t* txn_msb,
                          uint64_t* txn_lsb, int32_t* txn_node) {
    if (!h || !total) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_notified before ad_cfk_store_open");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    std::vector<uint32_t> cnt(c.K);
    HIPCHK(h, hipMemcpyAsync(cnt.data(), c.nt_cnt, (size_t)c.K * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    size_t tot = 0;
    for (uint32_t k = 0; k < c.K; ++k) { if (counts) counts[k] = cnt[k]; tot += cnt[k]; }
    *total = tot;
    if (!event && !tag && !txn_msb && !txn_lsb && !txn_node) return AD_OK;
    size_t o = 0;
    for (uint32_t k = 0; k < c.K && tot; ++k) {
        if (!cnt[k]) continue;
        const size_t b = c.nt_base_host[k];
        if (event) {
            HIPCHK(h, hipMemcpyAsync(event + o, c.nt_ev + b, cnt[k] * 4, hipMemcpyDeviceToHost, st));
        }
        if (tag) HIPCHK(h, hipMemcpyAsync(tag + o, c.nt_tag + b, cnt[k], hipMemcpyDeviceToHost, st));
        if (txn_msb) HIPCHK(h, hipMemcpyAsync(txn_msb + o, c.nt_tm + b, cnt[k] * 8, hipMemcpyDeviceToHost, st));
        if (txn_lsb) HIPCHK(h, hipMemcpyAsync(txn_lsb + o, c.nt_tl + b, cnt[k] * 8, hipMemcpyDeviceToHost, st));
        if (txn_node) HIPCHK(h, hipMemcpyAsync(txn_node + o, c.nt_tn + b, cnt[k] * 4, hipMemcpyDeviceToHost, st));
        o += cnt[k];
    }
    HIPCHK(h, hipStreamSynchronize(st));
    if (event) {                                 // event indices relative to the key's events of the call
        o = 0;
        for (uint32_t k = 0; k < c.K; ++k) {
            for (uint32_t i = 0; i < cnt[k]; ++i) event[o + i] -= c.ev_off_host[k];
            o += cnt[k];
        }
    }
    return AD_OK;
}

// After ad_cfk_store_notify: key's notWaiting flags for all of its rows (a large-tier key can hold more rows than the
// bulk call's [keys x capacity] output has room for).  rows_cap: the caller's room; *rows: the key's rows.
int ad_cfk_store_notify_key(ad_handle* h, uint32_t key, uint8_t* not_waiting, size_t rows_cap, size_t* rows) {
    if (!h || !rows) return AD_ERR_ARGUMENT;
    auto& c = h->cs;
    if (!c.K) return set_err(h, AD_ERR_STATE, "ad_cfk_store_notify_key before ad_cfk_store_open");
    if (key >= c.K) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_notify_key: key out of range");
    hipSetDevice(h->device);
    uint32_t n = 0;
    HIPCHK(h, hipMemcpyAsync(&n, c.cnt + key, 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    *rows = n;
    if (not_waiting && n) {
        if (rows_cap < n) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_notify_key: not_waiting holds fewer than the key's rows");
        HIPCHK(h, hipMemcpyAsync(not_waiting, c.out + c.rbase(key), n, hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
    }
    return AD_OK;
}
