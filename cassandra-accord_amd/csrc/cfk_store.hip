// cfk_store.hip — ad_cfk_store_*: device-resident CommandsForKey states driven by CommandsForKey.update events
// (cfk_store_kernels.h), with CommandsForKey.notifyManaged's release rule over the resident rows (notify_kernels.h).
#include "engine_internal.h"

int ad_cfk_store_open(ad_handle* h, uint32_t keys, uint32_t capacity) {
    if (!h) return AD_ERR_ARGUMENT;
    if (keys == 0 || capacity == 0 || capacity > 64 * NF_MAX_WORDS)
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_open: keys >= 1 and 1 <= capacity <= 8192");
    hipSetDevice(h->device);
    auto& c = h->cs;
    c.K = keys;
    c.cap = (capacity + 63) & ~63u;
    c.words = c.cap / 64;
    const size_t rows = (size_t)c.K * c.cap;
    CK(dalloc(h, S_CS0 + 0, &c.cnt, c.K)); CK(dalloc(h, S_CS0 + 1, &c.tm, rows)); CK(dalloc(h, S_CS0 + 2, &c.tl, rows));
    CK(dalloc(h, S_CS0 + 3, &c.tn, rows)); CK(dalloc(h, S_CS0 + 4, &c.em, rows)); CK(dalloc(h, S_CS0 + 5, &c.el, rows));
    CK(dalloc(h, S_CS0 + 6, &c.en, rows)); CK(dalloc(h, S_CS0 + 7, &c.st, rows)); CK(dalloc(h, S_CS0 + 8, &c.slot, rows));
    CK(dalloc(h, S_CS0 + 9, &c.bits, rows * c.words)); CK(dalloc(h, S_CS0 + 10, &c.out, rows));
    CK(dalloc(h, S_CS0 + 11, &c.pre, 2 * rows)); CK(dalloc(h, S_CS0 + 12, &c.flags, 4));
    CK(dalloc(h, S_CS0 + 13, &c.pbm, c.K)); CK(dalloc(h, S_CS0 + 14, &c.pbl, c.K)); CK(dalloc(h, S_CS0 + 15, &c.pbn, c.K));
    CK(dalloc(h, S_CS0 + 16, &c.lp_cnt, c.K)); CK(dalloc(h, S_CS0 + 17, &c.lpm, rows));
    CK(dalloc(h, S_CS0 + 18, &c.lpl, rows)); CK(dalloc(h, S_CS0 + 19, &c.lpn, rows));
    CK(dalloc(h, S_CS0 + 20, &c.lp_bits, rows * c.words));
    HIPCHK(h, hipMemsetAsync(c.pbm, 0, (size_t)c.K * 8, h->st));
    HIPCHK(h, hipMemsetAsync(c.pbl, 0, (size_t)c.K * 8, h->st));
    HIPCHK(h, hipMemsetAsync(c.pbn, 0, (size_t)c.K * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.lp_cnt, 0, (size_t)c.K * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.cnt, 0, (size_t)c.K * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.flags, 0, 16, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
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
    if (m == 0) return AD_OK;
    if (!ev->txn_msb || !ev->txn_lsb || !ev->txn_node || !ev->status || !ev->exec_msb || !ev->exec_lsb || !ev->exec_node)
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: an event array is missing");
    for (size_t e = 0; e < m; ++e)
        if (ev->status[e] > AD_ST_INVALID) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: status out of range");
    if (ev->op)
        for (size_t e = 0; e < m; ++e) {
            if (ev->op[e] > AD_CFK_OP_LOADING) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: op out of range");
            if (ev->op[e] == AD_CFK_OP_PRUNE && ev->exec_node[e] < 0)
                return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: a PRUNE event's interval (exec_node) is negative");
            if (ev->op[e] == AD_CFK_OP_LOADING && ev->deps_off[e + 1] - ev->deps_off[e] > 1)
                return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: a LOADING event names at most one witness");
        }
    const size_t nd = ev->deps_off[m];
    if (nd && (!ev->deps_msb || !ev->deps_lsb || !ev->deps_node))
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_store_apply: deps without arrays");
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
    a.K = c.K; a.cap = c.cap; a.words = c.words; a.cnt = c.cnt;
    a.tm = c.tm; a.tl = c.tl; a.tn = c.tn; a.em = c.em; a.el = c.el; a.en = c.en; a.st = c.st; a.slot = c.slot; a.bits = c.bits;
    a.ev_off = eo; a.etm = etm; a.etl = etl; a.etn = etn; a.est = est; a.eem = eem; a.eel = eel; a.een = een;
    a.dep_off = doff; a.dtm = dtm; a.dtl = dtl; a.dtn = dtn;
    a.overflow = c.flags; a.bad = c.flags + 1;
    a.pbm = c.pbm; a.pbl = c.pbl; a.pbn = c.pbn; a.lp_cnt = c.lp_cnt; a.lpm = c.lpm; a.lpl = c.lpl; a.lpn = c.lpn;
    a.lp_bits = c.lp_bits; a.eop = eop;
    k_cfk_apply<<<c.K, CS_T, 0, st>>>(a);
    HIPCHK(h, hipGetLastError());
    uint32_t f[2] = {0, 0};
    HIPCHK(h, hipMemcpyAsync(f, c.flags, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (f[1]) return set_err(h, AD_ERR_UNSORTED, "ad_cfk_store_apply: an event's deps are not strictly ascending");
    if (f[0]) return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_store_apply: a key outgrew the store's capacity");
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
    a.tm = c.tm; a.tl = c.tl; a.tn = c.tn; a.em = c.em; a.el = c.el; a.en = c.en; a.st = c.st;
    a.pre = c.pre; a.out = c.out; a.bad_order = c.flags + 2; a.bad_miss = c.flags + 3;
    a.lp_cnt = c.lp_cnt; a.lpm = c.lpm; a.lpl = c.lpl; a.lpn = c.lpn; a.lp_bits = c.lp_bits;
    k_cfk_notify<<<c.K, NF_T, 0, st>>>(a);
    HIPCHK(h, hipGetLastError());
    if (rows) HIPCHK(h, hipMemcpyAsync(rows, c.cnt, (size_t)c.K * 4, hipMemcpyDeviceToHost, st));
    if (not_waiting) HIPCHK(h, hipMemcpyAsync(not_waiting, c.out, (size_t)c.K * c.cap, hipMemcpyDeviceToHost, st));
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
    const size_t base = (size_t)key * c.cap;
    std::vector<uint32_t> slot(n);
    std::vector<uint64_t> bits((size_t)n * c.words);
    if (n) {
        HIPCHK(h, hipMemcpyAsync(slot.data(), c.slot + base, (size_t)n * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(bits.data(), c.bits + base * c.words, (size_t)n * c.words * 8, hipMemcpyDeviceToHost, st));
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
        const uint64_t* b = bits.data() + (size_t)slot[r] * c.words;
        for (uint32_t w = 0; w < c.words; ++w)
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
    const size_t base = (size_t)key * c.cap;
    std::vector<uint32_t> slot(n);
    std::vector<uint64_t> bits((size_t)L * c.words);
    if (n) HIPCHK(h, hipMemcpyAsync(slot.data(), c.slot + base, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    if (L) {
        HIPCHK(h, hipMemcpyAsync(bits.data(), c.lp_bits + base * c.words, (size_t)L * c.words * 8, hipMemcpyDeviceToHost, st));
        if (lp_msb) HIPCHK(h, hipMemcpyAsync(lp_msb, c.lpm + base, (size_t)L * 8, hipMemcpyDeviceToHost, st));
        if (lp_lsb) HIPCHK(h, hipMemcpyAsync(lp_lsb, c.lpl + base, (size_t)L * 8, hipMemcpyDeviceToHost, st));
        if (lp_node) HIPCHK(h, hipMemcpyAsync(lp_node, c.lpn + base, (size_t)L * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    std::vector<uint32_t> row_of(c.cap, 0xFFFFFFFFu);
    for (uint32_t r = 0; r < n; ++r) {
        if (slot[r] >= n) return set_err(h, AD_ERR_DEVICE, "ad_cfk_store_pruning: slot out of range");
        row_of[slot[r]] = r;
    }
    size_t tot = 0;
    std::vector<uint32_t> tmp;
    for (uint32_t j = 0; j < L; ++j) {
        tmp.clear();
        const uint64_t* b = bits.data() + (size_t)j * c.words;
        for (uint32_t w = 0; w < c.words; ++w)
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
