// shard.hip — CFK history across batches and key-range sharding (export, RCCL exchange, home merge, level rounds).
#include "engine_internal.h"

#include <algorithm>

extern "C" {
// ---------------------------------------------------------------------------------------------------
// Key-range sharding across GPUs (shard_kernels.h)
// ---------------------------------------------------------------------------------------------------
static size_t align8(size_t x) { return (x + 7) & ~(size_t)7; }

int ad_cfk_retain(ad_handle* h, size_t* retained) {
    if (!h) return AD_ERR_ARGUMENT;
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_cfk_retain: run ad_preaccept_deps on the batch first");
    if (h->sharded) return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_retain: not in sharded mode");
    if (h->Q) return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_retain: key batches only (no range txns)");
    if (h->stage_pending) return set_err(h, AD_ERR_STATE, "ad_cfk_retain: a batch is staged (ad_load_batch_commit it first)");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    CK(complete_entries(h));
    hipStream_t st = h->st;
    const size_t n = h->n, P = h->P;
    const uint32_t* gid = h->hist_active ? h->gid : nullptr;
    // the next batch's first global rank; every later query's window starts at or above next - W
    uint64_t last_g = 0, last_ts = 0;
    if (n) {
        uint32_t lg = (uint32_t)(n - 1);
        if (gid) HIPCHK(h, hipMemcpyAsync(&lg, gid + n - 1, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(&last_ts, h->tx_ts + n - 1, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        last_g = lg;
    }
    const uint64_t next = n ? last_g + 1 : h->hist_next;
    const uint64_t wlo = h->cfg.window == 0 ? next : (next > h->cfg.window ? next - h->cfg.window : 0);
    uint8_t* keep = nullptr;
    unsigned long long* segmax = nullptr;
    uint32_t *rows = nullptr, *tot = nullptr;
    CK(dalloc(h, S_HKEEP, &keep, std::max<size_t>(n, 1)));
    CK(dalloc(h, S_HSEGM, &segmax, std::max<size_t>(P, 1)));
    CK(dalloc(h, S_HROWS2, &rows, std::max<size_t>(n, 1) + 16));
    tot = rows + std::max<size_t>(n, 1);
    uint32_t H = 0;
    if (n) {
        HIPCHK(h, hipMemsetAsync(keep, 0, n, st));
        if (P) {
            HIPCHK(h, hipMemsetAsync(segmax, 0, P * 8, st));
            const int g = ceil_div((long)P, 256);
            k_hist_seg_wmax<<<g, 256, 0, st>>>(P, h->seg_start, h->e_meta, h->e_exec1, last_ts + 1, segmax);
            k_hist_keep<<<g, 256, 0, st>>>(P, h->seg_start, h->e_txn, h->e_meta, h->e_exec1, segmax, gid, wlo, keep);
        }
        device_scan(CompactFlagOp{keep, rows, tot, n}, n, (uint32_t*)h->scratch, st);
        HIPCHK(h, hipMemcpyAsync(&H, tot, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    // the kept rows (own slots: the next load overwrites the batch arrays)
    uint64_t *otm, *otl, *oem, *oel, *okeys;
    int32_t *otn, *oen;
    uint8_t* ost;
    uint32_t *okoff, *ogid, *ocnt;
    const size_t H1 = std::max<size_t>(H, 1);
    CK(dalloc(h, S_HTM, &otm, H1)); CK(dalloc(h, S_HTL, &otl, H1)); CK(dalloc(h, S_HTN, &otn, H1));
    CK(dalloc(h, S_HEM, &oem, H1)); CK(dalloc(h, S_HEL, &oel, H1)); CK(dalloc(h, S_HEN, &oen, H1));
    CK(dalloc(h, S_HST, &ost, H1)); CK(dalloc(h, S_HKOFF, &okoff, H1 + 1)); CK(dalloc(h, S_HGIDS, &ogid, H1));
    CK(dalloc(h, S_HCNT, &ocnt, H1 + 16));
    uint32_t HP = 0;
    if (H) {
        HistGather g{};
        g.H = H; g.rows = rows; g.tm = h->tm; g.tl = h->tl; g.em = h->em; g.el = h->el; g.tn = h->tn; g.en = h->en;
        g.st = h->status; g.key_off = h->key_off; g.gid = gid;
        g.otm = otm; g.otl = otl; g.oem = oem; g.oel = oel; g.otn = otn; g.oen = oen; g.ost = ost; g.ocnt = ocnt; g.ogid = ogid;
        k_hist_gather_rows<<<ceil_div((long)H, 256), 256, 0, st>>>(g);
        scan_offsets(h, ocnt, okoff, H);
        HIPCHK(h, hipMemcpyAsync(&HP, okoff + H, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        CK(dalloc(h, S_HKEYS, &okeys, std::max<size_t>(HP, 1)));
        k_hist_gather_keys<<<ceil_div((long)H, 256), 256, 0, st>>>(H, rows, h->key_off, h->keys, okoff, okeys);
    }
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(st));
    h->hist_n = H;
    h->hist_p = HP;
    h->hist_next = next;
    h->hist_valid = true;
    if (retained) *retained = H;
    return AD_OK;
}

// Status transitions of kept rows between batches (after ad_cfk_retain, before the next ad_load_batch): all m
// are checked on the device first (held, legal per CommandsForKeyTest's table, executeAt rules); any refusal
// applies none.
int ad_cfk_update(ad_handle* h, size_t m, const uint32_t* gid, const uint8_t* status, const uint64_t* exec_msb,
                  const uint64_t* exec_lsb, const int32_t* exec_node) {
    if (!h || (m && (!gid || !status))) return AD_ERR_ARGUMENT;
    if ((exec_msb != nullptr) != (exec_lsb != nullptr) || (exec_msb != nullptr) != (exec_node != nullptr))
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_update: executeAt is all three arrays or none");
    if (!h->hist_valid) return set_err(h, AD_ERR_STATE, "ad_cfk_update: ad_cfk_retain first (updates apply to the kept rows)");
    for (size_t i = 0; i < m; ++i) {
        if (i && gid[i] <= gid[i - 1]) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_update: gid must be strictly ascending");
        if (status[i] > AD_ST_INVALID) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_update: status out of range");
    }
    if (m == 0) return AD_OK;
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    // staging: gid, status, executeAt (8-aligned sections), then the per-update rows and the refusal flag
    const size_t o_st = m * 4, o_m = (o_st + m + 7) & ~(size_t)7, o_l = o_m + m * 8, o_n = o_l + m * 8;
    const size_t o_row = (o_n + m * 4 + 7) & ~(size_t)7, o_bad = o_row + m * 4, total = o_bad + 64;
    uint8_t* buf = nullptr;
    CK(dalloc(h, S_CFKU, &buf, total));
    HIPCHK(h, hipMemcpyAsync(buf, gid, m * 4, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(buf + o_st, status, m, hipMemcpyHostToDevice, st));
    if (exec_msb) {
        HIPCHK(h, hipMemcpyAsync(buf + o_m, exec_msb, m * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(buf + o_l, exec_lsb, m * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(buf + o_n, exec_node, m * 4, hipMemcpyHostToDevice, st));
    }
    HIPCHK(h, hipMemsetAsync(buf + o_bad, 0, 4, st));
    CfkUpdate a{};
    a.m = m; a.H = h->hist_n;
    a.ugid = (const uint32_t*)buf; a.ust = buf + o_st;
    if (exec_msb) { a.um = (const uint64_t*)(buf + o_m); a.ul = (const uint64_t*)(buf + o_l); a.un = (const int32_t*)(buf + o_n); }
    a.hgid = (const uint32_t*)h->bufs[S_HGIDS].p;
    a.htm = (const uint64_t*)h->bufs[S_HTM].p; a.htl = (const uint64_t*)h->bufs[S_HTL].p; a.htn = (const int32_t*)h->bufs[S_HTN].p;
    a.hst = (uint8_t*)h->bufs[S_HST].p;
    a.hem = (uint64_t*)h->bufs[S_HEM].p; a.hel = (uint64_t*)h->bufs[S_HEL].p; a.hen = (int32_t*)h->bufs[S_HEN].p;
    a.row = (uint32_t*)(buf + o_row); a.bad = (uint32_t*)(buf + o_bad);
    const int g = ceil_div((long)m, 256);
    k_cfk_update_check<<<g, 256, 0, st>>>(a);
    uint32_t bad = 0;
    HIPCHK(h, hipMemcpyAsync(&bad, a.bad, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (bad) {
        std::vector<uint32_t> rows(m);
        HIPCHK(h, hipMemcpyAsync(rows.data(), a.row, m * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        for (size_t i = 0; i < m; ++i) {
            if (!(rows[i] & 0x80000000u)) continue;
            const uint32_t why = rows[i] & 0xFF;
            const char* what = why == CU_NOT_HELD ? "not a kept row (never loaded, or pruned as applied / invalidated)"
                             : why == CU_TRANSITION ? "not a legal status transition (CommandsForKeyTest TRANSITIONS)"
                                                    : "executeAt below the TxnId, or changed after commit";
            return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_update: gid " + std::to_string(gid[i]) + ": " + what);
        }
    }
    k_cfk_update_apply<<<g, 256, 0, st>>>(a);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(st));
    return AD_OK;
}

int ad_cfk_reset(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    h->hist_valid = false;
    h->hist_n = h->hist_p = 0;
    h->hist_next = 0;
    return AD_OK;
}

int ad_cfk_rows(ad_handle* h, size_t* hist_rows, uint32_t* gid) {
    if (!h || !hist_rows) return AD_ERR_ARGUMENT;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "ad_cfk_rows: no batch loaded");
    hipSetDevice(h->device);
    *hist_rows = h->hist_active ? h->hist_rows : 0;
    if (gid && h->n) {
        if (h->hist_active) {
            HIPCHK(h, hipMemcpyAsync(gid, h->gid, h->n * 4, hipMemcpyDeviceToHost, h->st));
            HIPCHK(h, hipStreamSynchronize(h->st));
        } else {
            for (size_t i = 0; i < h->n; ++i) gid[i] = (uint32_t)i;
        }
    }
    return AD_OK;
}

int ad_shard_setup(ad_handle* h, const uint32_t* gid, const uint8_t* home_store, uint32_t self, uint32_t world, size_t n_global) {
    if (!h || (!gid && h->n) || (!home_store && h->n) || world == 0 || world > (uint32_t)MAX_STORES || self >= world)
        return AD_ERR_ARGUMENT;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "ad_shard_setup: load the store's batch first");
    if (h->hist_active) return set_err(h, AD_ERR_UNSUPPORTED, "ad_shard_setup: the batch carries CFK history rows");
    hipSetDevice(h->device);
    const size_t n = h->n;
    for (size_t i = 0; i < n; ++i) {
        if (gid[i] >= n_global || (i > 0 && gid[i] <= gid[i - 1])) return set_err(h, AD_ERR_ARGUMENT, "gid must be ascending global ranks < n_global");
        if (home_store[i] >= world) return set_err(h, AD_ERR_ARGUMENT, "home store out of range");
    }
    std::vector<uint8_t> home(n);
    for (size_t i = 0; i < n; ++i) home[i] = home_store[i] == self ? 1 : 0;
    h->home_host.assign(home_store, home_store + n);
    h->holders_host.clear();
    h->ks_levels = false;
    h->ks_phase = -1;
    CK(dalloc(h, S_GID, &h->gid, n)); CK(dalloc(h, S_HOME, &h->home, n)); CK(dalloc(h, S_HSTORE, &h->hstore, n));
    if (n) {
        HIPCHK(h, hipMemcpyAsync(h->gid, gid, n * 4, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->home, home.data(), n, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->hstore, home_store, n, hipMemcpyHostToDevice, h->st));
    }
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->sharded = true;
    h->n_global = n_global;
    h->self = self;
    h->world = world;
    h->holders = nullptr;
    h->dcnt.assign(world, 0);
    h->have_deps = h->have_merged = h->have_levels = false;
    return AD_OK;
}

// Blob of one destination: header u64[3 + 3 nvc] = {magic, rows, nvc, per vc (keys, k2t, txns)}, then
// gid[rows], then per vc key_off[rows+1] k2t_off[rows+1] ent_off[rows+1] tcnt[rows] keys k2t txns (8-aligned).
// nvc = 2R (key, direct per view) or 3R (then RangeDeps per view follow: vc >= 2R, keys = (start, end) pairs);
// the header word holds nvc | (number of RangeDeps classes) << 16.
static size_t blob_layout(size_t rows, int nvc, int nv, const uint32_t* cnt /* [nvc*3] */, uint64_t* sec /* [SEC_PER_DEST] or null */) {
    size_t off = align8((3 + 3 * (size_t)nvc) * 8);
    if (sec) sec[0] = off;
    off = align8(off + rows * 4);
    for (int c = 0; c < nvc; ++c) {
        const size_t nk = cnt[3 * c], nm = cnt[3 * c + 1], nt = cnt[3 * c + 2];
        const size_t kw = c >= 2 * nv ? 2 : 1;
        const size_t sz[7] = {(rows + 1) * 4, (rows + 1) * 4, (rows + 1) * 4, rows * 4, nk * 8 * kw, nm * 4, nt * 4};
        for (int k = 0; k < 7; ++k) {
            if (sec) sec[1 + 7 * c + k] = off;
            off = align8(off + sz[k]);
        }
    }
    return off;
}

}  // extern "C"

// exported CSR vc of the store: key / direct per view, then RangeDeps per view
static const Csr& export_csr(ad_handle* h, int vc) {
    const int nvc2 = 2 * (int)h->cfg.replicas;
    return vc < nvc2 ? h->deps[vc] : h->rdeps[vc - nvc2];
}

template <int NVC>
void launch_export_offsets(ad_handle* h, size_t K, const uint32_t* list, const ExportOffs& o) {
    ExportOffsetsOp<NVC> op{};
    op.list = list; op.n = K;
    for (int c = 0; c < NVC; ++c) {
        const Csr& x = export_csr(h, c);
        op.key_off[c] = x.key_off; op.k2t_off[c] = x.k2t_off; op.tcnt[c] = x.tcnt;
        op.ok[c] = o.ok[c]; op.om[c] = o.om[c]; op.ot[c] = o.ot[c];
    }
    device_scan(op, K, (typename ExportOffsetsOp<NVC>::S*)h->scratch, h->st);
}

template <int NV>
void launch_export_offsets_nv(ad_handle* h, size_t K, const uint32_t* list, const ExportOffs& o) {
    if (h->Q > 0) launch_export_offsets<3 * NV>(h, K, list, o);
    else launch_export_offsets<2 * NV>(h, K, list, o);
}

extern "C" {

// Pack this store's deps rows (every view, key + direct class, and RangeDeps when the store holds range
// txns) per destination store: the local txns homed at destination d that have deps here, TxnIds as global
// ranks.  bytes[d] = blob size for d.
int ad_shard_export(ad_handle* h, uint64_t* bytes /* [world] */) {
    if (!h || !bytes) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->sharded || !h->have_deps) return set_err(h, AD_ERR_STATE, "ad_shard_export: ad_shard_setup + ad_preaccept_deps first");
    hipSetDevice(h->device);
    const size_t n = h->n;
    const int nv = (int)h->cfg.replicas;
    const int nvc = (h->Q > 0 ? 3 : 2) * nv;
    const uint32_t W = h->world;
    hipStream_t st = h->st;
    // 1. rows with deps, partitioned by destination
    uint32_t *rank = nullptr, *list = nullptr, *xtot = h->totd;              // totals: totd[0..MAX_STORES)
    CK(dalloc(h, S_XRANK, &rank, n)); CK(dalloc(h, S_XLIST, &list, n));
    std::vector<uint32_t> tot(MAX_STORES, 0);
    if (n) {
        DestOp op{};
        op.dest = h->hstore; op.nvc = nvc; op.rank = rank; op.totals = xtot; op.n = n;
        for (int c = 0; c < nvc; ++c) op.tcnt[c] = export_csr(h, c).tcnt;
        device_scan(op, n, (DestOp::S*)h->scratch, st);
        k_export_list<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->hstore, rank, xtot, list);
        HIPCHK(h, hipMemcpyAsync(tot.data(), xtot, MAX_STORES * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    size_t K = 0;
    for (uint32_t d = 0; d < W; ++d) K += tot[d];
    // 2. offsets over the export list, read at every destination boundary
    uint32_t* xoff = nullptr;
    CK(dalloc(h, S_XOFF, &xoff, (size_t)3 * nvc * (K + 1)));
    ExportOffs o{};
    for (int c = 0; c < nvc; ++c) {
        o.ok[c] = xoff + (size_t)(3 * c + 0) * (K + 1);
        o.om[c] = xoff + (size_t)(3 * c + 1) * (K + 1);
        o.ot[c] = xoff + (size_t)(3 * c + 2) * (K + 1);
    }
    uint32_t* bnd = nullptr;
    CK(dalloc(h, S_XBND, &bnd, (size_t)(MAX_STORES + 1) * NVX_MAX * 3));
    std::vector<uint32_t> hb((size_t)(W + 1) * nvc * 3, 0);
    if (K) {
        NV_DISPATCH((int)h->cfg.replicas, launch_export_offsets_nv, h, K, list, o);
        k_export_bounds<<<1, 256, 0, st>>>((int)W, nvc, xtot, o, bnd);
        HIPCHK(h, hipMemcpyAsync(hb.data(), bnd, hb.size() * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    // 3. per-destination layout, headers, fill
    std::vector<uint64_t> sec((size_t)MAX_STORES * SEC_PER_DEST, 0);
    h->send_sizes.assign(W, 0);
    const size_t hdr_words = 3 + 3 * (size_t)nvc;
    h->send_hdr.assign((size_t)W * hdr_words, 0);
    size_t total = 0;
    std::vector<size_t> base(W, 0);
    for (uint32_t d = 0; d < W; ++d) {
        std::vector<uint32_t> cnt((size_t)3 * nvc, 0);
        for (int c = 0; c < nvc; ++c)
            for (int k = 0; k < 3; ++k) cnt[3 * c + k] = hb[((size_t)(d + 1) * nvc + c) * 3 + k] - hb[((size_t)d * nvc + c) * 3 + k];
        const size_t sz = blob_layout(tot[d], nvc, nv, cnt.data(), sec.data() + (size_t)d * SEC_PER_DEST);
        for (int k = 0; k < SEC_PER_DEST; ++k) sec[(size_t)d * SEC_PER_DEST + k] += total;
        uint64_t* hd = h->send_hdr.data() + (size_t)d * hdr_words;
        hd[0] = 0xAD5EC0DFull; hd[1] = tot[d]; hd[2] = (uint64_t)nvc | ((uint64_t)(nvc - 2 * nv) << 16);
        for (int c = 0; c < 3 * nvc; ++c) hd[3 + c] = cnt[c];
        base[d] = total;
        h->send_sizes[d] = sz;
        bytes[d] = sz;
        total += sz;
    }
    CK(dalloc(h, S_SEND, &h->send, std::max<size_t>(total, 8)));
    uint64_t* dsec = nullptr;
    CK(dalloc(h, S_XSEC, &dsec, sec.size()));
    HIPCHK(h, hipMemsetAsync(h->send, 0, total, st));
    HIPCHK(h, hipMemcpyAsync(dsec, sec.data(), sec.size() * 8, hipMemcpyHostToDevice, st));
    for (uint32_t d = 0; d < W; ++d)
        HIPCHK(h, hipMemcpyAsync(h->send + base[d], h->send_hdr.data() + (size_t)d * hdr_words, hdr_words * 8, hipMemcpyHostToDevice, st));
    if (K) {
        ExportFillArgs fa{};
        fa.K = K; fa.nvc = nvc; fa.list = list; fa.dest = h->hstore; fa.totals = xtot; fa.gid = h->gid; fa.bnd = bnd;
        fa.sec = dsec; fa.send = h->send; fa.o = o;
        for (int c = 0; c < nvc; ++c) {
            const Csr& x = export_csr(h, c);
            fa.key_off[c] = x.key_off; fa.keys[c] = x.keys; fa.k2t_off[c] = x.k2t_off; fa.k2t[c] = x.k2t;
            fa.ent_off[c] = x.ent_off; fa.tcnt[c] = x.tcnt; fa.txns[c] = x.txns;
            fa.kw[c] = c >= 2 * nv ? 2 : 1;
        }
        k_export_fill<<<ceil_div((long)K, 256), 256, 0, st>>>(fa);
    }
    HIPCHK(h, hipStreamSynchronize(st));   // host header / section buffers
    h->send_bytes = total;
    return AD_OK;
}

int ad_shard_send_to_host(ad_handle* h, void* dst) {
    if (!h || !dst || !h->send) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (h->send_bytes) HIPCHK(h, hipMemcpyAsync(dst, h->send, h->send_bytes, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

// Views into the received per-source blobs (concatenated in source order, sizes[s] bytes each).
static int parse_recv(ad_handle* h, const uint64_t* sizes) {
    const int nv = (int)h->cfg.replicas, nvc2 = 2 * nv, nvc3 = 3 * nv;
    const uint32_t W = h->world;
    std::vector<size_t> off(W, 0);
    for (uint32_t s = 1; s < W; ++s) off[s] = off[s - 1] + sizes[s - 1];
    // the header's first three words (magic, rows, nvc), then the per-vc counts of its nvc classes
    const size_t hdr_max = 3 + 3 * (size_t)nvc3;
    std::vector<uint64_t> hdr(hdr_max * W, 0);
    for (uint32_t s = 0; s < W; ++s) {
        if (sizes[s] < (3 + 3 * (size_t)nvc2) * 8) return set_err(h, AD_ERR_ARGUMENT, "shard blob " + std::to_string(s) + ": truncated");
        HIPCHK(h, hipMemcpyAsync(hdr.data() + s * hdr_max, h->recv + off[s], std::min<size_t>(hdr_max * 8, sizes[s]),
                                 hipMemcpyDeviceToHost, h->st));
    }
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->src_csr.assign((size_t)W * nvc3, Csr{});
    h->src_gid.assign(W, nullptr);
    h->src_n.assign(W, 0);
    h->src_ranges.assign(W, 0);
    for (uint32_t s = 0; s < W; ++s) {
        const uint64_t* hd = hdr.data() + s * hdr_max;
        const int nvc = (int)(hd[2] & 0xFFFF);
        if (hd[0] != 0xAD5EC0DFull || (hd[2] != (uint64_t)nvc2 && hd[2] != ((uint64_t)nvc3 | ((uint64_t)nv << 16))))
            return set_err(h, AD_ERR_ARGUMENT, "shard blob " + std::to_string(s) + ": bad header (replicas must match)");
        if (sizes[s] < (3 + 3 * (size_t)nvc) * 8) return set_err(h, AD_ERR_ARGUMENT, "shard blob " + std::to_string(s) + ": truncated");
        h->src_ranges[s] = nvc == nvc3 ? 1 : 0;
        const size_t rows = hd[1];
        std::vector<uint32_t> cnt((size_t)3 * nvc);
        for (int c = 0; c < 3 * nvc; ++c) cnt[c] = (uint32_t)hd[3 + c];
        std::vector<uint64_t> sec(SEC_PER_DEST, 0);
        if (blob_layout(rows, nvc, nv, cnt.data(), sec.data()) > sizes[s])
            return set_err(h, AD_ERR_ARGUMENT, "shard blob " + std::to_string(s) + " exceeds its size");
        uint8_t* b = h->recv + off[s];
        h->src_gid[s] = (uint32_t*)(b + sec[0]);
        h->src_n[s] = (uint32_t)rows;
        for (int c = 0; c < nvc; ++c) {
            Csr& x = h->src_csr[(size_t)s * nvc3 + c];
            x.nkeys = cnt[3 * c]; x.nk2t = cnt[3 * c + 1]; x.ncap = cnt[3 * c + 2];
            x.key_off = (uint32_t*)(b + sec[1 + 7 * c]); x.k2t_off = (uint32_t*)(b + sec[2 + 7 * c]);
            x.ent_off = (uint32_t*)(b + sec[3 + 7 * c]); x.tcnt = (uint32_t*)(b + sec[4 + 7 * c]);
            x.keys = (uint64_t*)(b + sec[5 + 7 * c]); x.k2t = (int32_t*)(b + sec[6 + 7 * c]); x.txns = (uint32_t*)(b + sec[7 + 7 * c]);
        }
    }
    return AD_OK;
}

int ad_shard_import_host(ad_handle* h, const void* src, uint32_t world, const uint64_t* sizes /* [world] */) {
    if (!h || !src || !sizes || world != h->world) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    size_t total = 0;
    for (uint32_t s = 0; s < world; ++s) total += sizes[s];
    CK(dalloc(h, S_RECV, &h->recv, std::max<size_t>(total, 8)));
    if (total) HIPCHK(h, hipMemcpyAsync(h->recv, src, total, hipMemcpyHostToDevice, h->st));
    return parse_recv(h, sizes);
}

int ad_comm_unique_id(uint8_t* out /* [128] */) {
    if (!out) return AD_ERR_ARGUMENT;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return AD_ERR_DEVICE;
    std::memcpy(out, &id, sizeof(id) < 128 ? sizeof(id) : 128);
    return AD_OK;
}

int ad_comm_init(ad_handle* h, uint32_t world, uint32_t rank, const uint8_t* id_bytes) {
    if (!h || !id_bytes || rank >= world) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (h->comm) return set_err(h, AD_ERR_STATE, "ad_comm_init: the handle already has a communicator");
    if (h->sharded && world != h->world) return set_err(h, AD_ERR_ARGUMENT, "ad_comm_init: world differs from ad_shard_setup's");
    ncclUniqueId id;
    std::memcpy(&id, id_bytes, sizeof(id));
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclCommInitRank(&comm, (int)world, id, (int)rank);
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    h->comm = comm;
    return AD_OK;
}

// Tears the handle's communicator down (ncclCommAbort: the peers may have failed their init, so no collective
// teardown); the handle can then take another ad_comm_init or stay on a host transport.
int ad_comm_destroy(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (h->comm) {
        hipStreamSynchronize(h->st);
        ncclCommAbort(h->comm);
        h->comm = nullptr;
    }
    return AD_OK;
}

// RCCL all-to-all of the per-destination blobs over xGMI (grouped point-to-point send/recv; the recv
// sizes come from the peers' export sizes, exchanged by the caller).
int ad_shard_alltoall(ad_handle* h, const uint64_t* recv_sizes /* [world] */) {
    if (!h || !recv_sizes) return AD_ERR_ARGUMENT;
    if (!h->comm || !h->send) return set_err(h, AD_ERR_STATE, "ad_shard_alltoall: ad_comm_init + ad_shard_export first");
    hipSetDevice(h->device);
    const uint32_t W = h->world;
    size_t total = 0;
    for (uint32_t s = 0; s < W; ++s) total += recv_sizes[s];
    CK(dalloc(h, S_RECV, &h->recv, std::max<size_t>(total, 8)));
    if (h->send_sizes.size() != W) return set_err(h, AD_ERR_STATE, "ad_shard_alltoall: export for this world first");
    size_t so = 0, ro = 0;
    if (ncclGroupStart() != ncclSuccess) return set_err(h, AD_ERR_DEVICE, "ncclGroupStart");
    // every send/recv is checked; on an argument error the group is still closed before returning
    ncclResult_t first = ncclSuccess;
    std::string what;
    for (uint32_t p = 0; p < W && first == ncclSuccess; ++p) {
        if (h->send_sizes[p]) {
            ncclResult_t r = ncclSend(h->send + so, h->send_sizes[p], ncclUint8, (int)p, h->comm, h->st);
            if (r != ncclSuccess) { first = r; what = "ncclSend to " + std::to_string(p); }
        }
        if (first == ncclSuccess && recv_sizes[p]) {
            ncclResult_t r = ncclRecv(h->recv + ro, recv_sizes[p], ncclUint8, (int)p, h->comm, h->st);
            if (r != ncclSuccess) { first = r; what = "ncclRecv from " + std::to_string(p); }
        }
        so += h->send_sizes[p];
        ro += recv_sizes[p];
    }
    ncclResult_t r = ncclGroupEnd();
    if (first != ncclSuccess) return set_err(h, AD_ERR_DEVICE, what + ": " + ncclGetErrorString(first));
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclGroupEnd (send/recv): ") + ncclGetErrorString(r));
    return parse_recv(h, recv_sizes);
}

// Home txns: merge every store's fragment per view (k_merge over sources with row indirection), then
// Deps.merge across the replica views.  sizes[view * 3 + cls] (view == replicas: merged).
int ad_shard_merge(ad_handle* h, ad_csr_sizes* sizes, size_t* n_home) {
    if (h) h->merge_heavy = true;      // fragments from every store: any shape
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (h->src_csr.empty()) return set_err(h, AD_ERR_STATE, "ad_shard_merge: exchange the blobs first");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const size_t n = h->n;
    const int nv = (int)h->cfg.replicas, nvc = 2 * nv;
    if (h->world > (uint32_t)MAXV) return set_err(h, AD_ERR_UNSUPPORTED, "more than 8 shards");
    if (h->src_csr.size() != (size_t)h->world * 3 * nv) return set_err(h, AD_ERR_STATE, "ad_shard_merge: exchange the blobs first");
    bool ranges = false;
    for (uint32_t s = 0; s < h->world; ++s) ranges |= h->src_ranges[s] != 0;
    // home rows + global ids
    CK(dalloc(h, S_HROWS, &h->home_rows, n + 1));
    uint32_t* tot = nullptr;
    CK(dalloc(h, S_NK, &tot, 16));
    if (n) device_scan(CompactFlagOp{h->home, h->home_rows, tot, n}, n, (uint32_t*)h->scratch, st);
    else HIPCHK(h, hipMemsetAsync(tot, 0, 4, st));
    uint32_t Hh = 0;
    HIPCHK(h, hipMemcpyAsync(&Hh, tot, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    const size_t H = Hh;
    h->H = H;
    CK(dalloc(h, S_HGID, &h->home_gid, H));
    CK(dalloc(h, S_SROWS, &h->src_rows, H * h->world));
    if (ranges) {
        CK(dalloc(h, S_NONEROWS, &h->none_rows, std::max<size_t>(H, 1)));
        if (H) HIPCHK(h, hipMemsetAsync(h->none_rows, 0xFF, H * 4, st));
    }
    if (H) {
        k_home_gid<<<ceil_div((long)H, 256), 256, 0, st>>>(H, h->home_rows, h->gid, h->home_gid);
        for (uint32_t s = 0; s < h->world; ++s)
            k_source_rows<<<ceil_div((long)H, 256), 256, 0, st>>>(H, h->home_gid, h->src_gid[s], h->src_n[s], h->src_rows + s * H);
    }
    // per (view, class): union over sources (PartialDeps.with); RangeDeps from the sources that carry them
    // (a source without range classes holds no range dependency: its rows are all absent)
    h->sdeps.resize(nvc);
    for (int pass = 0; pass < (ranges ? 2 : 1); ++pass) {
        const int nx = pass == 0 ? nvc : nv, v0 = pass == 0 ? 0 : nvc;
        std::vector<Csr*> out(nx);
        std::vector<size_t> blocks(nx);
        std::vector<int> kw(nx, pass == 0 ? 1 : 2);
        std::vector<std::array<const Csr*, MAXV>> in(nx);
        std::vector<std::array<const int32_t*, MAXV>> rows(nx);
        for (int k = 0; k < nx; ++k) {
            const int vc = v0 + k;
            out[k] = pass == 0 ? &h->sdeps[vc] : &h->srdeps[k];
            blocks[k] = pass == 0 ? CSR_SHARD0 + vc : CSR_SRANGE0 + k;
            for (uint32_t s = 0; s < h->world; ++s) {
                in[k][s] = &h->src_csr[(size_t)s * 3 * nv + vc];
                rows[k][s] = (pass == 0 || h->src_ranges[s]) ? h->src_rows + s * H : h->none_rows;
            }
        }
        CK(merge_multi(h, H, nx, out.data(), blocks.data(), kw.data(),
                       reinterpret_cast<const Csr* const (*)[MAXV]>(in.data()),
                       reinterpret_cast<const int32_t* const (*)[MAXV]>(rows.data()), (int)h->world, nullptr));
    }
    // Deps.merge across views (key, direct, and range when any store held range txns)
    const int mc = ranges ? 3 : 2;
    Csr* mout[3] = {&h->smerged[0], &h->smerged[1], &h->smerged[2]};
    size_t mblocks[3] = {CSR_SMERGED0, CSR_SMERGED0 + 1, CSR_SMERGED0 + 2};
    int mkw[3] = {1, 1, 2};
    const Csr* min_[3][MAXV] = {};
    for (int v = 0; v < nv; ++v) { min_[0][v] = &h->sdeps[2 * v]; min_[1][v] = &h->sdeps[2 * v + 1]; min_[2][v] = &h->srdeps[v]; }
    uint64_t ent = 0;
    CK(merge_multi(h, H, mc, mout, mblocks, mkw, min_, nullptr, nv, &ent));
    h->shard_ranges = ranges;
    h->merged_entries = ent;
    h->times.merged_entries = ent;
    if (n_home) *n_home = H;
    if (sizes) {
        // merge outputs carry exact unique-TxnId offsets (MultiOffsetsOp), so ncap is the TxnId total
        for (int v = 0; v <= nv; ++v) {
            for (int c = 0; c < 2; ++c) {
                const Csr& x = v < nv ? h->sdeps[2 * v + c] : h->smerged[c];
                sizes[v * 3 + c] = ad_csr_sizes{H, x.nkeys, x.nk2t, x.ncap, x.ncap};
            }
            if (ranges) {
                const Csr& x = v < nv ? h->srdeps[v] : h->smerged[2];
                sizes[v * 3 + 2] = ad_csr_sizes{H, x.nkeys, x.nk2t, x.ncap, x.ncap};
            } else {
                sizes[v * 3 + 2] = ad_csr_sizes{H, 0, 0, 0, 0};
            }
        }
    }
    return AD_OK;
}

int ad_shard_fetch(ad_handle* h, uint32_t view, uint32_t cls, ad_csr_out* out, uint32_t* home_gid) {
    if (!h || !out || cls >= AD_NUM_CLASSES || view > h->cfg.replicas) return AD_ERR_ARGUMENT;
    if (h->sdeps.empty()) return set_err(h, AD_ERR_STATE, "ad_shard_fetch: ad_shard_merge first");
    hipSetDevice(h->device);
    const size_t n_saved = h->n;
    h->n = h->H;                          // fetch_csr / fetch_empty work over the home txns
    int rc;
    if (cls == AD_CLASS_RANGE && !h->shard_ranges) rc = fetch_empty(h, out);
    else if (cls == AD_CLASS_RANGE) rc = fetch_csr(h, view < h->cfg.replicas ? h->srdeps[view] : h->smerged[2], 2, out);
    else rc = fetch_csr(h, view < h->cfg.replicas ? h->sdeps[2 * view + cls] : h->smerged[cls], 1, out);
    h->n = n_saved;
    if (rc == AD_OK && home_gid && h->H) {
        HIPCHK(h, hipMemcpyAsync(home_gid, h->home_gid, h->H * 4, hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
    }
    return rc;
}

// One round of the distributed level fixpoint: local chains from the replicated global levels, then
// this store's levels back into the global array.  *changed: this store raised some global level.
int ad_shard_levels_round(ad_handle* h, int first, uint32_t* changed) {
    if (!h || !changed) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->sharded || !h->have_deps) return set_err(h, AD_ERR_STATE, "ad_shard_levels_round: sharded deps first");
    hipSetDevice(h->device);
    CK(complete_entries(h));
    hipStream_t st = h->st;
    const size_t n = h->n;
    // Unmanaged txns (range txns, key-domain sync points / ephemeral reads) and the key txns depending on range
    // txns also wait on their merged deps: rules (b) and (c).  Every such constraint is local to one store — a
    // dependency edge T -> D comes from a key or range slice both hold, a (c) bound from one key's chain — so
    // each store applies the ones it holds from the Deps.merge of its own replica views (the global merged
    // deps restricted to its keys), computed once per batch.
    const bool mixed = h->Q > 0 || h->n_special > 0 || h->n_large > 0;
    if (first && mixed) CK(stage_merge(h));
    h->ks_levels = false;
    CK(dalloc(h, S_G, &h->G, h->n_global + 1));
    uint32_t* flag = nullptr;
    CK(dalloc(h, S_NE, &flag, 16));
    if (first) HIPCHK(h, hipMemsetAsync(h->G, 0, (h->n_global + 1) * 4, st));
    else if (n) k_levels_gather<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->gid, h->G, h->lvl);
    LevelInputs li{};
    li.n = n; li.P = h->P; li.e_txn = h->e_txn; li.e_meta = h->e_meta; li.e_exec1 = h->e_exec1;
    li.seg_start = h->seg_start; li.sval = h->sval; li.nh = h->nh_valid ? h->nh : nullptr;
    if (!h->nh_valid && h->sf_ntiles) {               // k_seg_fuse's per-tile second-entry lists
        li.sec = (const uint32_t*)h->bufs[S_SFSEC].p; li.sec_cap = SF_SEC; li.sec_tiles = (uint32_t)h->sf_ntiles;
        li.sec_cnt = li.sec + h->sf_ntiles * (size_t)SF_SEC;
    } li.prm = h->prm; li.key_off = h->key_off; li.meta = h->meta; li.ex1 = h->ex1;
    li.lvl = h->lvl; li.order = h->order;
    li.ukey = h->ukey; li.useg = h->useg; li.U = h->P ? h->hprm.n_keys_u : 0;
    if (mixed) {
        if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_shard_levels_round: first round missing");
        CK(merged_ready(h));
        li.merged_key = &h->merged[AD_CLASS_KEY];
        li.merged_direct = &h->merged[AD_CLASS_DIRECT_KEY];
        li.merged_range = &h->merged[AD_CLASS_RANGE];
    }
    li.n_large = mixed ? h->n_large : 0;
    li.n_special = mixed ? h->n_special : 0;
    li.exec_bits = h->pack.total_bits;
    li.keep_levels = first ? 0 : 1;
    int iters = 0;
    CK(levels_run(h, li, false, &iters));
    if (first) h->ls.chains_ready = true;
    HIPCHK(h, hipMemsetAsync(flag, 0, 4, st));
    if (h->holders) {
        const uint32_t W = h->world;
        HIPCHK(h, hipMemsetAsync(h->dcnt_dev, 0, W * 4, st));
        const uint32_t others = ((1u << W) - 1u) & ~(1u << h->self);
        if (n) k_level_deltas<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->gid, h->holders, others, h->G, h->lvl,
                                                                     h->dbase_dev, h->dcnt_dev, h->dout, flag);
        HIPCHK(h, hipMemcpyAsync(h->dcnt.data(), h->dcnt_dev, W * 4, hipMemcpyDeviceToHost, st));
    } else {
        if (n) k_levels_scatter<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->gid, h->G, h->lvl, flag);
        // the flag also rides in G[n_global], so the RCCL all-reduce(max) returns "any store changed"
        HIPCHK(h, hipMemcpyAsync(h->G + h->n_global, flag, 4, hipMemcpyDeviceToDevice, st));
    }
    HIPCHK(h, hipMemcpyAsync(changed, flag, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    h->level_iters += (uint32_t)iters;
    return AD_OK;
}

int ad_shard_set_holders(ad_handle* h, const uint8_t* holders) {
    if (!h || (!holders && h->n)) return AD_ERR_ARGUMENT;
    if (!h->sharded) return set_err(h, AD_ERR_STATE, "ad_shard_set_holders: ad_shard_setup first");
    hipSetDevice(h->device);
    const size_t n = h->n;
    const uint32_t W = h->world, self_bit = 1u << h->self, all = (1u << W) - 1u;
    std::vector<uint64_t> cap(W, 0);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t m = holders[i];
        if (!(m & self_bit) || (m & ~all)) return set_err(h, AD_ERR_ARGUMENT, "holders: every mask holds this store and only stores < world");
        for (uint32_t d = 0; d < W; ++d) cap[d] += (d != h->self) && ((m >> d) & 1u);
    }
    h->dbase.assign(W + 1, 0);
    for (uint32_t d = 0; d < W; ++d) {
        if (h->dbase[d] + cap[d] > 0xFFFFFFFFull) return set_err(h, AD_ERR_UNSUPPORTED, "holders: more than 2^32 shared rows");
        h->dbase[d + 1] = h->dbase[d] + (uint32_t)cap[d];
    }
    CK(dalloc(h, S_HOLD, &h->holders, std::max<size_t>(n, 1)));
    CK(dalloc(h, S_DBASE, &h->dbase_dev, MAX_STORES + 1));
    CK(dalloc(h, S_DCNT, &h->dcnt_dev, MAX_STORES));
    CK(dalloc(h, S_DOUT, &h->dout, std::max<size_t>(h->dbase[W], 1)));
    if (n) HIPCHK(h, hipMemcpyAsync(h->holders, holders, n, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, hipMemcpyAsync(h->dbase_dev, h->dbase.data(), (W + 1) * 4, hipMemcpyHostToDevice, h->st));
    h->holders_host.assign(holders, holders + n);
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->dcnt.assign(W, 0);
    return AD_OK;
}

int ad_shard_levels_deltas(ad_handle* h, uint32_t* counts, uint64_t* pairs) {
    if (!h || !counts) return AD_ERR_ARGUMENT;
    if (!h->holders) return set_err(h, AD_ERR_STATE, "ad_shard_levels_deltas: ad_shard_set_holders + a round first");
    hipSetDevice(h->device);
    size_t at = 0;
    for (uint32_t d = 0; d < h->world; ++d) {
        counts[d] = h->dcnt[d];
        if (pairs && h->dcnt[d])
            HIPCHK(h, hipMemcpyAsync(pairs + at, h->dout + h->dbase[d], (size_t)h->dcnt[d] * 8, hipMemcpyDeviceToHost, h->st));
        at += h->dcnt[d];
    }
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

static int apply_level_pairs(ad_handle* h, const uint64_t* dev_pairs, size_t m) {
    if (m) k_level_apply<<<ceil_div((long)m, 256), 256, 0, h->st>>>(m, dev_pairs, h->G);
    HIPCHK(h, hipGetLastError());
    return AD_OK;
}

int ad_shard_levels_apply(ad_handle* h, const uint64_t* pairs, size_t m) {
    if (!h || (m && !pairs)) return AD_ERR_ARGUMENT;
    if (!h->G) return set_err(h, AD_ERR_STATE, "ad_shard_levels_apply: a level round first");
    hipSetDevice(h->device);
    for (size_t i = 0; i < m; ++i)
        if ((pairs[i] >> 32) >= h->n_global) return set_err(h, AD_ERR_ARGUMENT, "ad_shard_levels_apply: global rank out of range");
    uint64_t* buf = nullptr;
    CK(dalloc(h, S_DRECV, &buf, std::max<size_t>(m, 1)));
    if (m) HIPCHK(h, hipMemcpyAsync(buf, pairs, m * 8, hipMemcpyHostToDevice, h->st));
    CK(apply_level_pairs(h, buf, m));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

// RCCL: every store all-gathers the per-destination pair counts (a world x world matrix: row s = what store s
// sends), then the pairs move by grouped point-to-point send/recv and are max-folded into G.
int ad_shard_levels_exchange(ad_handle* h, uint32_t* any_sent) {
    if (!h || !any_sent) return AD_ERR_ARGUMENT;
    if (!h->comm || !h->holders || !h->G) return set_err(h, AD_ERR_STATE, "ad_shard_levels_exchange: ad_comm_init + ad_shard_set_holders + a round first");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const uint32_t W = h->world;
    uint32_t* mat = nullptr;
    CK(dalloc(h, S_DMAT, &mat, (size_t)MAX_STORES * MAX_STORES));
    ncclResult_t r = ncclAllGather(h->dcnt_dev, mat, W, ncclUint32, h->comm, st);
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclAllGather (level counts): ") + ncclGetErrorString(r));
    std::vector<uint32_t> M((size_t)W * W);
    HIPCHK(h, hipMemcpyAsync(M.data(), mat, (size_t)W * W * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    uint64_t total_sent = 0, recv_total = 0;
    for (uint32_t s = 0; s < W; ++s)
        for (uint32_t d = 0; d < W; ++d) total_sent += M[(size_t)s * W + d];
    for (uint32_t s = 0; s < W; ++s) recv_total += M[(size_t)s * W + h->self];
    *any_sent = total_sent ? 1u : 0u;
    if (!total_sent) return AD_OK;
    uint64_t* buf = nullptr;
    CK(dalloc(h, S_DRECV, &buf, std::max<size_t>(recv_total, 1)));
    if (ncclGroupStart() != ncclSuccess) return set_err(h, AD_ERR_DEVICE, "ncclGroupStart");
    ncclResult_t first = ncclSuccess;
    std::string what;
    size_t ro = 0;
    for (uint32_t p = 0; p < W && first == ncclSuccess; ++p) {
        const uint32_t sn = h->dcnt[p], rn = M[(size_t)p * W + h->self];
        if (sn) {
            ncclResult_t e = ncclSend(h->dout + h->dbase[p], (size_t)sn * 8, ncclUint8, (int)p, h->comm, st);
            if (e != ncclSuccess) { first = e; what = "ncclSend (levels) to " + std::to_string(p); }
        }
        if (first == ncclSuccess && rn) {
            ncclResult_t e = ncclRecv(buf + ro, (size_t)rn * 8, ncclUint8, (int)p, h->comm, st);
            if (e != ncclSuccess) { first = e; what = "ncclRecv (levels) from " + std::to_string(p); }
        }
        ro += rn;
    }
    r = ncclGroupEnd();
    if (first != ncclSuccess) return set_err(h, AD_ERR_DEVICE, what + ": " + ncclGetErrorString(first));
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclGroupEnd (levels): ") + ncclGetErrorString(r));
    CK(apply_level_pairs(h, buf, recv_total));
    HIPCHK(h, hipStreamSynchronize(st));
    return AD_OK;
}

int ad_shard_levels_get(ad_handle* h, uint32_t* G) {
    if (!h || !G || !h->G) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    HIPCHK(h, hipMemcpyAsync(G, h->G, h->n_global * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

int ad_shard_levels_set(ad_handle* h, const uint32_t* G) {
    if (!h || !G || !h->G) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    HIPCHK(h, hipMemcpyAsync(h->G, G, h->n_global * 4, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

// RCCL all-reduce(max) of the replicated global level array and, in its last element, of the stores'
// "raised a level this round" flags (*any_changed, if given: no separate host collective per round).
int ad_shard_levels_allreduce(ad_handle* h, uint32_t* any_changed) {
    if (!h || !h->comm || !h->G) return set_err(h, AD_ERR_STATE, "ad_shard_levels_allreduce: ad_comm_init + a round first");
    hipSetDevice(h->device);
    ncclResult_t r = ncclAllReduce(h->G, h->G, h->n_global + 1, ncclUint32, ncclMax, h->comm, h->st);
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
    if (any_changed) {
        HIPCHK(h, hipMemcpyAsync(any_changed, h->G + h->n_global, 4, hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
    }
    return AD_OK;
}

// Home txns' levels and execution order (by (level, executeAt)), as global ranks; on the device.
int ad_shard_order(ad_handle* h, uint32_t* level_out, uint32_t* order_out) {
    if (!h || (!h->G && !h->ks_levels) || h->sdeps.empty())
        return set_err(h, AD_ERR_STATE, "ad_shard_order: levels (rounds, gather or Kahn waves) + ad_shard_merge first");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    hipStream_t st = h->st;
    const size_t H = h->H, n = h->n;
    if (H == 0) return AD_OK;
    // the Kahn waves leave the levels in lvl already; the other protocols in the global array G
    if (n && !h->ks_levels) k_levels_gather<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->gid, h->G, h->lvl);
    uint32_t *ord, *tmp;
    CK(dalloc(h, S_ORDER, &ord, std::max(n, H) + 1));
    // the one-exchange path solves levels without a local level pass: the order's sort buffers are sized here
    if (!ls_reserve_order(h->ls, H, st)) return set_err(h, AD_ERR_NOMEM, "ad_shard_order: out of device memory");
    CK(dalloc(h, S_MSCR, &tmp, 2 * H + 2));
    levels_order_rows(h, H, h->home_rows, ord);
    k_home_gid<<<ceil_div((long)H, 256), 256, 0, st>>>(H, ord, h->home_gid, tmp);           // order -> global ids
    k_home_gid<<<ceil_div((long)H, 256), 256, 0, st>>>(H, h->home_rows, h->lvl, tmp + H);  // home levels
    if (order_out) HIPCHK(h, hipMemcpyAsync(order_out, tmp, H * 4, hipMemcpyDeviceToHost, st));
    if (level_out) HIPCHK(h, hipMemcpyAsync(level_out, tmp + H, H * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    return AD_OK;
}

// Accept / GetDeps on a sharded store: per local row, the number of TxnIds of the GLOBAL batch below the row's
// executeAt (the arrival position the query is answered at; the store holds only its slice, so the caller that
// has the whole batch supplies it).  Valid until the next load.
int ad_shard_query_positions(ad_handle* h, const uint32_t* gq) {
    if (!h || (!gq && h->n)) return AD_ERR_ARGUMENT;
    if (!h->sharded) return set_err(h, AD_ERR_STATE, "ad_shard_query_positions: ad_shard_setup first");
    hipSetDevice(h->device);
    for (size_t i = 0; i < h->n; ++i)
        if (gq[i] > h->n_global) return set_err(h, AD_ERR_ARGUMENT, "ad_shard_query_positions: position beyond the global batch");
    CK(dalloc(h, S_GQPOS, &h->gqpos, std::max<size_t>(h->n, 1)));
    if (h->n) HIPCHK(h, hipMemcpyAsync(h->gqpos, gq, h->n * 4, hipMemcpyHostToDevice, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->gq_ready = true;
    return AD_OK;
}

// ---- one-exchange levels (global_levels.h, levels.hip)
int ad_shard_level_edges(ad_handle* h, size_t* m, uint64_t* out) {
    if (!h || !m) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->sharded || !h->have_deps) return set_err(h, AD_ERR_STATE, "ad_shard_level_edges: sharded deps first");
    hipSetDevice(h->device);
    if (out) {
        if (!h->gl_ready) return set_err(h, AD_ERR_STATE, "ad_shard_level_edges: compute the edges first (out == NULL)");
        if (*m < h->gl_m) return set_err(h, AD_ERR_ARGUMENT, "ad_shard_level_edges: output smaller than the edge count");
        if (h->gl_m) HIPCHK(h, hipMemcpyAsync(out, h->gl_edges, h->gl_m * 8, hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
        *m = h->gl_m;
        return AD_OK;
    }
    // range txns, sync points and ephemeral reads: (b)/(c) constraints from the store's own Deps.merge
    const bool mixed = h->Q > 0 || h->n_special > 0 || h->n_large > 0;
    if (mixed && !h->have_merged) {
        CK(stage_merge(h));
        h->merged_has_range = h->Q > 0;
    }
    return levels_export_edges(h, m, true, false);
}

int ad_shard_levels_solve(ad_handle* h, const uint64_t* edges, size_t m, uint32_t* depth) {
    if (!h || (m && !edges)) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->sharded) return set_err(h, AD_ERR_STATE, "ad_shard_levels_solve: ad_shard_setup first");
    hipSetDevice(h->device);
    uint64_t* buf = nullptr;
    CK(dalloc(h, S_GLIN, &buf, std::max<size_t>(m, 1)));
    if (m) HIPCHK(h, hipMemcpyAsync(buf, edges, m * 8, hipMemcpyHostToDevice, h->st));
    CK(dalloc(h, S_G, &h->G, h->n_global + 1));
    h->ks_levels = false;
    return levels_solve_edges(h, buf, m, h->n_global, h->G, depth);
}

// RCCL: every store's edge count (all-gather), then each store's edges to every peer (grouped send/recv),
// concatenated in store order on every store, and the solve.
int ad_shard_levels_gather(ad_handle* h, uint32_t* depth) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->comm || !h->gl_ready) return set_err(h, AD_ERR_STATE, "ad_shard_levels_gather: ad_comm_init + ad_shard_level_edges first");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const uint32_t W = h->world;
    uint64_t *cnt_dev = nullptr, *all = nullptr;
    CK(dalloc(h, S_DMAT, &cnt_dev, 2 * (size_t)MAX_STORES));
    const uint64_t mine = h->gl_m;
    HIPCHK(h, hipMemcpyAsync(cnt_dev + MAX_STORES, &mine, 8, hipMemcpyHostToDevice, st));
    ncclResult_t r = ncclAllGather(cnt_dev + MAX_STORES, cnt_dev, 1, ncclUint64, h->comm, st);
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclAllGather (edge counts): ") + ncclGetErrorString(r));
    std::vector<uint64_t> cnt(W);
    HIPCHK(h, hipMemcpyAsync(cnt.data(), cnt_dev, W * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    std::vector<uint64_t> off(W + 1, 0);
    for (uint32_t s = 0; s < W; ++s) off[s + 1] = off[s] + cnt[s];
    CK(dalloc(h, S_GLIN, &all, std::max<uint64_t>(off[W], 1)));
    if (mine) HIPCHK(h, hipMemcpyAsync(all + off[h->self], h->gl_edges, mine * 8, hipMemcpyDeviceToDevice, st));
    if (ncclGroupStart() != ncclSuccess) return set_err(h, AD_ERR_DEVICE, "ncclGroupStart");
    ncclResult_t first = ncclSuccess;
    std::string what;
    for (uint32_t p = 0; p < W && first == ncclSuccess; ++p) {
        if (p == h->self) continue;
        if (mine) {
            ncclResult_t e = ncclSend(h->gl_edges, mine * 8, ncclUint8, (int)p, h->comm, st);
            if (e != ncclSuccess) { first = e; what = "ncclSend (level edges) to " + std::to_string(p); }
        }
        if (first == ncclSuccess && cnt[p]) {
            ncclResult_t e = ncclRecv(all + off[p], cnt[p] * 8, ncclUint8, (int)p, h->comm, st);
            if (e != ncclSuccess) { first = e; what = "ncclRecv (level edges) from " + std::to_string(p); }
        }
    }
    r = ncclGroupEnd();
    if (first != ncclSuccess) return set_err(h, AD_ERR_DEVICE, what + ": " + ncclGetErrorString(first));
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclGroupEnd (level edges): ") + ncclGetErrorString(r));
    CK(dalloc(h, S_G, &h->G, h->n_global + 1));
    h->ks_levels = false;
    return levels_solve_edges(h, all, off[W], h->n_global, h->G, depth);
}

int ad_shard_bounds(const uint64_t* keys, size_t nkeys, uint32_t shards, uint64_t* bounds_out) {
    if (!keys || !bounds_out || shards == 0) return AD_ERR_ARGUMENT;
    std::vector<uint64_t> k(keys, keys + nkeys);
    std::sort(k.begin(), k.end());
    k.erase(std::unique(k.begin(), k.end()), k.end());
    bounds_out[0] = 0;
    for (uint32_t s = 1; s < shards; ++s) bounds_out[s] = k.empty() ? 0 : k[std::min(k.size() - 1, k.size() * s / shards)];
    bounds_out[shards] = UINT64_MAX;
    return AD_OK;
}

}  // extern "C"
