// deps.hip — the deps stage: CFK elision scan, walks, per-txn KeyDeps layout and unions, RangeDeps join.
#include "engine_internal.h"

// ---------------------------------------------------------------------------------------------------
// deps
// ---------------------------------------------------------------------------------------------------
// Capacity (elements) of CSR block `block`'s data buffers as currently allocated (0 if none).
size_t csr_cap(ad_handle* h, size_t block, int which, size_t elem) {
    const size_t slot = S_CSR0 + 10 * block + which;
    return slot < h->bufs.size() ? h->bufs[slot].cap / elem : 0;
}

static __global__ void k_ovf_sizes(uint32_t count, const uint2* items, const uint32_t* const* key_off, const uint32_t* const* k2t_off,
                            uint32_t* ne) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint32_t t = items[i].x, c = items[i].y;
    ne[i] = k2t_off[c][t + 1] - k2t_off[c][t] - (key_off[c][t + 1] - key_off[c][t]);
}

// CSRs that overflowed the LDS union: one sync to learn how many; each gets a 1024-thread workgroup with
// 128 KiB of LDS, or a slice of global memory above UNION_CAP_BIG entries.  The CSR blocks are the key
// classes (large txns) and, when the batch has ranges, the RangeDeps views (item.y >= 2R: range view).
int union_overflow(ad_handle* h, LdsUnionArgs la, uint32_t* ovf_count, uint2* ovf, bool has_range) {
    hipStream_t st = h->st;
    uint32_t count = 0;
    HIPCHK(h, hipMemcpyAsync(&count, ovf_count, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (count == 0) return AD_OK;
    count = std::min<uint32_t>(count, 1u << 20);
    (void)has_range;
    const int nv = (int)h->cfg.replicas, nvc = 2 * nv;
    // tables of all CSRs the first pass may have queued: key classes [0, nvc), range views [nvc, nvc+nv)
    LdsUnionArgs b = la;
    std::vector<const uint32_t*> ko(nvc + nv), mo(nvc + nv);
    for (int c = 0; c < nvc + nv; ++c) {
        const Csr& x = c < nvc ? h->deps[c] : h->rdeps[c - nvc];
        ko[c] = x.key_off; mo[c] = x.k2t_off;
        b.key_off[c] = x.key_off; b.k2t_off[c] = x.k2t_off; b.ent_off[c] = x.ent_off; b.k2t[c] = x.k2t;
        b.txns[c] = x.txns; b.tcnt[c] = x.tcnt;
    }
    const uint32_t** dko = nullptr;
    uint32_t* ne = nullptr;
    CK(dalloc(h, S_OVFT, (uint64_t**)&dko, 2 * (nvc + nv)));
    CK(dalloc(h, S_OVFN, &ne, count));
    HIPCHK(h, hipMemcpyAsync(dko, ko.data(), (nvc + nv) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemcpyAsync(dko + nvc + nv, mo.data(), (nvc + nv) * 8, hipMemcpyHostToDevice, st));
    k_ovf_sizes<<<ceil_div((long)count, 256), 256, 0, st>>>(count, ovf, dko, dko + nvc + nv, ne);
    std::vector<uint32_t> hne(count);
    HIPCHK(h, hipMemcpyAsync(hne.data(), ne, count * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    std::vector<uint64_t> goff(count, 0);
    uint64_t gtot = 0;
    for (uint32_t i = 0; i < count; ++i) {
        if (hne[i] > (uint32_t)UNION_CAP_BIG) {
            uint64_t n2 = 1;
            while (n2 < hne[i]) n2 <<= 1;
            goff[i] = gtot;
            gtot += n2;
        }
    }
    uint32_t* gbuf = nullptr;
    uint64_t* dgoff = nullptr;
    CK(dalloc(h, S_OVFG, &gbuf, std::max<uint64_t>(gtot, 1)));
    CK(dalloc(h, S_OVFO, &dgoff, count));
    HIPCHK(h, hipMemcpyAsync(dgoff, goff.data(), count * 8, hipMemcpyHostToDevice, st));
    b.items = ovf; b.gbuf = gbuf; b.gbuf_off = dgoff;
    k_union_big<<<count, UB_BIG, 0, st>>>(b, count);
    HIPCHK(h, hipStreamSynchronize(st));    // host tables
    return AD_OK;
}

// Accept / GetDeps bound: per txn the number of batch TxnIds below its executeAt (TxnIds and executeAts share
// one packed order; tx_ts ascends with the batch).
// An executeAt below its TxnId is no valid Accept / GetDeps bound (executeAt >= TxnId, Timestamp order): flagged
// (ERR_EXECBELOW -> AD_ERR_ARGUMENT) instead of answered from a wrong position.
static __global__ __launch_bounds__(256) void k_query_pos(size_t n, const uint64_t* __restrict__ tx_ts, const uint64_t* __restrict__ ex1,
                                                   uint32_t* __restrict__ qpos, int bound_max, Params* prm) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool bad = false;
    if (i < n) {
        if (bound_max) {
            qpos[i] = (uint32_t)n;                          // Timestamp.MAX: every TxnId is below it
        } else {
            const uint64_t e1 = ex1[i];
            bad = e1 == 0 || e1 - 1 < tx_ts[i];
            const uint64_t e = e1 ? e1 - 1 : 0;
            size_t lo = bad ? 0 : i, hi = n;                 // executeAt >= TxnId: the search starts at i
            while (lo < hi) { const size_t m = (lo + hi) >> 1; if (tx_ts[m] < e) lo = m + 1; else hi = m; }
            qpos[i] = (uint32_t)lo;
        }
    }
    if (__ballot(bad) && __lane_id() == 0) atomicOr(&prm->err, (unsigned)ERR_EXECBELOW);
}

// AD_OVF_MAIN=1: the overflowed rows run on the main stream after the finish (an A/B switch)
static bool ovf_on_main() {
    const char* e = getenv("AD_OVF_MAIN");
    return e && e[0] == '1';
}
int side_fork(ad_handle* h) {
    if (!h->xst) {
        HIPCHK(h, hipStreamCreateWithFlags(&h->xst, hipStreamNonBlocking));
        HIPCHK(h, hipEventCreateWithFlags(&h->xev0, hipEventDisableTiming));
        HIPCHK(h, hipEventCreateWithFlags(&h->xev1, hipEventDisableTiming));
    }
    HIPCHK(h, hipEventRecord(h->xev0, h->st));
    HIPCHK(h, hipStreamWaitEvent(h->xst, h->xev0, 0));
    h->xjoin = true;
    return AD_OK;
}
void side_join(ad_handle* h) {
    if (!h->xjoin) return;
    hipEventRecord(h->xev1, h->xst);
    hipStreamWaitEvent(h->st, h->xev1, 0);
    h->xjoin = false;
}

// Fills in the lone entries the deps stage's gather skipped (k_gather_entries<true>): called before anything
// that reads every sorted entry (execution levels other than the pull pass, MaxConflicts, recovery, CFK retain,
// sharded level passes).
int complete_entries(ad_handle* h) {
    if (h->state_partial) {              // k_seg_fuse wrote no entry state: the gather + ElideOp scan rebuild all of it
        side_join(h);                    // (k_txn_finish_ovf, on the side stream beside the levels, reads the state
                                         // this rewrites)
        h->state_partial = h->keys_partial = h->entries_partial = false;
        const size_t P = h->P;
        if (P) {
            KScope ks(K_GATHER, P);
            k_gather_entries<false><<<ceil_div((long)P, 256), 256, 0, h->st>>>(P, h->sval, h->prec, h->skey, h->e_txn,
                                                                              h->e_meta, h->e_exec1);
            ElideOp eop{h->skey, h->e_meta, h->e_exec1, h->seg_start, h->ud_prev, h->pm_w, h->pm_c,
                        h->nh, h->ukey, h->useg, h->hprm.key_min, P, h->prm,
                        h->key_bits > 32 ? h->keys : nullptr, h->sval};
            scan_any(h, eop, P);
            h->nh_valid = true;
        }
        HIPCHK(h, hipGetLastError());
        return AD_OK;
    }
    if (h->keys_partial) {               // k_seg_fuse's batches: the distinct keys and segment starts, from its tiles
        h->keys_partial = false;
        const size_t nt = h->sf_ntiles;
        KScope ks(K_SEG_KEYS, h->P);
        if (nt) k_seg_tile_scan<<<1, 1024, 0, h->st>>>(nt, h->P, (uint32_t*)h->bufs[S_SFCNT].p, h->useg);
        if (nt) k_seg_ukeys<<<(unsigned)nt, SF_T, 0, h->st>>>(nt, (const uint32_t*)h->bufs[S_SFLO].p,
                                                             (const uint32_t*)h->bufs[S_SFCNT].p, h->skey, h->hprm.key_min,
                                                             h->ukey, h->useg);
        HIPCHK(h, hipGetLastError());
    }
    if (!h->entries_partial) return AD_OK;
    h->entries_partial = false;
    const size_t P = h->P;
    if (P) k_complete_singletons<<<ceil_div((long)P, 256), 256, 0, h->st>>>(P, h->sval, h->prec, h->skey, h->e_txn, h->e_meta,
                                                                          h->e_exec1, h->ud_prev, h->pm_w, h->pm_c);
    HIPCHK(h, hipGetLastError());
    return AD_OK;
}

// The key-class CSRs a deps stage computes: R replies (+ the union view, see stage_deps), keyDeps only or keyDeps
// + directKeyDeps; stage_prepare asks too (k_pack clears that many count bytes per pair).
int deps_class_plan(const ad_handle* h, bool want_union, bool* uni_out) {
    const bool uni = want_union && h->Q == 0 && !h->accept && !h->sharded && !h->hist_active && h->n_large == 0 &&
                     (int)h->cfg.replicas + 1 <= MAXV;
    if (uni_out) *uni_out = uni;
    const int nv = (int)h->cfg.replicas + (uni ? 1 : 0);
    return h->n_special > 0 ? 2 * nv : nv;
}

static int stage_deps_impl(ad_handle* h);
// On an error after the finish's side stream forked, nothing may reuse the buffers k_txn_finish_ovf still reads or
// writes: join it on every error return.
int stage_deps(ad_handle* h) {
    const int rc = stage_deps_impl(h);
    if (rc != AD_OK) side_join(h);
    return rc;
}

static int stage_deps_impl(ad_handle* h) {
    StageScope sc(h, STAGE_DEPS);
    const size_t n = h->n, P = h->P, Q = h->Q;
    // The union view (ad_run_pipeline): Deps.merge of the R replies is the union of their (key, TxnId) relations
    // (RelationMultiMap.LinearMerger folds them with linearUnion per key), and the R views walk the same segments
    // and differ only in the in-flight entries a view dropped.  So the walk emits a view R = "kept by some view"
    // alongside the R replies, and k_txn_finish lays it out as one more class: the merged Deps come out of the deps
    // stage and stage_merge runs no merge kernel.  Key-only PreAccept batches of one store (no range txns, no
    // virtual items: their joins are per real view).
    const bool want_u = h->want_union;
    h->want_union = false;                                // one stage call (the overflow re-run below re-arms it)
    bool uni = false;
    deps_class_plan(h, want_u, &uni);
    h->deps_union = uni;
    const int nv = (int)h->cfg.replicas + (uni ? 1 : 0), nvc = 2 * nv;
    hipStream_t st = h->st;
    // directKeyDeps entries come only from key-domain sync points (CommandsForKey.managesExecution is false
    // for them, Deps.java:80-106); without any in the batch every directKeyDeps CSR is empty, so only the R
    // keyDeps classes are computed (computed class k = CSR cls[k]) and the direct CSRs are zero offsets.
    const bool direct = h->n_special > 0;
    const int nc = direct ? nvc : nv;
    const int nc_real = direct ? 2 * (int)h->cfg.replicas : (int)h->cfg.replicas;   // classes of the R replies
    int cls[NVC_MAX];
    for (int k = 0; k < nc; ++k) cls[k] = direct ? k : 2 * k;
    h->deps_direct = direct;
    h->deps.resize(nvc);
    for (int vc = 0; vc < nvc; ++vc) CK(alloc_csr(h, vc, h->deps[vc], n));
    for (int v = 0; v < nv; ++v) CK(alloc_csr(h, CSR_RANGE0 + v, h->rdeps[v], n));
    for (int k = 0; k < nc; ++k) dirty_csr(h, cls[k]);
    for (int v = 0; v < nv; ++v) dirty_csr(h, CSR_RANGE0 + v);
    // lone entries skipped when nothing of this stage reads them (PreAccept bound: the executeAt-bound walks
    // visit every entry; large / range txns query every key in their ranges)
    const bool skip = P > 0 && !h->accept && h->n_large == 0 && Q == 0 && h->key_bits <= 32;
    // the same batches, unless a key segment outgrew a tile: gather + elision state + count walk in one kernel
    // (seg_fuse_kernels.h); its overflow flag comes back with the totals, and an overflowing batch re-runs here on
    // the three-kernel path
    const bool fuse = skip && !h->seg_long;
    const uint32_t* fuse_hpart = nullptr;
    h->keys_partial = false;
    h->state_partial = false;
    uint32_t* fuse_over = h->totd + MAX_TOTALS - 6;      // (MAX_TOTALS - 5: the merge's speculation guard)
    if (P > 0 && !fuse) {
        h->entries_partial = skip;
        KScope ks(K_GATHER, P);
        if (skip) k_gather_entries<true><<<ceil_div((long)P, 256), 256, 0, st>>>(P, h->sval, h->prec, h->skey, h->e_txn, h->e_meta, h->e_exec1);
        else k_gather_entries<false><<<ceil_div((long)P, 256), 256, 0, st>>>(P, h->sval, h->prec, h->skey, h->e_txn, h->e_meta, h->e_exec1);
    }
    if (P > 0 && !fuse) {
        ElideOp eop{h->skey, h->e_meta, h->e_exec1, h->seg_start, h->ud_prev, h->pm_w, h->pm_c,
                    h->nh, h->ukey, h->useg, h->hprm.key_min, P, h->prm,
                    h->key_bits > 32 ? h->keys : nullptr, h->sval};
        KScope ks(K_SCAN_ELIDE, P);
        scan_any(h, eop, P);
    }
    // ---- executeAt-bound queries: the arrival position of each bound (first TxnId >= executeAt)
    const uint32_t* qpos = nullptr;
    if (h->accept) {
        CK(dalloc(h, S_QPOS, &h->qpos, std::max<size_t>(n, 1)));
        if (n) k_query_pos<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->tx_ts, h->ex1, h->qpos, h->bound_max ? 1 : 0, h->prm);
        qpos = h->qpos;
    }
    // ---- virtual items of large txns
    h->V = 0;
    VItemArgs va{};
    va.n = n; va.meta = h->meta; va.key_off = h->key_off; va.keys = h->keys; va.range_off = h->range_off;
    va.rs = h->range_s; va.re = h->range_e; va.e_txn = h->e_txn;
    va.ukey = h->ukey; va.useg = h->useg; va.prm = h->prm; va.vn = h->vn; va.voff = h->voff; va.qpos = qpos;
    if (h->n_large > 0) {
        KScope ks(K_VITEMS);
        k_vitems<false><<<ceil_div((long)n, 256), 256, 0, st>>>(va);
        scan_offsets(h, h->vn, h->voff, n);
        uint32_t V = 0;
        HIPCHK(h, hipMemcpyAsync(&V, h->voff + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        h->V = V;
        // 12 B + 4 B per (view, class) per item (C4: ~2.5 * 10^9 items): the item's key and segment come from
        // its distinct-key index, the fill slots overwrite the counts in place
        CK(dalloc(h, S_VTXN, &h->vi_txn, V)); CK(dalloc(h, S_VPOS, &h->vi_pos, V)); CK(dalloc(h, S_VSEG, &h->vi_u, V));
        CK(dalloc(h, S_VCNT, &h->vcnt, (size_t)V * nc));
        va.vi_txn = h->vi_txn; va.vi_pos = h->vi_pos; va.vi_u = h->vi_u;
        if (V > 0) k_vitems_fill<<<ceil_div((long)n * WAVE, 256), 256, 0, st>>>(va);
    }
    // ---- walk (count)
    WalkArgs wa{};
    wa.e_txn = h->e_txn; wa.e_meta = h->e_meta; wa.e_exec1 = h->e_exec1; wa.seg_start = h->seg_start;
    wa.ud_prev = h->ud_prev; wa.pm_w = h->pm_w; wa.pm_c = h->pm_c; wa.tx_ts = h->tx_ts; wa.meta = h->meta; wa.P = P;
    wa.window = h->cfg.window; wa.thresh = ad_drop_threshold(h->cfg.drop_p); wa.seed = h->cfg.seed;
    wa.union_last = uni ? 1 : 0;
    wa.gid = (h->sharded || h->hist_active) ? h->gid : nullptr;
    wa.nh = h->nh; wa.prm = h->prm;
    wa.sval = h->sval; wa.cnt8 = h->cnt8; wa.cntx = h->cntx; wa.inl = h->inl; wa.dfr = h->dfr; wa.dst = h->dst;
    wa.key_off = h->key_off;
    CK(dalloc(h, S_POSOF, &wa.posof, std::max<size_t>(P, 1)));
    uint32_t* heavy = h->totd + MAX_TOTALS - 1;          // heavy-merge hint (read with the totals)
    uint32_t* items_count = heavy - 1;                    // the fill walk's items (count walk)
    uint32_t* dtx_count = heavy - 2;                      // deferred small txns (offsets scan)
    uint32_t* fovf_count = h->totd + MAX_TOTALS - 7;      // k_txn_finish's overflowed (txn, class) rows
    uint32_t *items = nullptr, *dtx = nullptr;
    CK(dalloc(h, S_OVI, &items, std::max<size_t>(P, 1)));
    CK(dalloc(h, S_DTX, &dtx, std::max<size_t>(n, 1)));
    wa.items_out = items; wa.items_count = items_count;

    wa.V = h->V; wa.vi_txn = h->vi_txn; wa.vi_pos = h->vi_pos; wa.vi_u = h->vi_u; wa.useg = h->useg;
    wa.vcnt = h->vcnt; wa.vdst = h->vcnt;
    wa.qpos = qpos; wa.ex1 = h->ex1; wa.bound_max = h->bound_max ? 1 : 0;
    wa.gqpos = (h->accept && h->sharded) ? h->gqpos : nullptr;
    // [overflow flag, deferred txns, items, heavy-merge hint]; the pairs' counts (segment heads keep zero);
    // deferred flags
    if (fuse) {
        h->entries_partial = true;
        const size_t ntiles = (P + SF_TILE - 1) / SF_TILE;
        SegFuseArgs f{};
        f.P = P; f.ntiles = ntiles; f.skey = h->skey; f.prec = h->prec; f.overflow = fuse_over;
        CK(dalloc(h, S_SFLO, &f.tile_lo, ntiles + 1)); CK(dalloc(h, S_SFCNT, &f.tile_cnt, 4 * ntiles + 2 * SF_PARTS));
        f.hpart = f.tile_cnt + 4 * ntiles;
        CK(dalloc(h, S_SFSEC, &f.sec, ntiles * (size_t)SF_SEC + ntiles));
        f.sec_cnt = f.sec + ntiles * (size_t)SF_SEC;
        const bool packed = h->cnt8_cleared == ncb_of(nc);   // k_pack cleared the count bytes and deferred flags
        h->cnt8_cleared = 0;
        const bool small = h->small_cleared;                  // ... and the small counters (pack_clear_list)
        h->small_cleared = false;
        if (!(packed && small))
            fill_multi(st, {{fovf_count, 8, 0}, {dtx_count, 12, 0}, {f.hpart, 2 * SF_PARTS * 4, 0},
                            {packed ? nullptr : h->cnt8, (size_t)ncb_of(nc) * P, 0}, {packed ? nullptr : h->dfr, n, 0}});
        f.e_txn = h->e_txn; f.e_meta = h->e_meta; f.e_exec1 = h->e_exec1; f.seg_start = h->seg_start; f.ud_prev = h->ud_prev;
        f.pm_w = h->pm_w; f.pm_c = h->pm_c;
        // the pull pass's chains from the tile's LDS copy (k_pack zeroed succ and the level flags): key Read/Write
        // batches only (no sync points: the pull pass's own condition)
        if (h->chains_pending && !direct && h->n_large == 0 && h->n_special == 0) {
            f.c_txn = h->ls.c_txn; f.c_meta = h->ls.c_meta; f.c_exec1 = h->ls.c_exec1; f.c_pair = h->ls.c_pair;
            f.succ = h->ls.succ; f.any_long = h->ls.flags + 7; f.any_far = h->ls.flags + 18;
            h->chains_prebuilt = true;
        }
        h->chains_pending = false;
        { KScope ks(K_SEG_FUSE, P); launch_seg_fuse_nv(nv, f, wa, direct, st); }
        fuse_hpart = f.hpart;              // n_keys_u: summed by the deps publish (PubExtra)
        h->nh_valid = false;               // no dense non-head list: the level chain build runs over every position
        h->keys_partial = true;            // ukey / useg on demand (complete_entries)
        h->state_partial = true;           // the entry state too (k_seg_fuse writes it for re-walked segments only)
        h->sf_ntiles = ntiles;
    } else {
        h->chains_pending = false;
        h->chains_prebuilt = false;
        h->nh_valid = true;
        const bool packed = h->cnt8_cleared == ncb_of(nc);
        h->cnt8_cleared = 0;
        h->small_cleared = false;
        fill_multi(st, {{fovf_count, 4, 0}, {dtx_count, 12, 0}, {packed ? nullptr : h->cnt8, (size_t)ncb_of(nc) * P, 0},
                        {packed ? nullptr : h->dfr, n, 0}});
        launch_walk_nv(nv, wa, false, direct, true, st);
    }
    TxnArgs ta{};
    static unsigned long long* ovf_dbg = nullptr;             // AD_OVF_TIMERS=1 (diagnostics): printed per batch
    {
        const char* e = getenv("AD_OVF_TIMERS");
        if (e && e[0] == '1') {
            if (!ovf_dbg) hipMalloc(&ovf_dbg, 64);
            hipMemsetAsync(ovf_dbg, 0, 64, st);
            ta.dbg = ovf_dbg;
        }
    }
    ta.n = n; ta.P = P; ta.nvc = nc; ta.key_off = h->key_off; ta.keys = h->keys; ta.meta = h->meta; ta.cnt8 = h->cnt8; ta.cntx = h->cntx;
    ta.nk = h->nk; ta.ne = h->ne; ta.dst = h->dst; ta.prm = h->prm;
    ta.voff = h->voff; ta.vcnt = h->vcnt; ta.vdst = h->vcnt; ta.vi_u = h->vi_u; ta.ukey = h->ukey;
    CK(dalloc(h, S_FOVF, &ta.ovf_rows, std::max<size_t>(n, 1)));
    CK(dalloc(h, S_FOVFCM, &ta.ovf_cm, std::max<size_t>(n, 1)));
    ta.ovf_count = fovf_count;
    // every large txn's per-CSR totals, also when no range meets a CFK key (V = 0: a batch of range txns only); the
    // offsets scan reads them for every large txn
    if (n > 0 && h->n_large > 0) {
        KScope ks(K_VITEMS);
        launch_large_sums_nv(nv, ta, direct, st);
    }
    if (n > 0) {
        KScope ks(K_SCAN_OFFSETS, n);
        launch_offsets_nv(h, nv, direct, cls, heavy, dtx, dtx_count, ta.ovf_rows, ta.ovf_cm, fovf_count);
    } else {
        for (int k = 0; k < nc; ++k) csr_offsets(h, h->deps[cls[k]], h->nk, h->ne);
    }
    if (!direct)
        for (int v = 0; v < nv; ++v) CK(zero_csr(h, 2 * v + 1, h->deps[2 * v + 1], n));
    // ---- RangeDeps (count)
    RangeArgs ra{};
    ra.n = n; ra.Q = Q; ra.key_off = h->key_off; ra.keys = h->keys; ra.range_off = h->range_off; ra.rs = h->range_s;
    ra.re = h->range_e; ra.meta = h->meta; ra.es = h->es; ra.ee = h->ee; ra.eown = h->eown; ra.ix = h->ix; ra.prm = h->prm;
    ra.window = h->cfg.window; ra.thresh = wa.thresh; ra.seed = h->cfg.seed; ra.rnk = h->rnk; ra.rne = h->rne;
    ra.qpos = qpos;
    ra.gqpos = wa.gqpos;
    ra.gid = wa.gid;
    if (Q > 0 && n > 0) {
        launch_range_nv(nv, ra, false, st);
        for (int v = 0; v < nv; ++v) csr_offsets(h, h->rdeps[v], h->rnk + (size_t)v * n, h->rne + (size_t)v * n);
    }
    // ---- sizes -> host (one sync), allocate outputs
    const int ncsr = nc + nv;
    std::vector<uint32_t> tot(3 * ncsr, 0);
    auto csr_at = [&](int c) -> Csr& { return c < nc ? h->deps[cls[c]] : h->rdeps[c - nc]; };
    TotTable tt{};
    for (int c = 0; c < (Q > 0 ? ncsr : nc); ++c) {
        Csr& x = csr_at(c);
        tt.src[3 * c + 0] = x.key_off + n; tt.src[3 * c + 1] = x.k2t_off + n; tt.src[3 * c + 2] = x.ent_off + n;
        tt.count = 3 * c + 3;
    }
    const int ncol = tt.count;
    tt.src[tt.count++] = heavy;
    tt.src[tt.count++] = items_count;
    tt.src[tt.count++] = dtx_count;
    const int col_over = tt.count;
    tt.src[tt.count++] = fuse_over;
    // Speculative finish (small key batches whose key-class buffers from an earlier batch exist): k_txn_finish is
    // enqueued BEFORE the host reads the totals, into those buffers, behind k_cap_check's guard (a CSR total beyond
    // its buffer's capacity makes every thread exit).  The host reads the totals while the finish runs and re-runs
    // it after sizing only if the guard fired: no host round trip between the offsets scan and the finish.
    uint32_t* spec_bad = heavy - 3;
    bool spec = n > 0 && h->V == 0 && Q == 0;
    CapCheck capc{};
    for (int k = 0; k < nc && spec; ++k) {
        const int c = cls[k];
        const size_t base = S_CSR0 + 10 * (size_t)c;
        const size_t ck = csr_cap(h, c, 4, 8), cm = csr_cap(h, c, 5, 4), ct = csr_cap(h, c, 6, 4);
        if (!ck || !cm || !ct) { spec = false; break; }
        Csr& x = h->deps[c];
        const uint32_t* tots[3] = {x.key_off + n, x.k2t_off + n, x.ent_off + n};
        const size_t caps[3] = {ck, cm, ct};
        for (int q = 0; q < 3; ++q) { capc.tot[capc.m] = tots[q]; capc.cap[capc.m++] = (uint32_t)std::min<size_t>(caps[q], 0xFFFFFFFFu); }
        ta.out_key_off[k] = x.key_off; ta.out_k2t_off[k] = x.k2t_off; ta.out_ent_off[k] = x.ent_off; ta.out_tcnt[k] = x.tcnt;
        ta.out_keys[k] = (uint64_t*)h->bufs[base + 4].p; ta.out_k2t[k] = (int32_t*)h->bufs[base + 5].p;
        ta.out_txns[k] = (uint32_t*)h->bufs[base + 6].p;
    }
    ta.inl = h->inl; ta.dfr = h->dfr; ta.nrows = n;
    // the publish also evaluates the speculative finish's capacity guard (k_cap_check's rule) and sums the fused
    // kernel's head counts into n_keys_u (k_seg_heads): one launch
    PubExtra pex{};
    if (spec) {
        capc.bad = spec_bad;
        pex.cap = capc;
        tt.src[tt.count++] = spec_bad;
    }
    pex.hpart = fuse_hpart; pex.nparts = SF_PARTS; pex.prm = h->prm;
    std::vector<uint32_t> got(tt.count, 0);
    uint32_t seq = 0;
    host_mark(h, "deps publish");
    CK(publish_totals(h, tt, got.data(), &seq, &pex));  // the read-back first, then the speculative finish
    if (spec) {
        ta.w = wa;
        ta.spec_bad = spec_bad;
        // the overflowed rows (listed by the offsets scan) on the side stream, beside the finish
        const bool ovf_main = ovf_on_main();
        if (!ovf_main) {
            CK(side_fork(h));
            launch_finish_ovf_nv(nv, ta, direct, h->xst);
        }
        {
            KScope ks(K_TXN_LAYOUT, n);
            launch_finish_nv(nv, ta, direct, st);
        }
        if (ovf_main) launch_finish_ovf_nv(nv, ta, direct, st);
        ta.spec_bad = nullptr;
    }
    CK(wait_totals(h, seq, tt.count, got.data()));
    host_mark(h, "deps waited");
    if (fuse && got[col_over] != 0) {
        // a key segment too long for a k_seg_fuse tile: this batch takes the three-kernel path (the speculative
        // finish, if any, exited or is redone there)
        side_join(h);                                    // the speculative finish's side-stream rows
        HIPCHK(h, hipStreamSynchronize(st));
        h->seg_long = true;
        h->want_union = want_u;
        return stage_deps_impl(h);
    }
    std::copy(got.begin(), got.begin() + ncol, tot.begin());
    // k_txn_finish completes every small txn whose pairs kept all their ids inline; only the deferred ones need
    // the fill walk and the union (none on most C2 batches)
    const uint32_t nitems = n > 0 ? got[ncol + 1] : 0, ndtx = n > 0 ? got[ncol + 2] : 0;
    h->times.deferred_txns = ndtx;
    h->times.fill_items = nitems;
    h->merge_heavy = n == 0 || got[ncol] != 0 || h->n_large > 0 || Q > 0;
    CK(check_params(h));
    h->deps_entries = 0;
    h->times.range_entries = 0;
    h->times.vitems = h->V;
    for (int c = 0; c < ncsr; ++c) {
        Csr& x = csr_at(c);
        x.nkeys = tot[3 * c]; x.nk2t = tot[3 * c + 1]; x.ncap = tot[3 * c + 2];
        // the replies' entries (the union view's are the merged Deps': merged_entries)
        if (!(uni && c >= nc_real && c < nc)) h->deps_entries += x.ncap;
        if (c >= nc) h->times.range_entries += x.ncap;
        if (c < nc) {
            CK(alloc_csr_data(h, cls[c], x, 1));
            ta.out_key_off[c] = x.key_off; ta.out_k2t_off[c] = x.k2t_off; ta.out_keys[c] = x.keys; ta.out_k2t[c] = x.k2t;
            ta.out_ent_off[c] = x.ent_off; ta.out_txns[c] = x.txns; ta.out_tcnt[c] = x.tcnt;
            wa.k2t[c] = x.k2t;
        } else {
            CK(alloc_csr_data(h, CSR_RANGE0 + (c - nc), x, 2));
            const int v = c - nc;
            ra.key_off_v[v] = x.key_off; ra.k2t_off_v[v] = x.k2t_off; ra.keys_v[v] = x.keys; ra.k2t_v[v] = x.k2t;
        }
    }
    host_mark(h, "deps alloc");
    // ---- fill
    ta.inl = h->inl; ta.dfr = h->dfr;
    UnionArgs ua{};
    ua.n = n; ua.nvc = nc; ua.meta = h->meta; ua.rows = dtx; ua.nrows = ndtx;
    for (int vc = 0; vc < nc; ++vc) {
        Csr& c = h->deps[cls[vc]];
        ua.key_off[vc] = c.key_off; ua.k2t_off[vc] = c.k2t_off; ua.ent_off[vc] = c.ent_off; ua.k2t[vc] = c.k2t;
        ua.txns[vc] = c.txns; ua.tcnt[vc] = c.tcnt;
    }
    // small txns: k_txn_finish (re-walking in place the pairs that overflowed their inline ids); txns with more
    // than 4 keys (deferred) get their layout there and their lists from the fill walk of their pairs + k_txn_union
    // (unless the speculative launch above already did it)
    const bool spec_ok = spec && got[col_over + 1] == 0;
    h->times.deps_speculative = spec ? (spec_ok ? 1u : 2u) : 0u;
    ta.w = wa;
    if (n > 0 && !spec_ok) {
        side_join(h);                                    // a speculative side launch exited on the guard
        const bool ovf_main = ovf_on_main();
        if (!ovf_main) {
            CK(side_fork(h));
            launch_finish_ovf_nv(nv, ta, direct, h->xst);
        }
        {
            KScope ks(K_TXN_LAYOUT, n);
            launch_finish_nv(nv, ta, direct, st);
        }
        if (ovf_main) launch_finish_ovf_nv(nv, ta, direct, st);
    }
    if (n > 0 && h->V > 0) { KScope ks(K_VITEMS); launch_large_layout_nv(nv, ta, direct, st); }
    wa.items = items; wa.nitems = nitems;
    launch_walk_nv(nv, wa, true, direct, nitems > 0, st);
    if (ndtx > 0) { KScope ks(K_TXN_UNION, ndtx); launch_union_nv(nv, ua, direct, st); }
    if (Q > 0 && n > 0) launch_range_nv(nv, ra, true, st);
    // large txns' key CSRs and every RangeDeps CSR: LDS sort union (overflowing CSRs queued for a big pass)
    if (n > 0 && (h->n_large > 0 || Q > 0)) {
        KScope ks(K_UNION_LDS);
        LdsUnionArgs la{};
        la.n = n; la.meta = h->meta; la.prm = h->prm;
        constexpr uint32_t OVF_CAP = 1u << 20;
        uint32_t* ovf_count = nullptr;
        uint2* ovf = nullptr;
        CK(dalloc(h, S_OVF, &ovf_count, 64));
        CK(dalloc(h, S_OVFL, &ovf, OVF_CAP));
        HIPCHK(h, hipMemsetAsync(ovf_count, 0, 4, st));
        la.ovf_count = ovf_count; la.ovf = ovf; la.ovf_cap = OVF_CAP;
        if (h->n_large > 0) {
            la.ncsr = nc; la.csr_base = 0; la.csr_step = direct ? 1 : 2; la.only_large = 1;
            for (int vc = 0; vc < nvc; ++vc) {
                Csr& c = h->deps[vc];
                la.key_off[vc] = c.key_off; la.k2t_off[vc] = c.k2t_off; la.ent_off[vc] = c.ent_off; la.k2t[vc] = c.k2t;
                la.txns[vc] = c.txns; la.tcnt[vc] = c.tcnt;
            }
            // one workgroup per (large txn, CSR), not per (txn, CSR)
            uint32_t* lrows = nullptr;
            CK(dalloc(h, S_LROWS, &lrows, n + 64));
            device_scan(LargeRowsOp{h->meta, lrows, lrows + n, n}, n, (uint32_t*)h->scratch, st);
            la.rows = lrows; la.rows_total = lrows + n;
            k_union_lds_views<<<dim3((unsigned)h->n_large, (unsigned)(direct ? 2 : 1)), UB, 0, st>>>(la, nv);
            la.rows = nullptr; la.rows_total = nullptr;
        }
        if (Q > 0) {
            la.ncsr = nv; la.csr_base = nvc; la.csr_step = 1; la.only_large = 0;
            for (int v = 0; v < nv; ++v) {
                Csr& c = h->rdeps[v];
                la.key_off[nvc + v] = c.key_off; la.k2t_off[nvc + v] = c.k2t_off; la.ent_off[nvc + v] = c.ent_off;
                la.k2t[nvc + v] = c.k2t; la.txns[nvc + v] = c.txns; la.tcnt[nvc + v] = c.tcnt;
            }
            // small lists by single-wave workgroups, the rest queued for 256-thread workgroups
            uint32_t* med_count = nullptr;
            uint2* med = nullptr;
            CK(dalloc(h, S_UMEDC, &med_count, 64));
            CK(dalloc(h, S_UMED, &med, (size_t)n * nv + 1));
            HIPCHK(h, hipMemsetAsync(med_count, 0, 4, st));
            la.med_count = med_count; la.med = med;
            k_union_lds_small<<<(unsigned)n, US_T, 0, st>>>(la);
            k_union_lds_list<<<8192, UB, 0, st>>>(la);
        }
        CK(union_overflow(h, la, ovf_count, ovf, Q > 0));
    }
    // Virtual-item work arrays are dead once the CSRs are filled; they stay allocated for the next batch
    // (re-allocating C4's ~90 GB of them every batch cost more than the walks) unless the merge runs out of
    // HBM, when release_dead gives them back (STAGE_MERGE).
    host_mark(h, "deps deps_end");
    if (!h->xdefer) side_join(h);
    if (ta.dbg) {
        side_join(h);
        hipStreamSynchronize(h->xst);
        hipStreamSynchronize(st);
        unsigned long long d[5];
        uint32_t oc = 0;
        hipMemcpy(d, ta.dbg, sizeof d, hipMemcpyDeviceToHost);
        hipMemcpy(&oc, ta.ovf_count, 4, hipMemcpyDeviceToHost);
        fprintf(stderr, "ovf_timers count %u rows %llu clocks avg %.0f max %llu walks %llu emits %llu path %s\n", oc, d[0],
                d[0] ? (double)d[1] / (double)d[0] : 0.0, d[2], d[3], d[4], fuse ? "fuse" : "three-kernel");
    }
    h->have_deps = true;
    h->ls.chains_ready = false;
    h->times.deps_entries = h->deps_entries;
    h->times.key_classes = (uint32_t)nc;
    h->times.level_edges = h->P;
    h->times.walk_items = (uint32_t)(h->P - (h->P ? h->hprm.n_keys_u : 0));
    return AD_OK;
}
