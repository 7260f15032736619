// levels.hip — execution levels and order (level_kernels.h, block_levels.h).
#include "engine_internal.h"
#include "global_levels.h"

// ---------------------------------------------------------------------------------------------------
// levels
// ---------------------------------------------------------------------------------------------------
// Execution order over a batch carrying CFK history: the kept rows (current statuses, ad_cfk_update) and the
// new txns in one graph, APPLIED / INVALID rows done (no edge into or out of them): the constraint edges of
// the combined rows (global_levels.h, the same rules as every level path) solved by the Kahn wavefronts.
// Stable txns of earlier batches are released as soon as what they wait for has applied.
static int levels_history(ad_handle* h, bool want_order) {
    const size_t n = h->n;
    hipStream_t st = h->st;
    size_t m = 0;
    uint32_t depth = 0;
    KScope ks(K_KAHN, h->P);
    CK(levels_export_edges(h, &m, false, true));
    CK(levels_solve_edges(h, h->gl_edges, m, n, h->lvl, &depth));
    uint32_t* key = nullptr;
    CK(dalloc(h, S_GLKEY, &key, std::max<size_t>(n, 1)));
    if (n) k_done_levels<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->meta, h->lvl, key);
    if (want_order && n) {
        if (!ls_reserve_order(h->ls, n, st)) return set_err(h, AD_ERR_NOMEM, "exec levels: out of device memory");
        order_rows(h->ls, n, nullptr, h->ex1, key, h->pack.total_bits, h->order, st);
    }
    HIPCHK(h, hipGetLastError());
    h->level_iters = depth;
    h->times.level_rounds = 0;
    h->times.level_blocks = 0;
    h->have_levels = true;
    return AD_OK;
}

int stage_levels(ad_handle* h, bool want_order) {
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_exec_levels before ad_merge_deps");
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_exec_levels needs ad_preaccept_deps on this batch (its key chains)");
    if (h->hist_active) return levels_history(h, want_order);
    // k_seg_fuse left the entry state to complete_entries: the pull pass's own chain build reads it (the chains
    // k_seg_fuse prebuilt in ad_run_pipeline do not)
    if (h->state_partial && !h->chains_prebuilt) CK(complete_entries(h));
    LevelInputs li{};
    li.n = h->n; li.P = h->P; li.e_txn = h->e_txn; li.e_meta = h->e_meta; li.e_exec1 = h->e_exec1;
    li.seg_start = h->seg_start; li.sval = h->sval; li.nh = h->nh_valid ? h->nh : nullptr;
    if (!h->nh_valid && h->sf_ntiles) {               // k_seg_fuse's per-tile second-entry lists
        li.sec = (const uint32_t*)h->bufs[S_SFSEC].p; li.sec_cap = SF_SEC; li.sec_tiles = (uint32_t)h->sf_ntiles;
        li.sec_cnt = li.sec + h->sf_ntiles * (size_t)SF_SEC;
    } li.prm = h->prm; li.key_off = h->key_off; li.meta = h->meta; li.ex1 = h->ex1;
    li.lvl = h->lvl; li.order = h->order;
    li.merged_key = &h->merged[AD_CLASS_KEY];
    li.merged_direct = &h->merged[AD_CLASS_DIRECT_KEY];
    li.ukey = h->ukey; li.useg = h->useg; li.U = h->P ? h->hprm.n_keys_u : 0;
    li.merged_range = &h->merged[AD_CLASS_RANGE];
    li.n_large = h->n_large;
    li.n_special = h->n_special;
    li.exec_bits = h->pack.total_bits;
    li.kahn_ok = h->level_mode != AD_LEVELS_FIXPOINT ? 1 : 0;
    li.chains_prebuilt = h->chains_prebuilt ? 1 : 0;        // k_seg_fuse built them (ad_run_pipeline)
    h->times.chains_fused = (uint32_t)li.chains_prebuilt;
    h->chains_prebuilt = false;
    li.force_blocks = (h->level_mode == AD_LEVELS_BLOCKS || h->level_mode == AD_LEVELS_BLOCKS_WIDE) ? 1 : 0;
    li.wide_words = h->level_mode == AD_LEVELS_BLOCKS_WIDE ? 1 : 0;
    h->ls.pull_off = h->level_mode == AD_LEVELS_KAHN;
    h->ls.pull_force_abort = h->level_mode == AD_LEVELS_PULL_ABORT;
    h->ls.bl_rounds = 0;
    h->ls.bl_used = false;
    h->order_pending = false;
    set_level_pub(h);
    li.order_verify = nullptr;
    if (h->pub_host) {                       // the optimistic order's failure flag: a host-mapped word
        __atomic_store_n(h->pub_host + 1, 0u, __ATOMIC_RELEASE);
        li.order_verify = h->pub_dev + 1;
    }
    li.order_pending = &h->order_pending;
    int iters = 0;
    // only the pull pass reads nothing but multi-entry key segments; every other level path reads every entry
    const bool pull_first = li.kahn_ok && !li.force_blocks && h->P > 0 && !h->ls.pull_off && h->n_large == 0 &&
                            h->n_special == 0 && h->merged[AD_CLASS_DIRECT_KEY].ncap == 0 &&
                            !(h->merged_has_range && h->merged[AD_CLASS_RANGE].ncap > 0);
    if (!pull_first) {
        side_join(h);                                     // the other level paths read the merged Deps
        CK(merged_ready(h));
        CK(complete_entries(h));
    }
    li.complete = [](void* x) { return complete_entries((ad_handle*)x); };
    li.complete_ctx = h;
    host_mark(h, "levels enqueue");
    int rc = run_levels(h->ls, li, want_order, h->st, &iters, h->err);
    if (rc != AD_OK) return rc;
    h->level_iters = (uint32_t)iters;
    h->times.level_rounds = h->ls.bl_rounds;
    h->times.level_blocks = h->ls.bl_used ? h->ls.bl.nblocks : 0;
    h->times.level_path = h->ls.mixpull_path ? 10u + (uint32_t)h->ls.mixpull_path : (uint32_t)h->ls.pull_path;
    h->have_levels = true;
    return AD_OK;
}

// After a stream sync: if the optimistic execution order failed its verification, redo it on the
// general path (radix sort by executeAt) and wait for it.
bool order_failed(const ad_handle* h) {
    return h->order_pending && h->pub_host && __atomic_load_n(h->pub_host + 1, __ATOMIC_ACQUIRE) != 0u;
}
int finish_order(ad_handle* h) {
    if (!h->order_pending) return AD_OK;
    const bool bad = order_failed(h);
    h->order_pending = false;
    if (!bad) return AD_OK;
    order_rows(h->ls, h->n, nullptr, h->ex1, h->lvl, h->pack.total_bits, h->order, h->st);
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}


int levels_run(ad_handle* h, const LevelInputs& li, bool want_order, int* iters) {
    set_level_pub(h);
    return run_levels(h->ls, li, want_order, h->st, iters, h->err);
}
void levels_order_rows(ad_handle* h, size_t m, const uint32_t* rows, uint32_t* out) {
    order_rows(h->ls, m, rows, h->ex1, h->lvl, h->pack.total_bits, out, h->st);
}

// ---------------------------------------------------------------------------------------------------
// one-exchange sharded levels (global_levels.h)
// ---------------------------------------------------------------------------------------------------
int levels_export_edges(ad_handle* h, size_t* m_out, bool global_ranks, bool done_aware) {
    CK(complete_entries(h));
    CK(merged_ready(h));
    const size_t n = h->n, P = h->P;
    hipStream_t st = h->st;
    const uint32_t* gid = global_ranks ? h->gid : nullptr;
    h->gl_ready = false;
    // key chains in executeAt order (stable insertion per segment: only slow-path bumps move)
    uint32_t *c_txn, *c_pair;
    uint8_t* c_meta;
    uint64_t* c_exec1;
    int32_t* last_w;
    unsigned long long *ecnt, *eoff, *xcnt, *xoff;
    const size_t P1 = std::max<size_t>(P, 1), n1 = std::max<size_t>(n, 1);
    CK(dalloc(h, S_GLCT, &c_txn, P1)); CK(dalloc(h, S_GLCM, &c_meta, P1)); CK(dalloc(h, S_GLCE, &c_exec1, P1));
    CK(dalloc(h, S_GLCP, &c_pair, P1)); CK(dalloc(h, S_GLLW, &last_w, P1));
    CK(dalloc(h, S_GLEC, &ecnt, P1)); CK(dalloc(h, S_GLEO, &eoff, P + 1));
    CK(dalloc(h, S_GLXC, &xcnt, n1)); CK(dalloc(h, S_GLXO, &xoff, n + 1));
    CK(ensure_scratch(h, std::max(h->scratch_cap, std::max(device_scan_scratch<WriteLinkOp<false>>(P1),
                                                            device_scan_scratch<SumOp<unsigned long long>>(std::max(P1, n1))))));
    const int gP = ceil_div((long)P1, 256), gn = ceil_div((long)n1, 256);
    if (P > 0) {
        k_chain_copy<<<gP, 256, 0, st>>>(P, h->e_txn, h->e_meta, h->e_exec1, h->sval, c_txn, c_meta, c_exec1, c_pair);
        k_chain_order<<<gP, 256, 0, st>>>(P, h->seg_start, c_txn, c_meta, c_exec1, c_pair);
        if (done_aware) k_chain_mask_invalid<<<gP, 256, 0, st>>>(P, c_meta);
        device_scan(WriteLinkOp<false>{P, h->seg_start, c_meta, last_w}, P, (WriteLinkOp<false>::S*)h->scratch, st);
        k_chain_edges<false><<<gP, 256, 0, st>>>(P, h->seg_start, c_txn, c_meta, last_w, gid, done_aware ? 1 : 0, ecnt, nullptr, nullptr);
        scan_any(h, SumOp<unsigned long long>{ecnt, eoff, P}, P);
    } else {
        HIPCHK(h, hipMemsetAsync(eoff, 0, 8, st));
    }
    // (b) direct / range dependency edges and (c) unmanaged chain bounds, from this store's merged views
    const Csr* md = &h->merged[AD_CLASS_DIRECT_KEY];
    const Csr* mr = &h->merged[AD_CLASS_RANGE];
    const Csr* mk = &h->merged[AD_CLASS_KEY];
    const bool has_b = h->have_merged && ((md->ncap > 0) || (h->merged_has_range && mr->ncap > 0));
    const bool has_c = h->have_merged && (h->n_large > 0 || h->n_special > 0) && mk->nkeys > 0 && P > 0;
    XEdgeArgs xa{};
    if (has_b || has_c) {
        EdgeArgs& ea = xa.e;
        ea.n = n; ea.meta = h->meta; ea.ex1 = h->ex1;
        const Csr* bc[2] = {md, h->merged_has_range ? mr : nullptr};
        for (int c = 0; c < 2; ++c)
            if (bc[c] && bc[c]->ncap > 0) { ea.ent_off[c] = bc[c]->ent_off; ea.tcnt[c] = bc[c]->tcnt; ea.txns[c] = bc[c]->txns; }
        ea.mk_key_off = mk->key_off; ea.mk_keys = mk->keys; ea.mk_k2t_off = mk->k2t_off; ea.mk_k2t = mk->k2t;
        ea.mk_ent_off = mk->ent_off; ea.mk_txns = mk->txns;
        int32_t* cons = nullptr;
        CK(dalloc(h, S_GLCONS, &cons, std::max<size_t>(mk->nkeys, 1)));
        ea.cons_pos = cons; ea.ukey = h->ukey; ea.useg = h->useg; ea.U = P ? h->hprm.n_keys_u : 0;
        ea.c_exec1 = c_exec1; ea.c_txn = c_txn; ea.seg_start = h->seg_start;
        ea.e_txn = h->e_txn; ea.e_meta = h->e_meta; ea.e_exec1 = h->e_exec1;
        xa.c_meta = c_meta; xa.do_b = has_b ? 1 : 0; xa.do_c = has_c ? 1 : 0; xa.done_aware = done_aware ? 1 : 0;
        if (has_c) k_unmanaged_prep<<<ceil_div((long)n * WAVE, 256), 256, 0, st>>>(ea);
        if (n) {
            k_xedge_pairs<false><<<gn, 256, 0, st>>>(xa, gid, xcnt, nullptr, nullptr);
            scan_any(h, SumOp<unsigned long long>{xcnt, xoff, n}, n);
        }
    }
    unsigned long long ta = 0, tb = 0;
    if (P > 0) HIPCHK(h, hipMemcpyAsync(&ta, eoff + P, 8, hipMemcpyDeviceToHost, st));
    if ((has_b || has_c) && n) HIPCHK(h, hipMemcpyAsync(&tb, xoff + n, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    CK(dalloc(h, S_GLE, &h->gl_edges, std::max<size_t>(ta + tb, 1)));
    if (ta) k_chain_edges<true><<<gP, 256, 0, st>>>(P, h->seg_start, c_txn, c_meta, last_w, gid, done_aware ? 1 : 0, nullptr, eoff, h->gl_edges);
    if (tb) k_xedge_pairs<true><<<gn, 256, 0, st>>>(xa, gid, nullptr, xoff, h->gl_edges + ta);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipStreamSynchronize(st));
    h->gl_m = ta + tb;
    h->gl_ready = true;
    *m_out = h->gl_m;
    return AD_OK;
}

// Levels of N txns from an edge set over them (device, m edges): in-degrees, edges sorted by source into
// successor lists, then Kahn wavefronts over them (batches of launches per host sync; narrow deep frontiers
// inside one workgroup, k_kahn_small).  Result in L[0..N] (N + 1 words); *depth = number of levels.
int levels_solve_edges(ad_handle* h, const uint64_t* d_edges, size_t m, size_t N, uint32_t* L, uint32_t* depth) {
    hipStream_t st = h->st;
    uint32_t *src, *dst, *src2, *dst2, *indeg, *rem, *fl, *front;
    uint64_t* xoff;
    const size_t m1 = std::max<size_t>(m, 1), N1 = std::max<size_t>(N, 1);
    CK(dalloc(h, S_GLSRC, &src, m1)); CK(dalloc(h, S_GLDST, &dst, m1));
    CK(dalloc(h, S_GLSRC2, &src2, m1)); CK(dalloc(h, S_GLDST2, &dst2, m1));
    CK(dalloc(h, S_GLDEG, &indeg, N1)); CK(dalloc(h, S_GLREM, &rem, N1)); CK(dalloc(h, S_GLXOFF, &xoff, N + 1));
    CK(dalloc(h, S_GLFL, &fl, 4 * 64 + 64)); CK(dalloc(h, S_GLFRONT, &front, 2 * KS_MAX + 4));
    CK(ensure_scratch(h, std::max(h->scratch_cap, (size_t)(3 * (radix_hist_len(m1) + 128) + 64 * 1024) * 4)));
    HIPCHK(h, hipMemsetAsync(indeg, 0, N1 * 4, st));
    HIPCHK(h, hipMemsetAsync(L, 0, (N + 1) * 4, st));
    HIPCHK(h, hipMemsetAsync(fl, 0, (4 * 64 + 64) * 4, st));
    uint32_t* bad = fl + 4 * 64;             // [0] bad edge; [1] always zero (the first wavefront's gate)
    if (m) k_edges_split<<<ceil_div((long)m, 256), 256, 0, st>>>(m, d_edges, src, dst, indeg, (uint32_t)N, bad);
    uint32_t hb = 0;
    HIPCHK(h, hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (hb) return set_err(h, AD_ERR_ARGUMENT, "level edges: a global rank out of range or a self edge");
    const uint32_t* xs = dst;
    const uint32_t* ssrc = src;
    if (m) {
        const int bits = std::max(1, bits_of(N - 1));
        if (radix_sort_pairs(src, dst, src2, dst2, m, bits, radix_scratch(h, m), st)) { ssrc = src2; xs = dst2; }
        k_xoff_bounds<<<ceil_div((long)N + 1, 256), 256, 0, st>>>(m, ssrc, (uint32_t)N, xoff);
    } else {
        HIPCHK(h, hipMemsetAsync(xoff, 0, (N + 1) * 8, st));
    }
    HIPCHK(h, hipMemcpyAsync(rem, indeg, N1 * 4, hipMemcpyDeviceToDevice, st));
    constexpr int KB_MAX = 64;
    const int gn = std::min(ceil_div((long)N1, 256), KAHN_GRID);
    int KB = 16, lv = 0;
    bool more = N > 0;
    while (more) {
        HIPCHK(h, hipMemsetAsync(fl, 0, KB * 4, st));
        for (int k = 0; k < KB; ++k)
            k_kahn_step<<<gn, 256, 0, st>>>(N, (uint32_t)(lv + k), indeg, rem, L, nullptr, nullptr, nullptr,
                                            k == 0 ? bad + 1 : fl + (k - 1), k == 0, fl + k, xoff, xs);
        uint32_t fh[KB_MAX];
        HIPCHK(h, hipMemcpyAsync(fh, fl, KB * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        int k = 0;
        while (k < KB && fh[k]) ++k;
        if (k < KB) { lv += k + 1; break; }
        lv += KB;
        KB = std::min(KB_MAX, 2 * KB);
        // a deep graph: narrow wavefronts run inside one workgroup until one is wide again
        uint32_t* kst = front + 2 * KS_MAX;
        HIPCHK(h, hipMemsetAsync(kst, 0, 16, st));
        k_frontier_collect<<<ceil_div((long)N, 256), 256, 0, st>>>(N, (uint32_t)lv, indeg, L, front, kst);
        k_kahn_small<<<1, KS_T, 0, st>>>((uint32_t)lv, kst, front, front + KS_MAX, rem, L, nullptr, nullptr, nullptr, xoff, xs);
        uint32_t ks[3] = {0, 0, 0};
        HIPCHK(h, hipMemcpyAsync(ks, kst, 12, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        if (ks[0] == 0) { lv = (int)ks[1] + 1; break; }
        if ((int)ks[1] != lv) KB = 16;          // resumed at a new wide level
        lv = (int)ks[1];
    }
    // every txn released exactly once: the in-degrees are consumed (a cycle would leave some unreleased)
    HIPCHK(h, hipMemsetAsync(bad, 0, 4, st));
    if (N) k_rem_check<<<ceil_div((long)N, 256), 256, 0, st>>>(N, rem, bad);
    HIPCHK(h, hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    HIPCHK(h, hipGetLastError());
    if (hb) return set_err(h, AD_ERR_ARGUMENT, "level edges: the gathered constraints contain a cycle");
    if (depth) *depth = (uint32_t)lv;
    h->level_iters = (uint32_t)lv;
    return AD_OK;
}
