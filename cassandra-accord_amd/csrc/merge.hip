// merge.hip — Deps.merge of the replica views (and of host / shard parts) on the device.
#include "engine_internal.h"

// ---------------------------------------------------------------------------------------------------
// merge
// ---------------------------------------------------------------------------------------------------
static bool getenv_flag(const char* name) { const char* e = getenv(name); return e && *e && *e != '0'; }

template <int K>
void launch_multi_offsets(ad_handle* h, size_t n, const uint32_t* mk, const uint32_t* me, const uint32_t* mu, Csr* const* out) {
    MultiOffsetsOp<K> op{};
    op.n = n; op.mk = mk; op.me = me; op.mu = mu;
    for (int c = 0; c < K; ++c) { op.key_off[c] = out[c]->key_off; op.ent_off[c] = out[c]->ent_off; op.k2t_off[c] = out[c]->k2t_off; }
    scan_any(h, op, n);
}

// K unions computed together (count, one fused offsets scan, ONE host sync, allocation, write):
// out[k] = Deps.merge over in[k][0..np) per output txn; rows[k][v] (nullable) maps output txn -> input row.
int merge_multi(ad_handle* h, size_t n, int K, Csr* const* out, const size_t* out_block, const int* kw,
                const Csr* const (*in)[MAXV], const int32_t* const (*rows)[MAXV], int np, uint64_t* entries) {
    hipStream_t st = h->st;
    uint32_t *mk, *me, *mu;
    CK(dalloc(h, S_MSCR, &mk, 3 * (size_t)K * n + 3));
    me = mk + (size_t)K * n;
    mu = me + (size_t)K * n;
    uint32_t* hl;                                   // heavy-txn lists [K * n] + counters [K]
    CK(dalloc(h, S_MHL, &hl, (size_t)K * n + 64));
    uint32_t* hc = hl + (size_t)K * n;
    uint8_t* hs;                                    // heavy txns' identical-replies flags [K * n]
    CK(dalloc(h, S_MHS, &hs, (size_t)K * n + 64));
    if (n > 0) HIPCHK(h, hipMemsetAsync(hc, 0, (size_t)K * 4, st));
    std::vector<MergeArgs> ma(K);
    for (int k = 0; k < K; ++k) {
        CK(alloc_csr(h, out_block[k], *out[k], n));
        dirty_csr(h, out_block[k]);
        MergeArgs& a = ma[k];
        a = MergeArgs{};
        a.n = n; a.nv = np;
        for (int v = 0; v < np; ++v) {
            const Csr& c = *in[k][v];
            a.key_off[v] = c.key_off; a.keys[v] = c.keys; a.k2t_off[v] = c.k2t_off; a.k2t[v] = c.k2t;
            a.ent_off[v] = c.ent_off; a.txns[v] = c.txns; a.tcnt[v] = c.tcnt;
            a.row[v] = rows ? rows[k][v] : nullptr;
        }
        a.mk = mk + (size_t)k * n; a.me = me + (size_t)k * n; a.mu = mu + (size_t)k * n;
        if (h->merge_heavy) { a.hlist = hl + (size_t)k * n; a.hcount = hc + k; a.hsame = hs + (size_t)k * n; }
        if (n > 0) merge_launch(a, np, false, kw[k], st);
    }
    if (n > 0) {
        KScope ks(K_MERGE_OFFSETS, n * (size_t)K);
        switch (K) {
            case 1: launch_multi_offsets<1>(h, n, mk, me, mu, out); break;
            case 2: launch_multi_offsets<2>(h, n, mk, me, mu, out); break;
            case 3: launch_multi_offsets<3>(h, n, mk, me, mu, out); break;
            case 4: launch_multi_offsets<4>(h, n, mk, me, mu, out); break;
            case 5: launch_multi_offsets<5>(h, n, mk, me, mu, out); break;
            case 6: launch_multi_offsets<6>(h, n, mk, me, mu, out); break;
            case 7: launch_multi_offsets<7>(h, n, mk, me, mu, out); break;
            case 8: launch_multi_offsets<8>(h, n, mk, me, mu, out); break;
            case 10: launch_multi_offsets<10>(h, n, mk, me, mu, out); break;
            case 12: launch_multi_offsets<12>(h, n, mk, me, mu, out); break;
            case 14: launch_multi_offsets<14>(h, n, mk, me, mu, out); break;
            case 16: launch_multi_offsets<16>(h, n, mk, me, mu, out); break;
            default: return set_err(h, AD_ERR_UNSUPPORTED, "merge_multi: unsupported output count");
        }
    } else {
        for (int k = 0; k < K; ++k) {
            HIPCHK(h, hipMemsetAsync(out[k]->key_off, 0, 4, st));
            HIPCHK(h, hipMemsetAsync(out[k]->ent_off, 0, 4, st));
            HIPCHK(h, hipMemsetAsync(out[k]->k2t_off, 0, 4, st));
        }
    }
    std::vector<uint32_t> tot(3 * K, 0);
    TotTable tt{};
    for (int k = 0; k < K; ++k) {
        tt.src[3 * k + 0] = out[k]->key_off + n; tt.src[3 * k + 1] = out[k]->k2t_off + n; tt.src[3 * k + 2] = out[k]->ent_off + n;
    }
    tt.count = 3 * K;
    // Speculative write pass (as the deps stage's finish): into the output buffers an earlier batch left, behind
    // k_cap_check's guard, enqueued before the host reads the merged sizes; re-run after sizing only if it fired.
    uint32_t* spec_bad = h->totd + MAX_TOTALS - 5;
    bool spec = n > 0;
    CapCheck capc{};
    for (int k = 0; k < K && spec; ++k) {
        const size_t base = S_CSR0 + 10 * out_block[k];
        const size_t ck = csr_cap(h, out_block[k], 4, 8 * (size_t)kw[k]), cm = csr_cap(h, out_block[k], 5, 4),
                     ct = csr_cap(h, out_block[k], 6, 4);
        if (!ck || !cm || !ct) { spec = false; break; }
        const Csr& m = *out[k];
        const uint32_t* tots[3] = {m.key_off + n, m.k2t_off + n, m.ent_off + n};
        const size_t caps[3] = {ck, cm, ct};
        for (int q = 0; q < 3; ++q) { capc.tot[capc.m] = tots[q]; capc.cap[capc.m++] = (uint32_t)std::min<size_t>(caps[q], 0xFFFFFFFFu); }
        MergeArgs& a = ma[k];
        a.o_key_off = m.key_off; a.o_keys = (uint64_t*)h->bufs[base + 4].p; a.o_k2t_off = m.k2t_off;
        a.o_k2t = (int32_t*)h->bufs[base + 5].p; a.o_ent_off = m.ent_off; a.o_txns = (uint32_t*)h->bufs[base + 6].p;
        a.o_tcnt = m.tcnt;
    }
    if (spec) {
        capc.bad = spec_bad;
        k_cap_check<<<1, 64, 0, st>>>(capc);
        tt.src[tt.count++] = spec_bad;
    }
    std::vector<uint32_t> got(tt.count, 0);
    uint32_t seq = 0;
    CK(publish_totals(h, tt, got.data(), &seq));       // the read-back first, then the speculative write
    if (spec) {
        for (int k = 0; k < K; ++k) {
            ma[k].spec_bad = spec_bad;
            merge_launch(ma[k], np, true, kw[k], st);
            ma[k].spec_bad = nullptr;
        }
    }
    CK(wait_totals(h, seq, tt.count, got.data()));
    std::copy(got.begin(), got.begin() + 3 * K, tot.begin());
    CK(check_params(h));
    const bool spec_ok = spec && got[3 * K] == 0;
    for (int k = 0; k < K; ++k) {
        Csr& m = *out[k];
        m.nkeys = tot[3 * k]; m.nk2t = tot[3 * k + 1]; m.ncap = tot[3 * k + 2];
        if (entries) *entries += m.nk2t - m.nkeys;
        CK(alloc_csr_data(h, out_block[k], m, kw[k]));
        MergeArgs& a = ma[k];
        a.o_key_off = m.key_off; a.o_keys = m.keys; a.o_k2t_off = m.k2t_off; a.o_k2t = m.k2t;
        a.o_ent_off = m.ent_off; a.o_txns = m.txns; a.o_tcnt = m.tcnt;
        if (n > 0 && !spec_ok) merge_launch(a, np, true, kw[k], st);
    }
    return AD_OK;
}

// Deps.merge of `np` parts per class into h->merged.  parts[cls][v] are batched per-txn CSRs over the loaded batch;
// view_rows[v] (nullable) maps txn -> row of part v, -1 = leave that reply out for the txn.
int merge_parts(ad_handle* h, const Csr* const parts[3][MAXV], int np, bool has_range, const int32_t* const* view_rows,
                bool has_direct) {
    const size_t n = h->n;
    h->merged_entries = 0;
    h->merged_cap = false;
    h->mcap_entries_pending = false;
    Csr* out[3];
    size_t blocks[3];
    int kw[3];
    const Csr* in[3][MAXV] = {};
    const int32_t* rows[3][MAXV] = {};
    int K = 0;
    for (int cls = 0; cls < 3; ++cls) {
        if ((cls == AD_CLASS_RANGE && !has_range) || (cls == AD_CLASS_DIRECT_KEY && !has_direct)) {
            // an empty class in every part: an empty merged class (zero offsets, kept from the previous batch
            // when still valid)
            CK(zero_csr(h, CSR_MERGED0 + cls, h->merged[cls], n));
            continue;
        }
        out[K] = &h->merged[cls];
        blocks[K] = CSR_MERGED0 + cls;
        kw[K] = cls == AD_CLASS_RANGE ? 2 : 1;
        for (int v = 0; v < np; ++v) { in[K][v] = parts[cls][v]; rows[K][v] = view_rows ? view_rows[v] : nullptr; }
        ++K;
    }
    CK(merge_multi(h, n, K, out, blocks, kw, in, view_rows ? rows : nullptr, np, &h->merged_entries));
    h->merged_exact = true;
    h->have_merged = true;
    return AD_OK;
}

// Deps.merge of the R replies' key classes (merge_kernels.h: k_merge_ref, one thread per txn; the txns whose replies
// differ merged in the same pass): the merged rows as references to a reply plus a region of merged rows, one launch,
// no host round trip.  Batches whose deps stage saw no heavy txn, no range and no virtual items (the rest go through merge_parts).
template <int NV>
static void launch_merge_cap(const MergeCapArgs& a, unsigned g, hipStream_t st) { k_merge_ref<NV><<<g, 256, 0, st>>>(a); }
template <int NV>
static void launch_merge_ready_counts(const MergeCapArgs& a, uint32_t* k, uint32_t* m, uint32_t* t, hipStream_t st) {
    k_merge_ready_counts<NV><<<ceil_div((long)a.n, 256), 256, 0, st>>>(a, k, m, t);
}
template <int NV>
static void launch_merge_ready_copy(const MergeCapArgs& a, const Csr& x, const uint32_t* k, const uint32_t* m,
                                    const uint32_t* t, hipStream_t st) {
    k_merge_ready_copy<NV><<<ceil_div((long)a.n, 256), 256, 0, st>>>(a, x.key_off, x.k2t_off, x.ent_off, k, m, t, x.keys, x.k2t, x.txns);
}

static int merge_cap(ad_handle* h) {
    const size_t n = h->n;
    const int nv = (int)h->cfg.replicas;
    hipStream_t st = h->st;
    const bool direct = h->deps_direct;
    CK(zero_csr(h, CSR_MERGED0 + AD_CLASS_RANGE, h->merged[AD_CLASS_RANGE], n));
    if (!direct) CK(zero_csr(h, CSR_MERGED0 + AD_CLASS_DIRECT_KEY, h->merged[AD_CLASS_DIRECT_KEY], n));
    const unsigned g = (unsigned)ceil_div((long)n, 256);
    h->mcap_blocks = g;
    // per class two sets of 4 counters (merged txns, region keys / words / ids): this call's and the next's (zeroed by
    // this call), alternating
    uint32_t* ctr = nullptr;
    const bool fresh = h->bufs.size() <= S_MCL || !h->bufs[S_MCL].p;
    CK(dalloc(h, S_MCL, &ctr, 16));
    if (fresh) HIPCHK(h, hipMemsetAsync(ctr, 0, 64, st));
    const int ph = h->mcap_phase;
    h->mcap_phase ^= 1;
    const size_t n1 = std::max<size_t>(n, 1);
    for (int c = 0; c < (direct ? 2 : 1); ++c) {
        Csr m{};
        const size_t block = CSR_MCAP0 + c;
        MergeCapArgs& a = h->mcap_args[c];
        a = MergeCapArgs{};
        a.n = n;
        for (int v = 0; v < nv; ++v) {
            const Csr& x = h->deps[2 * v + c];
            m.nkeys += x.nkeys; m.nk2t += x.nk2t; m.ncap += x.ncap;
            a.key_off[v] = x.key_off; a.keys[v] = x.keys; a.k2t_off[v] = x.k2t_off; a.k2t[v] = x.k2t;
            a.ent_off[v] = x.ent_off; a.txns[v] = x.txns; a.tcnt[v] = x.tcnt;
        }
        CK(alloc_csr_data(h, block, m, 1));                  // the merged-row region: the replies' totals
        uint32_t* lst = nullptr;
        CK(dalloc(h, S_MCLS0 + c, &lst, 8 * n1));            // list, lidx, six per-list arrays
        CK(dalloc(h, S_MCK0 + c, &a.src, n1));
        CK(dalloc(h, S_MCP0 + c, &h->mcap_part[c], std::max<size_t>(h->mcap_blocks, 1)));
        a.list = lst; a.lidx = lst + n1;
        a.l_koff = lst + 2 * n1; a.l_moff = lst + 3 * n1; a.l_toff = lst + 4 * n1;
        a.l_kcnt = lst + 5 * n1; a.l_ment = lst + 6 * n1; a.l_tcnt = lst + 7 * n1;
        a.cnt = ctr + 8 * c + 4 * ph; a.cnt_next = ctr + 8 * c + 4 * (ph ^ 1);
        a.o_keys = m.keys; a.o_k2t = m.k2t; a.o_txns = m.txns;
        a.part = h->mcap_part[c]; a.part2 = g;
        if (n) {
            KScope ks(K_MERGE_CAP, n);
            NV_DISPATCH(nv, launch_merge_cap, a, g, st);
        }
        h->merged[c] = m;                                    // the region's sizes (ncap > 0 iff any reply has deps)
    }
    h->mcap_direct = direct;
    h->merged_cap = true;
    h->merged_exact = true;
    h->merged_compacted = false;
    h->mcap_entries_pending = n > 0;
    h->merged_entries = 0;
    h->have_merged = true;
    return AD_OK;
}

int merged_entries_resolve(ad_handle* h) {
    if (!h->mcap_entries_pending) return AD_OK;
    h->mcap_entries_pending = false;
    uint64_t tot = 0;
    if (h->merged_cap) {
        std::vector<uint32_t> p(h->mcap_blocks);
        for (int c = 0; c < (h->mcap_direct ? 2 : 1) && h->mcap_blocks; ++c) {
            HIPCHK(h, hipMemcpyAsync(p.data(), h->mcap_part[c], p.size() * 4, hipMemcpyDeviceToHost, h->st));
            HIPCHK(h, hipStreamSynchronize(h->st));
            for (uint32_t x : p) tot += x;
        }
        h->merged_entries = tot;
        h->times.merged_entries = tot;
    }
    return AD_OK;
}

int merged_ready(ad_handle* h) {
    if (!h->merged_cap) return AD_OK;
    CK(merged_entries_resolve(h));
    const size_t n = h->n;
    const int nv = (int)h->cfg.replicas;
    hipStream_t st = h->st;
    CK(ensure_scratch(h, device_scan_scratch<MultiOffsetsOp<1>>(std::max<size_t>(n, 1))));
    uint32_t* cnts = nullptr;
    CK(dalloc(h, S_MCE0, &cnts, 3 * std::max<size_t>(n, 1)));
    for (int c = 0; c < (h->mcap_direct ? 2 : 1); ++c) {
        const MergeCapArgs& a = h->mcap_args[c];
        Csr x{};
        const size_t block = CSR_MERGED0 + c;
        CK(alloc_csr(h, block, x, n));
        dirty_csr(h, block);
        uint32_t *kc = cnts, *me = cnts + std::max<size_t>(n, 1), *tc = cnts + 2 * std::max<size_t>(n, 1);
        if (n) {
            NV_DISPATCH(nv, launch_merge_ready_counts, a, kc, me, tc, st);
            MultiOffsetsOp<1> op{};
            op.n = n; op.mk = kc; op.me = me; op.mu = tc;
            op.key_off[0] = x.key_off; op.ent_off[0] = x.ent_off; op.k2t_off[0] = x.k2t_off;
            scan_any(h, op, n);
            HIPCHK(h, hipMemcpyAsync(x.tcnt, tc, n * 4, hipMemcpyDeviceToDevice, st));
        } else {
            HIPCHK(h, hipMemsetAsync(x.key_off, 0, 4, st));
            HIPCHK(h, hipMemsetAsync(x.k2t_off, 0, 4, st));
            HIPCHK(h, hipMemsetAsync(x.ent_off, 0, 4, st));
        }
        uint32_t tot[3] = {0, 0, 0};
        HIPCHK(h, hipMemcpyAsync(&tot[0], x.key_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(&tot[1], x.k2t_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(&tot[2], x.ent_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        x.nkeys = tot[0]; x.nk2t = tot[1]; x.ncap = tot[2];
        CK(alloc_csr_data(h, block, x, 1));
        if (n) NV_DISPATCH(nv, launch_merge_ready_copy, a, x, kc, me, tc, st);
        HIPCHK(h, hipGetLastError());
        h->merged[c] = x;
    }
    h->merged_cap = false;
    return AD_OK;
}

int stage_merge(ad_handle* h) {
    StageScope sc(h, STAGE_MERGE);
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_merge_deps before ad_preaccept_deps");
    const int nv = (int)h->cfg.replicas;
    h->merged_cap = false;
    h->mcap_entries_pending = false;
    if (h->deps_union) {
        // the deps stage built the union view (stage_deps): the merged key classes are its CSRs, the range class
        // is empty (no range txns in such a batch)
        const size_t n = h->n;
        h->merged[AD_CLASS_KEY] = h->deps[2 * nv];
        h->merged[AD_CLASS_DIRECT_KEY] = h->deps[2 * nv + 1];
        CK(zero_csr(h, CSR_MERGED0 + AD_CLASS_RANGE, h->merged[AD_CLASS_RANGE], n));
        h->merged_entries = 0;
        for (int c = 0; c < 2; ++c) h->merged_entries += h->merged[c].nk2t - h->merged[c].nkeys;
        h->merged_exact = false;
        h->merged_compacted = false;
        h->have_merged = true;
        return AD_OK;
    }
    side_join(h);                                       // the merge reads every reply's CSRs
    if (!h->merge_heavy && h->Q == 0 && h->n_large == 0 && !getenv_flag("AD_NO_MERGE_CAP")) {
        h->merged_has_range = false;
        if (!h->merge_side || getenv_flag("AD_NO_MERGE_SIDE")) return merge_cap(h);
        // ad_run_pipeline: the merge on the side stream, behind everything the main stream has queued (the finish,
        // and the overflowed rows already on xst), while the main stream runs the levels.  The level paths that
        // read the merged Deps join it first (stage_levels); the pull pass and the block walk of a key Read/Write
        // batch read only the key chains — C3's one-workgroup walk leaves the rest of the chip to the merge.
        CK(side_fork(h));
        hipStream_t main = h->st, tr = h->tracer.st;
        h->st = h->xst;
        h->tracer.st = h->xst;
        const int rc = merge_cap(h);
        h->st = main;
        h->tracer.st = tr;
        h->xjoin = true;
        if (rc == AD_OK) {
            HIPCHK(h, hipEventRecord(h->ev[4], h->xst));
            h->merge_sided = true;
        }
        return rc;
    }
    const Csr* parts[3][MAXV] = {};
    for (int v = 0; v < nv; ++v) {
        parts[0][v] = &h->deps[2 * v];
        parts[1][v] = &h->deps[2 * v + 1];
        parts[2][v] = &h->rdeps[v];
    }
    return merge_parts(h, parts, nv, h->Q > 0, nullptr, h->deps_direct);
}
