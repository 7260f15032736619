// engine.hip — host orchestration + C-ABI (include/accord_deps.h) of the gfx950 deps engine.
//
// One ad_handle = one CommandStore shard on one GPU: a HIP stream, a device arena and the loaded
// batch.  Stages:
//   prepare   batch statistics, timestamp packing (ts64), pair owners, footprint checks   (deps_kernels.h)
//   sort      stable LSD radix sort of (key, pair); range entries by (start, end, owner)  (radix_sort.h)
//   deps      CFK elision scan, per-pair / per-virtual-item walks (count, fill), per-txn KeyDeps
//             layout, TxnId unions; RangeDeps interval join                               (deps/union/range)
//   merge     Deps.merge of the R replica views per txn, all three classes                (merge_kernels.h)
//   levels    execution levels over key chains + deps                                     (level_kernels.h)
#include "engine_internal.h"

int set_err(ad_handle* h, int code, const std::string& msg) {
    h->err = msg;
    return code;
}

// Releases slot `slot` (its next dalloc allocates afresh).
int drelease(ad_handle* h, size_t slot) {
    if (slot < h->bufs.size() && h->bufs[slot].p) {
        HIPCHK(h, hipStreamSynchronize(h->st));
        HIPCHK(h, hipFree(h->bufs[slot].p));
        h->bufs[slot] = DBuf{};
    }
    return AD_OK;
}

// Buffers no later step of the running stage reads: while the deps of a new batch are built, the previous
// batch's merged Deps, uploaded replies, merge scratch and level state; while merging, the level state.
// (Full-size mixed batches hold ~10^9 dependency entries per replica view; this is what lets consecutive
// batches reuse one handle inside 288 GB.)
void release_dead(ad_handle* h) {
    (void)hipStreamSynchronize(h->st);
    auto rel = [&](size_t slot) {
        if (slot < h->bufs.size() && h->bufs[slot].p) { (void)hipFree(h->bufs[slot].p); h->bufs[slot] = DBuf{}; }
    };
    if (h->stage == STAGE_MERGE) {
        for (size_t sl : {S_VTXN, S_VPOS, S_VSEG, S_VCNT}) rel(sl);
        h->vi_txn = h->vi_pos = h->vi_u = h->vcnt = nullptr;
    }
    if (h->stage == STAGE_DEPS) {
        for (size_t blk = CSR_MERGED0; blk < CSR_HOST0 + 3 * MAXV; ++blk)
            for (size_t k = 0; k < 10; ++k) rel(S_CSR0 + 10 * blk + k);
        rel(S_MSCR); rel(S_MHL);
        h->have_merged = h->have_levels = false;
    }
    free_level_state(h->ls);
    h->have_levels = false;
}

int ensure_scratch(ad_handle* h, size_t bytes) {
    void* p;
    CK(dalloc(h, S_SCRATCH, (uint8_t**)&p, bytes));
    h->scratch = p;
    h->scratch_cap = bytes;
    return AD_OK;
}

int alloc_csr(ad_handle* h, size_t block, Csr& c, size_t n) {
    const size_t base = S_CSR0 + 10 * block;
    CK(dalloc(h, base + 0, &c.key_off, n + 1));
    CK(dalloc(h, base + 1, &c.k2t_off, n + 1));
    CK(dalloc(h, base + 2, &c.ent_off, n + 1));
    CK(dalloc(h, base + 3, &c.tcnt, n));
    return AD_OK;
}
int alloc_csr_data(ad_handle* h, size_t block, Csr& c, int kw) {
    const size_t base = S_CSR0 + 10 * block;
    CK(dalloc(h, base + 4, &c.keys, c.nkeys * kw));
    CK(dalloc(h, base + 5, &c.k2t, c.nk2t));
    CK(dalloc(h, base + 6, &c.txns, c.ncap));
    return AD_OK;
}

int zero_csr(ad_handle* h, size_t block, Csr& c, size_t n) {
    CK(alloc_csr(h, block, c, n));
    c.nkeys = c.nk2t = c.ncap = 0;
    CK(alloc_csr_data(h, block, c, 1));
    if (block < CSR_BLOCKS_MAX && h->zero_p[block] == c.key_off && h->zero_n[block] == n && h->zero_gen[block] == h->alloc_gen)
        return AD_OK;
    HIPCHK(h, hipMemsetAsync(c.key_off, 0, (n + 1) * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.k2t_off, 0, (n + 1) * 4, h->st));
    HIPCHK(h, hipMemsetAsync(c.ent_off, 0, (n + 1) * 4, h->st));
    if (n) HIPCHK(h, hipMemsetAsync(c.tcnt, 0, n * 4, h->st));
    if (block < CSR_BLOCKS_MAX) { h->zero_p[block] = c.key_off; h->zero_n[block] = n; h->zero_gen[block] = h->alloc_gen; }
    return AD_OK;
}

// key_off / ent_off / k2t_off of one batched CSR from per-txn (keys, entries) counts
void csr_offsets(ad_handle* h, Csr& c, const uint32_t* nk, const uint32_t* ne) {
    const size_t n = h->n;
    KScope ks(K_CSR_OFFSETS, n);
    scan_offsets(h, nk, c.key_off, n);
    scan_offsets(h, ne, c.ent_off, n);
    if (n) scan_any(h, Sum2Op<uint32_t>{nk, ne, c.k2t_off, n}, n);
    else hipMemsetAsync(c.k2t_off, 0, 4, h->st);
}

// The [n] totals of several device offset arrays and the batch Params -> host.  A stream sync costs the
// device a drain plus the host's wake-up and the next launches (30-45 us of idle device per sync on MI355X,
// measured in the C2 trace); instead one small kernel writes the values straight into host-mapped coherent
// memory, fences, then bumps a sequence word the host spins on.  A fault never publishes: after a few
// microseconds the host also polls the stream, and after 10 s of silence falls back to a stream sync.
static __global__ void k_collect_totals(TotTable t, uint32_t* out) {
    const int i = threadIdx.x;
    if (i < t.count) out[i] = *t.src[i];
}
static __global__ __launch_bounds__(128) void k_publish(TotTable t, const Params* __restrict__ prm, uint32_t* pub, uint32_t seq,
                                                        PubExtra ex) {
    const int i = threadIdx.x;
    if (ex.cap.bad || ex.hpart) {
        if (ex.cap.bad && i < WAVE) {
            const bool over = i < ex.cap.m && *ex.cap.tot[i] > ex.cap.cap[i];
            const uint64_t m = __ballot(over);
            if (i == 0) *ex.cap.bad = m ? 1u : 0u;
        }
        if (ex.hpart && i >= WAVE && i < 2 * WAVE) {
            uint32_t v = 0;
            uint32_t u = 0;
            for (int x = i - WAVE; x < ex.nparts; x += WAVE) { v += ex.hpart[x]; u += ex.hpart[ex.nparts + x]; }
#pragma unroll
            for (int o = WAVE / 2; o > 0; o >>= 1) { v += __shfl_xor(v, o); u += __shfl_xor(u, o); }
            if (i == WAVE) { ex.prm->n_keys_u = v; ex.prm->n_multi = u; }   // heads; multi-entry segments
        }
        __syncthreads();
    }
    if (i < t.count) pub[PUB_TOT + i] = *t.src[i];
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(prm);
    for (int w = i; w < (int)(sizeof(Params) / 4); w += blockDim.x) pub[PUB_PRM + w] = pw[w];
    __syncthreads();
    if (i == 0) {
        __threadfence_system();
        __hip_atomic_store(pub, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
static int pub_ready(ad_handle* h) {
    if (h->pub_host) return AD_OK;
    void* p = nullptr;
    if (hipHostMalloc(&p, PUB_WORDS * 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        return AD_ERR_DEVICE;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
        (void)hipGetLastError();
        hipHostFree(p);
        return AD_ERR_DEVICE;
    }
    std::memset(p, 0, PUB_WORDS * 4);
    h->pub_host = (uint32_t*)p;
    h->pub_dev = (uint32_t*)d;
    return AD_OK;
}
// Two halves so work can be enqueued between the publish and the wait (the speculative finish / merge write):
// publish_totals enqueues the read-back, wait_totals spins on it.
int publish_totals(ad_handle* h, const TotTable& t, uint32_t* host, uint32_t* seq_out, const PubExtra* ex) {
    if (pub_ready(h) != AD_OK) {        // no mapped memory: copy (the wait is a stream sync)
        if (ex && ex->cap.bad) k_cap_check<<<1, 64, 0, h->st>>>(ex->cap);
        if (ex && ex->hpart) k_seg_heads<<<1, SF_PARTS, 0, h->st>>>(ex->hpart, ex->prm, nullptr);
        if (t.count > 0) {
            k_collect_totals<<<1, MAX_TOTALS, 0, h->st>>>(t, h->totd);
            HIPCHK(h, hipMemcpyAsync(host, h->totd, (size_t)t.count * 4, hipMemcpyDeviceToHost, h->st));
        }
        HIPCHK(h, hipMemcpyAsync(&h->hprm, h->prm, sizeof(Params), hipMemcpyDeviceToHost, h->st));
        *seq_out = 0;
        return AD_OK;
    }
    const uint32_t seq = ++h->pub_seq;
    k_publish<<<1, 128, 0, h->st>>>(t, h->prm, h->pub_dev, seq, ex ? *ex : PubExtra{});
    HIPCHK(h, hipGetLastError());
    *seq_out = seq;
    return AD_OK;
}
int wait_totals(ad_handle* h, uint32_t seq, int count, uint32_t* host) {
    if (seq == 0) {
        HIPCHK(h, hipStreamSynchronize(h->st));
        return AD_OK;
    }
    volatile uint32_t* flag = h->pub_host;
    uint64_t spins = 0;
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        if ((++spins & 0x3FF) == 0) {
            const hipError_t q = hipStreamQuery(h->st);
            if (q != hipSuccess && q != hipErrorNotReady) {
                h->err = std::string("stream: ") + hipGetErrorString(q);
                return AD_ERR_DEVICE;
            }
            if (q == hipSuccess && __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) break;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                HIPCHK(h, hipStreamSynchronize(h->st));
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) { h->err = "publish: no result after the stream drained"; return AD_ERR_DEVICE; }
                break;
            }
        }
    }
    if (count > 0) std::memcpy(host, h->pub_host + PUB_TOT, (size_t)count * 4);
    std::memcpy(&h->hprm, h->pub_host + PUB_PRM, sizeof(Params));
    return AD_OK;
}
int read_totals_params(ad_handle* h, const TotTable& t, uint32_t* host) {
    uint32_t seq = 0;
    CK(publish_totals(h, t, host, &seq));
    return wait_totals(h, seq, t.count, host);
}
// the level stage's flag read-backs share the handle's mapped buffer (the totals region)
void set_level_pub(ad_handle* h) {
    if (pub_ready(h) == AD_OK) {
        h->ls.pub.host = h->pub_host; h->ls.pub.dev = h->pub_dev; h->ls.pub.seq = &h->pub_seq;
        h->ls.pub.off = PUB_TOT; h->ls.pub.cap = MAX_TOTALS;
    } else {
        h->ls.pub = Publisher{};
    }
}
int read_params(ad_handle* h) {
    TotTable t{};
    t.count = 0;
    return read_totals_params(h, t, nullptr);
}

int check_params(ad_handle* h) {
    const unsigned e = h->hprm.err;
    if (e & ERR_UNSORTED) return set_err(h, AD_ERR_UNSORTED, "batch TxnIds are not strictly ascending");
    if (e & ERR_KEYORDER) return set_err(h, AD_ERR_ARGUMENT, "a txn's keys must be strictly ascending (Keys), and range txns carry no keys");
    if (e & ERR_RANGEORDER) return set_err(h, AD_ERR_ARGUMENT, "a txn's ranges must be sorted, disjoint, start < end (Ranges), and key txns carry no ranges");
    if (e & ERR_CAP) return set_err(h, AD_ERR_UNSUPPORTED, "more than 8192 dependency entries in one txn's CSR (LDS union capacity)");
    if (e & ERR_EXECBELOW) return set_err(h, AD_ERR_ARGUMENT, "ad_accept_deps: an executeAt below its TxnId is no Accept / GetDeps bound");
    return AD_OK;
}

// ---------------------------------------------------------------------------------------------------
// prepare + sort
// ---------------------------------------------------------------------------------------------------
// The deps stage's small counters (totals words: k_txn_finish's overflow rows + the fused kernel's overflow flag, the
// deferred txns / fill items / heavy hint) and k_seg_fuse's partial sums, zeroed by k_pack's first block: the deps
// stage then needs no fill launch before k_seg_fuse (deps.hip reads small_cleared).
static int pack_clear_list(ad_handle* h, PackPlan& plan) {
    const size_t ntiles = (h->P + SF_TILE - 1) / SF_TILE;
    uint32_t* tile_cnt = nullptr;
    CK(dalloc(h, S_SFCNT, &tile_cnt, 4 * ntiles + 2 * SF_PARTS));
    plan.clr[0] = h->totd + MAX_TOTALS - 7; plan.clr_words[0] = 2;
    plan.clr[1] = h->totd + MAX_TOTALS - 3; plan.clr_words[1] = 3;
    plan.clr[2] = tile_cnt + 4 * ntiles;    plan.clr_words[2] = 2 * SF_PARTS;
    h->small_cleared = true;
    // ad_run_pipeline on a key-only batch whose levels will try the pull pass first: its succ words and flags zeroed
    // here too, so k_seg_fuse can build the chains (stage_deps decides; run_levels then skips k_chain_build)
    const bool pull = h->in_pipeline && h->P > 0 && h->Q == 0 && !h->ls.long_hint && !h->no_fused_chains &&
                      h->level_mode != AD_LEVELS_FIXPOINT && h->level_mode != AD_LEVELS_BLOCKS &&
                      h->level_mode != AD_LEVELS_BLOCKS_WIDE && h->level_mode != AD_LEVELS_KAHN && !h->hist_active;
    if (pull) {
        if (!ls_reserve_chains(h->ls, h->P, h->st)) return set_err(h, AD_ERR_NOMEM, "exec levels: out of device memory");
        plan.clr[3] = h->ls.flags; plan.clr_words[3] = 32;
        plan.succ = h->ls.succ;
        h->chains_pending = true;
    }
    return AD_OK;
}

int stage_prepare(ad_handle* h) {
    const size_t n = h->n, P = h->P, Q = h->Q;
    hipStream_t st = h->st;
    h->pack_enqueued = false;
    h->small_cleared = false;
    h->chains_pending = false;
    h->chains_prebuilt = false;
    // 512 partials: k_minmax_final is a one-workgroup, latency-bound fold (C2: 512 vs 1024 workgroups 0.728 vs 0.733
    // ms/step, three A/B pairs on one box, profiles/r06/minmax_blocks_ab.json); AD_MM_BLOCKS overrides
    static const size_t mm_cap = [] { const char* e = getenv("AD_MM_BLOCKS"); return e ? (size_t)std::max(1, atoi(e)) : (size_t)512; }();
    const int g = (int)std::min<size_t>(mm_cap, std::max<size_t>(1, (std::max(std::max(n, P), Q) + 255) / 256));
    {
        KScope ks(K_MINMAX, n);
        unsigned long long* partial = (unsigned long long*)h->scratch;
        k_minmax<<<g, 256, 0, st>>>(n, h->tm, h->tl, h->tn, h->em, h->el, h->en, h->key_off, h->keys, P, h->range_s, h->range_e, Q, partial);
        if (pub_ready(h) == AD_OK) {
            // the reduce publishes the Params itself: no k_publish launch between it and the host's read; k_pack
            // follows at once and derives its parameters from the device Params (PackPlan), the host reads them
            // while it runs
            const uint32_t seq = ++h->pub_seq;
            k_minmax_final<<<1, MM_FINAL_T, 0, st>>>(g, partial, h->prm, h->pub_dev, h->pub_dev + PUB_PRM, seq);
            if (n > 0) {
                bool uni_small = false;
                const uint32_t nl = h->n_large;
                h->n_large = 0;                                  // the plan as if no large txn: the union view's rule
                deps_class_plan(h, h->want_union, &uni_small);
                h->n_large = nl;
                PackPlan plan{h->prm, (int)h->cfg.replicas + (uni_small ? 1 : 0), (int)h->cfg.replicas, P ? 1 : 0, {}, {}};
                CK(pack_clear_list(h, plan));
                KScope ks(K_PACK, n);
                k_pack<<<ceil_div((long)n, 256), 256, 0, st>>>(n, TsPack{}, 0, h->tm, h->tl, h->tn, h->em, h->el, h->en,
                                                                h->status, h->key_off, h->keys, Q ? h->range_off : nullptr,
                                                                h->range_s, h->range_e, h->tx_ts, h->ex1, h->meta, h->prec,
                                                                h->ka, h->va, h->prm, (uint32_t*)h->cnt8, 0, h->dfr, plan);
                h->pack_enqueued = true;
            }
            CK(wait_totals(h, seq, 0, nullptr));
        } else {
            k_minmax_final<<<1, MM_FINAL_T, 0, st>>>(g, partial, h->prm);
            CK(read_params(h));
        }
    }
    const Params& p = h->hprm;
    if (n == 0) return AD_OK;
    int MB = bits_of(p.msb_max - p.msb_min), HB = bits_of(p.hlc_max - p.hlc_min), NB = bits_of((uint64_t)(p.node_max_b - p.node_min_b));
    if (MB + HB + 4 + NB > 63) return set_err(h, AD_ERR_UNSUPPORTED, "timestamp spread exceeds the 63-bit packed order key");
    h->pack.msb_min = p.msb_min;
    h->pack.hlc_min = p.hlc_min;
    h->pack.node_min = (int64_t)(int32_t)(p.node_min_b ^ 0x80000000u);
    h->pack.sh_flags = NB;
    h->pack.sh_hlc = NB + 4;
    h->pack.sh_msb = NB + 4 + HB;
    h->pack.total_bits = NB + 4 + HB + MB;
    h->key_bits = P ? bits_of(p.key_max - p.key_min) : 0;      // > 32: sorted in two 32-bit LSD halves
    h->n_large = p.n_large;
    h->n_special = p.n_special;
    h->rbase = Q ? p.rs_min : 0;
    h->wmax = Q ? p.rw_max : 0;
    h->range_bits = Q ? bits_of(p.re_max - p.rs_min) : 0;    // > 32: each endpoint sorted in two 32-bit halves
    // the deps stage's count bytes (ncb per pair) and deferred flags are cleared here, in pair / txn order, instead of
    // by a fill launch of their own
    const int ncb = ncb_of(deps_class_plan(h, h->want_union, nullptr));
    h->cnt8_cleared = ncb;
    if (h->pack_enqueued) {                      // k_pack already runs on the device Params (the same plan)
        h->pack_enqueued = false;
        return AD_OK;
    }
    PackPlan plan{};
    CK(pack_clear_list(h, plan));
    KScope ks(K_PACK, n);
    k_pack<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->pack, P ? p.key_min : 0, h->tm, h->tl, h->tn, h->em, h->el, h->en,
                                                    h->status, h->key_off, h->keys, Q ? h->range_off : nullptr, h->range_s,
                                                    h->range_e, h->tx_ts, h->ex1, h->meta, h->prec, h->ka, h->va, h->prm,
                                                    (uint32_t*)h->cnt8, ncb / 4, h->dfr, plan);
    return AD_OK;
}

RadixScratch radix_scratch(ad_handle* h, size_t n) {
    RadixScratch rs;
    const size_t hl = radix_hist_len(n);
    uint8_t* base = (uint8_t*)h->scratch;
    rs.hist = (uint32_t*)base;
    rs.offs = rs.hist + hl + 64;
    rs.agg = rs.offs + hl + 64;
    return rs;
}

int stage_sort(ad_handle* h) {
    const size_t n = h->n, P = h->P, Q = h->Q;
    hipStream_t st = h->st;
    if (P > 0) {
        uint32_t *k = h->ka, *v = h->va, *ko = h->kb, *vo = h->vb;
        if (radix_sort_pairs(k, v, ko, vo, P, std::min(h->key_bits, 32), radix_scratch(h, P), st)) { std::swap(k, ko); std::swap(v, vo); }
        if (h->key_bits > 32) {
            // wide key spread: stable second pass on the high half (LSD over the full 64-bit key)
            k_pair_key_half<<<ceil_div((long)P, 256), 256, 0, st>>>(P, h->keys, v, h->hprm.key_min, 32, k);
            if (radix_sort_pairs(k, v, ko, vo, P, h->key_bits - 32, radix_scratch(h, P), st)) { std::swap(k, ko); std::swap(v, vo); }
        }
        h->skey = k;
        h->sval = v;
    }
    if (Q > 0) {
        // (start, end, owner): stable by end, then stable by start, over the owner-ordered input; each endpoint
        // in one pass, or in two 32-bit halves (low, then high) for a spread beyond 32 bits
        k_range_prep<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->meta, h->range_off, h->range_s, h->range_e, h->rbase,
                                                              h->rowner, h->rk0, h->rv0);
        uint32_t *k = h->rk0, *v = h->rv0, *ko = h->rk1, *vo = h->rv1;
        const int rb = h->range_bits, lo_bits = std::min(rb, 32);
        const int gq = ceil_div((long)Q, 256);
        auto pass = [&](int bits) {
            if (radix_sort_pairs(k, v, ko, vo, Q, bits, radix_scratch(h, Q), st)) { std::swap(k, ko); std::swap(v, vo); }
        };
        if (rb > 32) k_range_key_half<<<gq, 256, 0, st>>>(Q, h->range_e, v, h->rbase, 0, k);
        pass(lo_bits);
        if (rb > 32) { k_range_key_half<<<gq, 256, 0, st>>>(Q, h->range_e, v, h->rbase, 32, k); pass(rb - 32); }
        k_range_key_half<<<gq, 256, 0, st>>>(Q, h->range_s, v, h->rbase, 0, k);
        pass(lo_bits);
        if (rb > 32) { k_range_key_half<<<gq, 256, 0, st>>>(Q, h->range_s, v, h->rbase, 32, k); pass(rb - 32); }
        k_range_gather<<<gq, 256, 0, st>>>(Q, v, h->range_s, h->range_e, h->rowner, h->es, h->ee, h->eown);
    }
    // the interval index over the sorted entries: a 64-ary tree of maximum ends
    RangeIndex ix{};
    size_t nodes = 0;
    ix.top = ri_levels(Q, ix.cnt, &nodes);
    ix.lv[0] = h->ee;
    if (ix.top > 0) {
        CK(dalloc(h, S_RIDX, &h->ri_nodes, nodes));
        size_t off = 0;
        for (int l = 1; l <= ix.top; ++l) {
            uint64_t* out = h->ri_nodes + off;
            k_ri_level<<<ceil_div((long)ix.cnt[l] * WAVE, 256), 256, 0, st>>>(ix.cnt[l], ix.cnt[l - 1], ix.lv[l - 1], out);
            ix.lv[l] = out;
            off += ix.cnt[l];
        }
    }
    h->ix = ix;
    return AD_OK;
}

int fetch_csr(ad_handle* h, const Csr& c, int kw, ad_csr_out* out) {
    const size_t n = h->n;
    hipStream_t st = h->st;
    std::vector<uint32_t> ent(n + 1), cnt(n);
    HIPCHK(h, hipMemcpyAsync(out->key_off, c.key_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
    if (c.nkeys) HIPCHK(h, hipMemcpyAsync(out->keys, c.keys, c.nkeys * 8 * kw, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(out->k2t_off, c.k2t_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
    if (c.nk2t) HIPCHK(h, hipMemcpyAsync(out->k2t, c.k2t, c.nk2t * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(ent.data(), c.ent_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
    if (n) HIPCHK(h, hipMemcpyAsync(cnt.data(), c.tcnt, n * 4, hipMemcpyDeviceToHost, st));
    std::vector<uint32_t> tx(c.ncap);
    if (c.ncap) HIPCHK(h, hipMemcpyAsync(tx.data(), c.txns, c.ncap * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    // compact the per-txn capacity regions (capacity = entries; count = unique TxnIds)
    uint32_t o = 0;
    out->txn_off[0] = 0;
    for (size_t i = 0; i < n; ++i) {
        if (cnt[i]) std::memcpy(out->txns + o, tx.data() + ent[i], cnt[i] * 4);
        o += cnt[i];
        out->txn_off[i + 1] = o;
    }
    return AD_OK;
}

int csr_sizes(ad_handle* h, const Csr& c, ad_csr_sizes* s) {
    s->n = h->n; s->keys = c.nkeys; s->k2t = c.nk2t; s->txn_cap = c.ncap;
    std::vector<uint32_t> cnt(h->n);
    if (h->n && c.ncap) {
        HIPCHK(h, hipMemcpyAsync(cnt.data(), c.tcnt, h->n * 4, hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
    }
    size_t t = 0;
    for (uint32_t x : cnt) t += x;
    s->txns = t;
    return AD_OK;
}

// Rows [lo, hi) of one CSR, offsets rebased to 0 (sizes always; the arrays when out != nullptr).
int fetch_rows(ad_handle* h, const Csr& c, int kw, size_t lo, size_t hi, ad_csr_sizes* s, ad_csr_out* out) {
    hipStream_t st = h->st;
    const size_t m = hi - lo;
    std::vector<uint32_t> ko(m + 1), mo(m + 1), eo(m + 1), cnt(m);
    HIPCHK(h, hipMemcpyAsync(ko.data(), c.key_off + lo, (m + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(mo.data(), c.k2t_off + lo, (m + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(eo.data(), c.ent_off + lo, (m + 1) * 4, hipMemcpyDeviceToHost, st));
    if (m) HIPCHK(h, hipMemcpyAsync(cnt.data(), c.tcnt + lo, m * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    size_t tot = 0;
    for (uint32_t x : cnt) tot += x;
    s->n = m; s->keys = ko[m] - ko[0]; s->k2t = mo[m] - mo[0]; s->txn_cap = eo[m] - eo[0]; s->txns = tot;
    if (!out) return AD_OK;
    for (size_t i = 0; i <= m; ++i) { out->key_off[i] = ko[i] - ko[0]; out->k2t_off[i] = mo[i] - mo[0]; }
    if (s->keys) HIPCHK(h, hipMemcpyAsync(out->keys, c.keys + (size_t)kw * ko[0], s->keys * 8 * kw, hipMemcpyDeviceToHost, st));
    if (s->k2t) HIPCHK(h, hipMemcpyAsync(out->k2t, c.k2t + mo[0], s->k2t * 4, hipMemcpyDeviceToHost, st));
    std::vector<uint32_t> tx(s->txn_cap);
    if (s->txn_cap) HIPCHK(h, hipMemcpyAsync(tx.data(), c.txns + eo[0], s->txn_cap * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    uint32_t o = 0;
    out->txn_off[0] = 0;
    for (size_t i = 0; i < m; ++i) {
        if (cnt[i]) std::memcpy(out->txns + o, tx.data() + (eo[i] - eo[0]), cnt[i] * 4);
        o += cnt[i];
        out->txn_off[i + 1] = o;
    }
    return AD_OK;
}

template <int NV>
void launch_mc(const McArgs& a, hipStream_t st) {
    k_mc_txns<NV><<<ceil_div((long)a.n, 256), 256, 0, st>>>(a);
}
template <int NV>
void launch_mc_ranges(const McRangeArgs& a, hipStream_t st) {
    const int g = ceil_div((long)a.n * WAVE, 256);
    if (a.U > 0) k_mc_range_keys<NV><<<g, 256, 0, st>>>(a);
    k_mc_range_entries<NV><<<g, 256, 0, st>>>(a);
}


// =====================================================================================================
// C-ABI
// =====================================================================================================
// The working buffers of a loaded batch of h->n rows, h->P pairs, h->Q ranges (grow-only slots).
static int load_working(ad_handle* h) {
    const size_t n = h->n, P = h->P, Q = h->Q;
    h->seg_long = false;
    h->keys_partial = false;
    const int nv = (int)h->cfg.replicas, nvc = 2 * nv;
    CK(dalloc(h, S_PRM, &h->prm, 1)); CK(dalloc(h, S_TOT, &h->totd, MAX_TOTALS));
    // a batch merged from host replies (ad_merge_host) never runs stage_prepare: its Params must read clean
    HIPCHK(h, hipMemsetAsync(h->prm, 0, sizeof(Params), h->st));
    CK(dalloc(h, S_TXTS, &h->tx_ts, n)); CK(dalloc(h, S_EX1, &h->ex1, n)); CK(dalloc(h, S_META, &h->meta, n));
    CK(dalloc(h, S_PTXN, &h->prec, P));
    CK(dalloc(h, S_KA, &h->ka, P)); CK(dalloc(h, S_VA, &h->va, P)); CK(dalloc(h, S_KB, &h->kb, P)); CK(dalloc(h, S_VB, &h->vb, P));
    CK(dalloc(h, S_ETXN, &h->e_txn, P)); CK(dalloc(h, S_EMETA, &h->e_meta, P));
    CK(dalloc(h, S_EEXEC, &h->e_exec1, P)); CK(dalloc(h, S_PMW, &h->pm_w, P)); CK(dalloc(h, S_PMC, &h->pm_c, P));
    CK(dalloc(h, S_SEG, &h->seg_start, P)); CK(dalloc(h, S_UD, &h->ud_prev, P));
    CK(dalloc(h, S_UIDX, &h->nh, P)); CK(dalloc(h, S_UKEY, &h->ukey, P)); CK(dalloc(h, S_USEG, &h->useg, P + 1));
    // per-pair / per-txn class words: the R replies' classes plus the union view's (ad_run_pipeline, stage_deps)
    const int nwc = 2 * std::min(nv + 1, MAXV);
    CK(dalloc(h, S_CNT, &h->cnt8, (size_t)ncb_of(nwc) * P)); CK(dalloc(h, S_DST, &h->dst, (size_t)nwc * P));
    CK(dalloc(h, S_CNTX, &h->cntx, (size_t)nwc * P)); CK(dalloc(h, S_INL, &h->inl, (size_t)nwc * P * WALK_INL));
    CK(dalloc(h, S_DFR, &h->dfr, n));
    CK(dalloc(h, S_NK, &h->nk, (size_t)nwc * n + n)); CK(dalloc(h, S_NE, &h->ne, (size_t)nwc * n + n));
    CK(dalloc(h, S_VN, &h->vn, n)); CK(dalloc(h, S_VOFF, &h->voff, n + 1));
    CK(dalloc(h, S_LVL, &h->lvl, n + 1)); CK(dalloc(h, S_ORDER, &h->order, n + 1));
    CK(dalloc(h, S_ROWN, &h->rowner, Q)); CK(dalloc(h, S_RK0, &h->rk0, Q)); CK(dalloc(h, S_RV0, &h->rv0, Q));
    CK(dalloc(h, S_RK1, &h->rk1, Q)); CK(dalloc(h, S_RV1, &h->rv1, Q));
    CK(dalloc(h, S_ES, &h->es, Q)); CK(dalloc(h, S_EE, &h->ee, Q)); CK(dalloc(h, S_EOWN, &h->eown, Q));
    CK(dalloc(h, S_RNK, &h->rnk, (size_t)nv * n)); CK(dalloc(h, S_RNE, &h->rne, (size_t)nv * n));
    const size_t big = std::max(std::max(P, n), Q);
    size_t sc = std::max<size_t>(1 << 20, 3 * (radix_hist_len(big) + 128) * 4 + 64 * 1024);
    sc = std::max(sc, device_scan_scratch<ElideOp>(big) + 4096);
    sc = std::max(sc, level_scratch_bytes(n, P));
    CK(ensure_scratch(h, sc));
    return AD_OK;
}

// ---- asynchronous batch upload (ad_load_batch_async / ad_load_batch_commit): the input SoA of the next batch
// is copied on a copy stream into a second set of input slots while the current batch runs; the commit swaps
// the two sets.  With pinned host buffers (ad_host_alloc) the copies are DMA transfers over PCIe that overlap
// the pipeline and the previous batch's paged-out results.
static const size_t IN_SLOTS[12] = {S_TM, S_TL, S_TN, S_EM, S_EL, S_EN, S_ST, S_KOFF, S_KEYS, S_ROFF, S_RS, S_RE};

static void bind_inputs(ad_handle* h) {
    h->tm = (uint64_t*)h->bufs[S_TM].p; h->tl = (uint64_t*)h->bufs[S_TL].p; h->tn = (int32_t*)h->bufs[S_TN].p;
    h->em = (uint64_t*)h->bufs[S_EM].p; h->el = (uint64_t*)h->bufs[S_EL].p; h->en = (int32_t*)h->bufs[S_EN].p;
    h->status = (uint8_t*)h->bufs[S_ST].p; h->key_off = (uint32_t*)h->bufs[S_KOFF].p; h->keys = (uint64_t*)h->bufs[S_KEYS].p;
    h->range_off = (uint32_t*)h->bufs[S_ROFF].p; h->range_s = (uint64_t*)h->bufs[S_RS].p; h->range_e = (uint64_t*)h->bufs[S_RE].p;
}

extern "C" {

int ad_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

int ad_open(int device, const ad_config* cfg, ad_handle** out) {
    if (!out || !cfg) return AD_ERR_ARGUMENT;
    if (cfg->replicas < 1 || cfg->replicas > (uint32_t)MAXV) return AD_ERR_ARGUMENT;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return AD_ERR_DEVICE;
    if (device < 0 || device >= count) return AD_ERR_ARGUMENT;
    ad_handle* h = new ad_handle();
    h->device = device;
    h->cfg.replicas = cfg->replicas;                  // window 0, no drops: the snapshot (ad_set_replica_model)
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return AD_ERR_DEVICE;
    }
    for (auto& e : h->ev) hipEventCreate(&e);
    h->tracer.st = h->st;
    *out = h;
    return AD_OK;
}

int ad_set_replica_model(ad_handle* h, const ad_replica_model* m) {
    if (!h || !m) return AD_ERR_ARGUMENT;
    if (!(m->drop_p >= 0.0f && m->drop_p <= 1.0f)) return set_err(h, AD_ERR_ARGUMENT, "drop_p outside [0, 1]");
    h->cfg.window = m->window;
    h->cfg.drop_p = m->drop_p;
    h->cfg.seed = m->seed;
    return AD_OK;
}

void ad_close(ad_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->comm) ncclCommDestroy(h->comm);
    if (h->st) hipStreamSynchronize(h->st);
    if (h->cst) { hipStreamSynchronize(h->cst); hipStreamDestroy(h->cst); }
    if (h->xst) { hipStreamSynchronize(h->xst); hipStreamDestroy(h->xst); }
    if (h->fst) { hipStreamSynchronize(h->fst); hipStreamDestroy(h->fst); }
    if (h->fev0) hipEventDestroy(h->fev0);
    if (h->fev1) hipEventDestroy(h->fev1);
    if (h->xev0) hipEventDestroy(h->xev0);
    if (h->xev1) hipEventDestroy(h->xev1);
    if (h->cev) hipEventDestroy(h->cev);
    if (h->sev) hipEventDestroy(h->sev);
    if (h->pub_host) hipHostFree(h->pub_host);
    for (auto& b : h->bufs) if (b.p) hipFree(b.p);
    for (auto& e : h->ev) if (e) hipEventDestroy(e);
    free_level_state(h->ls);
    if (h->st) hipStreamDestroy(h->st);
    delete h;
}

const char* ad_last_error(const ad_handle* h) { return h ? h->err.c_str() : "null handle"; }

int ad_load_batch(ad_handle* h, const ad_batch* b) {
    if (!h || !b) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    const size_t nb = b->n;
    if (nb >= (1ull << 31)) return set_err(h, AD_ERR_ARGUMENT, "batch too large");
    const size_t Pb = nb ? b->key_off[nb] : 0;
    const size_t Q = (nb && b->range_off) ? b->range_off[nb] : 0;
    if (Pb >= (1ull << 31) || Q >= (1ull << 31)) return set_err(h, AD_ERR_ARGUMENT, "batch too large");
    // CFK history from the previous batch (ad_cfk_retain): its kept rows go first, then the new txns
    const bool hist = h->hist_valid;
    if (hist && Q) return set_err(h, AD_ERR_UNSUPPORTED, "CFK history: key batches only (no range txns)");
    if (hist && h->sharded) return set_err(h, AD_ERR_UNSUPPORTED, "CFK history: not in sharded mode");
    const size_t H = hist ? h->hist_n : 0, HP = hist ? h->hist_p : 0;
    const size_t n = H + nb, P = HP + Pb;
    if (n >= (1ull << 31) || P >= (1ull << 31)) return set_err(h, AD_ERR_ARGUMENT, "batch too large");
    h->n = n; h->P = P; h->Q = Q;
    h->loaded = false;
    h->have_deps = h->have_merged = h->have_levels = false;
    h->mc_ready = false;
    h->mc_fast = nullptr;
    h->rc_ready = false;
    h->hist_active = hist;
    h->hist_rows = H;
    h->hist_valid = false;           // consumed: ad_cfk_retain on this batch carries the state on
    CK(dalloc(h, S_TM, &h->tm, n)); CK(dalloc(h, S_TL, &h->tl, n)); CK(dalloc(h, S_TN, &h->tn, n));
    CK(dalloc(h, S_EM, &h->em, n)); CK(dalloc(h, S_EL, &h->el, n)); CK(dalloc(h, S_EN, &h->en, n));
    CK(dalloc(h, S_ST, &h->status, n)); CK(dalloc(h, S_KOFF, &h->key_off, n + 1)); CK(dalloc(h, S_KEYS, &h->keys, P));
    CK(dalloc(h, S_ROFF, &h->range_off, n + 1)); CK(dalloc(h, S_RS, &h->range_s, Q)); CK(dalloc(h, S_RE, &h->range_e, Q));
    hipStream_t st = h->st;
    if (H) {
        auto d2d = [&](void* dst, size_t slot, size_t bytes) {
            return hipMemcpyAsync(dst, h->bufs[slot].p, bytes, hipMemcpyDeviceToDevice, st);
        };
        HIPCHK(h, d2d(h->tm, S_HTM, H * 8)); HIPCHK(h, d2d(h->tl, S_HTL, H * 8)); HIPCHK(h, d2d(h->tn, S_HTN, H * 4));
        HIPCHK(h, d2d(h->em, S_HEM, H * 8)); HIPCHK(h, d2d(h->el, S_HEL, H * 8)); HIPCHK(h, d2d(h->en, S_HEN, H * 4));
        HIPCHK(h, d2d(h->status, S_HST, H)); HIPCHK(h, d2d(h->key_off, S_HKOFF, H * 4));
        if (HP) HIPCHK(h, d2d(h->keys, S_HKEYS, HP * 8));
    }
    if (nb) {
        HIPCHK(h, hipMemcpyAsync(h->tm + H, b->txn_msb, nb * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->tl + H, b->txn_lsb, nb * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->tn + H, b->txn_node, nb * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->em + H, b->exec_msb, nb * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->el + H, b->exec_lsb, nb * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->en + H, b->exec_node, nb * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->status + H, b->status, nb, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->key_off + H, b->key_off, (nb + 1) * 4, hipMemcpyHostToDevice, st));
        if (Pb) HIPCHK(h, hipMemcpyAsync(h->keys + HP, b->keys, Pb * 8, hipMemcpyHostToDevice, st));
    } else if (!H) {
        HIPCHK(h, hipMemsetAsync(h->key_off, 0, 4, st));
    } else {
        const uint32_t end = (uint32_t)HP;                                           // empty batch: end offset
        HIPCHK(h, hipMemcpyAsync(h->key_off + H, &end, 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    if (hist) {
        // global arrival ranks: the kept rows' own, then next + i; the new key offsets follow the kept keys
        CK(dalloc(h, S_GID, &h->gid, std::max<size_t>(n, 1)));
        if (H) HIPCHK(h, hipMemcpyAsync(h->gid, h->bufs[S_HGIDS].p, H * 4, hipMemcpyDeviceToDevice, st));
        if (nb) k_hist_new_rows<<<ceil_div((long)nb + 1, 256), 256, 0, st>>>(H, nb, h->hist_next, (uint32_t)HP, h->gid, h->key_off);
        HIPCHK(h, hipGetLastError());
    }
    if (Q) {
        HIPCHK(h, hipMemcpyAsync(h->range_off, b->range_off, (n + 1) * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->range_s, b->range_start, Q * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->range_e, b->range_end, Q * 8, hipMemcpyHostToDevice, st));
    } else {
        HIPCHK(h, hipMemsetAsync(h->range_off, 0, (n + 1) * 4, st));
    }
    CK(load_working(h));
    HIPCHK(h, hipStreamSynchronize(st));
    h->loaded = true;
    h->gq_ready = false;
    return AD_OK;
}

int ad_load_batch_async(ad_handle* h, const ad_batch* b) {
    if (!h || !b) return AD_ERR_ARGUMENT;
    if (h->hist_valid) return set_err(h, AD_ERR_UNSUPPORTED, "ad_load_batch_async: the next batch carries CFK history (ad_load_batch)");
    if (h->stage_pending) return set_err(h, AD_ERR_STATE, "ad_load_batch_async: commit the staged batch first");
    hipSetDevice(h->device);
    const size_t n = b->n;
    if (n >= (1ull << 31)) return set_err(h, AD_ERR_ARGUMENT, "batch too large");
    const size_t P = n ? b->key_off[n] : 0;
    const size_t Q = (n && b->range_off) ? b->range_off[n] : 0;
    if (P >= (1ull << 31) || Q >= (1ull << 31)) return set_err(h, AD_ERR_ARGUMENT, "batch too large");
    if (!h->cst) {
        HIPCHK(h, hipStreamCreateWithFlags(&h->cst, hipStreamNonBlocking));
        HIPCHK(h, hipEventCreateWithFlags(&h->cev, hipEventDisableTiming));
        HIPCHK(h, hipEventCreateWithFlags(&h->sev, hipEventDisableTiming));
    }
    const size_t cnt[12] = {n * 8, n * 8, n * 4, n * 8, n * 8, n * 4, n, (n + 1) * 4, P * 8, (n + 1) * 4, Q * 8, Q * 8};
    uint8_t* d[12];
    for (int k = 0; k < 12; ++k) CK(dalloc(h, S_STG0 + k, &d[k], cnt[k]));
    // the staging slots held an earlier batch: copy only after the handle's stream is past its last use
    HIPCHK(h, hipEventRecord(h->sev, h->st));
    HIPCHK(h, hipStreamWaitEvent(h->cst, h->sev, 0));
    const void* src[12] = {b->txn_msb, b->txn_lsb, b->txn_node, b->exec_msb, b->exec_lsb, b->exec_node, b->status,
                           b->key_off, b->keys, b->range_off, b->range_start, b->range_end};
    for (int k = 0; k < 12; ++k) {
        if (k == 9 && !Q) { HIPCHK(h, hipMemsetAsync(d[k], 0, (n + 1) * 4, h->cst)); continue; }
        if (k == 7 && !n) { HIPCHK(h, hipMemsetAsync(d[k], 0, 4, h->cst)); continue; }
        if (cnt[k] && src[k]) HIPCHK(h, hipMemcpyAsync(d[k], src[k], cnt[k], hipMemcpyHostToDevice, h->cst));
    }
    HIPCHK(h, hipEventRecord(h->cev, h->cst));
    h->stg_n = n; h->stg_p = P; h->stg_q = Q;
    h->stage_pending = true;
    return AD_OK;
}

int ad_load_batch_commit(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    if (!h->stage_pending) return set_err(h, AD_ERR_STATE, "ad_load_batch_commit: no staged batch (ad_load_batch_async)");
    hipSetDevice(h->device);
    HIPCHK(h, hipEventSynchronize(h->cev));          // the host batch may be reused once this returns
    // checked before the staged batch is consumed: after ad_cfk_reset the caller can commit it again
    if (h->hist_valid) return set_err(h, AD_ERR_UNSUPPORTED, "ad_load_batch_commit: CFK history was retained after the async load (ad_cfk_reset, or ad_load_batch)");
    h->stage_pending = false;
    for (int k = 0; k < 12; ++k) std::swap(h->bufs[IN_SLOTS[k]], h->bufs[S_STG0 + k]);
    bind_inputs(h);
    h->n = h->stg_n; h->P = h->stg_p; h->Q = h->stg_q;
    h->loaded = false;
    h->have_deps = h->have_merged = h->have_levels = false;
    h->mc_ready = false;
    h->mc_fast = nullptr;
    h->rc_ready = false;
    h->hist_active = false;
    h->hist_rows = 0;
    CK(load_working(h));
    h->loaded = true;
    h->gq_ready = false;
    return AD_OK;
}

void* ad_host_alloc(size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, std::max<size_t>(bytes, 64), hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return p;
}

void ad_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

static int run_deps(ad_handle* h, ad_csr_sizes* sizes, bool accept, bool bound_max = false) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "no batch loaded");
    if (accept && h->sharded) {
        // the window sits at the bound's global arrival position (ad_shard_query_positions); Timestamp.MAX: after
        // every arrival of the global batch
        CK(dalloc(h, S_GQPOS, &h->gqpos, std::max<size_t>(h->n, 1)));
        if (bound_max) {
            if (h->n) HIPCHK(h, hipMemsetD32Async(h->gqpos, (int)h->n_global, h->n, h->st));
        } else if (!h->gq_ready) {
            return set_err(h, AD_ERR_STATE, "ad_accept_deps on a sharded store: ad_shard_query_positions first");
        }
    }
    if (accept && h->hist_active) return set_err(h, AD_ERR_UNSUPPORTED, "ad_accept_deps: not over a CFK history batch");
    hipSetDevice(h->device);
    h->accept = accept;
    h->bound_max = bound_max;
    int rc = stage_prepare(h);
    if (rc == AD_OK) rc = stage_sort(h);
    if (rc == AD_OK) rc = stage_deps(h);
    h->accept = false;
    h->bound_max = false;
    CK(rc);
    CK(read_params(h));
    CK(check_params(h));
    if (sizes) {
        const int nv = (int)h->cfg.replicas;
        for (int v = 0; v < nv; ++v) {
            CK(csr_sizes(h, h->deps[2 * v], &sizes[v * AD_NUM_CLASSES + 0]));
            CK(csr_sizes(h, h->deps[2 * v + 1], &sizes[v * AD_NUM_CLASSES + 1]));
            if (h->Q) CK(csr_sizes(h, h->rdeps[v], &sizes[v * AD_NUM_CLASSES + 2]));
            else sizes[v * AD_NUM_CLASSES + 2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
        }
    }
    return AD_OK;
}

int ad_preaccept_deps(ad_handle* h, ad_csr_sizes* sizes) { return run_deps(h, sizes, false); }
int ad_accept_deps(ad_handle* h, ad_csr_sizes* sizes) { return run_deps(h, sizes, true); }
int ad_ephemeral_read_deps(ad_handle* h, ad_csr_sizes* sizes) { return run_deps(h, sizes, true, true); }

extern "C++" {
int fetch_empty(ad_handle* h, ad_csr_out* out) {
    for (size_t i = 0; i <= h->n; ++i) { out->key_off[i] = 0; out->k2t_off[i] = 0; out->txn_off[i] = 0; }
    return AD_OK;
}
}

// CommandStore.preaccept's maxConflicts.get(keys) per view (conflict_kernels.h), over the sorted entries the
// deps stage left on the device: leaves max_rank / fast (and the batch-local rank) in their slots.
// CommandStore.preaccept around maxConflicts.get (conflict_kernels.h k_preaccept_rules): ExclusiveSyncPoints answer
// their TxnId, expired txns (timeout / rejectBefore) are rejected
static void apply_preaccept_rules(ad_handle* h, uint8_t* fast) {
    if (!h->n) return;
    PreacceptRules r{};
    r.n = h->n; r.nv = (int)h->cfg.replicas; r.key_off = h->key_off; r.keys = h->keys;
    if (h->Q > 0) { r.range_off = h->range_off; r.rs = h->range_s; r.re = h->range_e; }
    r.tm = h->tm; r.tl = h->tl; r.tn = h->tn;
    r.rb = McIntervals{h->rb_m, h->rb_s, h->rb_e, h->rb_cm, h->rb_cl, h->rb_cn};
    r.clock = h->rb_clock; r.now_hlc = h->rb_now; r.timeout = h->rb_timeout;
    r.fast = fast;
    k_preaccept_rules<<<ceil_div((long)h->n, 256), 256, 0, h->st>>>(r);
}

static int run_max_conflicts(ad_handle* h, uint32_t** rank_out, uint8_t** fast_out, uint32_t** local_out) {
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "no deps computed");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    CK(complete_entries(h));
    const size_t n = h->n, P = h->P;
    const int nv = (int)h->cfg.replicas;
    hipStream_t st = h->st;
    McArgs a{};
    a.n = n; a.P = P;
    a.e_txn = h->e_txn; a.e_meta = h->e_meta; a.e_exec1 = h->e_exec1; a.seg_start = h->seg_start;
    a.gid = (h->sharded || h->hist_active) ? h->gid : nullptr;
    a.window = h->cfg.window; a.thresh = ad_drop_threshold(h->cfg.drop_p); a.seed = h->cfg.seed;
    a.key_off = h->key_off; a.tx_ts = h->tx_ts;
    uint64_t* pm_e = nullptr;
    uint32_t *pm_r = nullptr, *inv = nullptr, *rank = nullptr, *local = nullptr;
    uint8_t* fst = nullptr;
    CK(dalloc(h, S_MCPE, &pm_e, std::max<size_t>(P, 1))); CK(dalloc(h, S_MCPR, &pm_r, std::max<size_t>(P, 1)));
    CK(dalloc(h, S_MCINV, &inv, std::max<size_t>(P, 1)));
    CK(dalloc(h, S_MCRANK, &rank, std::max<size_t>(n * nv, 1))); CK(dalloc(h, S_MCFAST, &fst, std::max<size_t>(n * nv, 1)));
    // sharded stores with range txns: the range kernels fold local rows, globalised afterwards
    const bool fold_local = h->Q > 0 && a.gid != nullptr;
    if (local_out || fold_local) CK(dalloc(h, S_MCLOCAL, &local, std::max<size_t>(n * nv, 1)));
    a.pm_e = pm_e; a.pm_r = pm_r; a.inv = inv; a.max_rank = rank; a.fast = fst; a.local_rank = local;
    if (P > 0) CK(ensure_scratch(h, std::max(h->scratch_cap, device_scan_scratch<MaxConflictOp>(P))));
    if (n > 0) {
        KScope ks(K_MAX_CONFLICTS, P);      // scan (+ inverse permutation) + per-txn walk and fold
        if (P > 0) {
            MaxConflictOp op{h->seg_start, h->e_meta, h->e_exec1, h->e_txn, h->sval, pm_e, pm_r, inv};
            scan_any(h, op, P);
        }
        NV_DISPATCH(nv, launch_mc, a, st);
        if (h->Q > 0) {
            // range footprints: range txns' CFK keys, and every txn against the range entries
            McRangeArgs ra{};
            ra.n = n; ra.meta = h->meta; ra.ex1 = h->ex1; ra.tx_ts = h->tx_ts; ra.key_off = h->key_off; ra.keys = h->keys;
            ra.range_off = h->range_off; ra.rs = h->range_s; ra.re = h->range_e;
            ra.ukey = h->ukey; ra.useg = h->useg; ra.U = P ? h->hprm.n_keys_u : 0;
            ra.e_txn = h->e_txn; ra.e_meta = h->e_meta; ra.e_exec1 = h->e_exec1; ra.pm_e = pm_e; ra.pm_r = pm_r;
            ra.Q = h->Q; ra.es = h->es; ra.ee = h->ee; ra.eown = h->eown; ra.ix = h->ix;
            ra.window = a.window; ra.thresh = a.thresh; ra.seed = a.seed; ra.fast = fst;
            ra.gid = a.gid;
            ra.max_rank = fold_local ? local : rank;
            NV_DISPATCH(nv, launch_mc_ranges, ra, st);
            if (fold_local)
                k_mc_globalize<<<ceil_div((long)(n * nv), 256), 256, 0, st>>>(n * nv, local, a.gid, rank);
        }
    }
    apply_preaccept_rules(h, fst);
    HIPCHK(h, hipGetLastError());
    h->mc_ready = true;
    h->mc_fast = fst;
    *rank_out = rank; *fast_out = fst;
    if (local_out) *local_out = local;
    return AD_OK;
}

int ad_max_conflicts(ad_handle* h, uint32_t* max_rank, uint8_t* fast) {
    if (!h) return AD_ERR_ARGUMENT;
    uint32_t* rank = nullptr;
    uint8_t* fst = nullptr;
    CK(run_max_conflicts(h, &rank, &fst, nullptr));
    const size_t n = h->n, nv = h->cfg.replicas;
    hipStream_t st = h->st;
    if (max_rank && n) HIPCHK(h, hipMemcpyAsync(max_rank, rank, n * nv * 4, hipMemcpyDeviceToHost, st));
    if (fast && n) HIPCHK(h, hipMemcpyAsync(fast, fst, n * nv, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    h->tracer.resolve();
    return AD_OK;
}

int ad_max_conflicts_carry(ad_handle* h, size_t m, const uint64_t* keys, const uint64_t* msb, const uint64_t* lsb,
                           const int32_t* node) {
    if (!h || (m && (!keys || !msb || !lsb || !node))) return AD_ERR_ARGUMENT;
    for (size_t i = 1; i < m; ++i)
        if (keys[i] <= keys[i - 1]) return set_err(h, AD_ERR_ARGUMENT, "carried MaxConflicts keys must be strictly ascending");
    hipSetDevice(h->device);
    CK(dalloc(h, S_MCCK, &h->mc_ck, std::max<size_t>(m, 1))); CK(dalloc(h, S_MCCM, &h->mc_cm, std::max<size_t>(m, 1)));
    CK(dalloc(h, S_MCCL, &h->mc_cl, std::max<size_t>(m, 1))); CK(dalloc(h, S_MCCN, &h->mc_cn, std::max<size_t>(m, 1)));
    if (m) {
        HIPCHK(h, hipMemcpyAsync(h->mc_ck, keys, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->mc_cm, msb, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->mc_cl, lsb, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->mc_cn, node, m * 4, hipMemcpyHostToDevice, h->st));
    }
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->mc_m = m;
    return AD_OK;
}

int ad_max_conflicts_carry_ranges(ad_handle* h, size_t m, const uint64_t* starts, const uint64_t* ends, const uint64_t* msb,
                                  const uint64_t* lsb, const int32_t* node) {
    if (!h || (m && (!starts || !ends || !msb || !lsb || !node))) return AD_ERR_ARGUMENT;
    for (size_t i = 0; i < m; ++i) {
        if (!(starts[i] < ends[i])) return set_err(h, AD_ERR_ARGUMENT, "carried MaxConflicts intervals need start < end");
        if (i && starts[i] < ends[i - 1])
            return set_err(h, AD_ERR_ARGUMENT, "carried MaxConflicts intervals must be sorted and disjoint");
    }
    hipSetDevice(h->device);
    const size_t c = std::max<size_t>(m, 1);
    CK(dalloc(h, S_MCIS, &h->mci_s, c)); CK(dalloc(h, S_MCIE, &h->mci_e, c)); CK(dalloc(h, S_MCIM, &h->mci_cm, c));
    CK(dalloc(h, S_MCIL, &h->mci_cl, c)); CK(dalloc(h, S_MCIN, &h->mci_cn, c));
    if (m) {
        HIPCHK(h, hipMemcpyAsync(h->mci_s, starts, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->mci_e, ends, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->mci_cm, msb, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->mci_cl, lsb, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->mci_cn, node, m * 4, hipMemcpyHostToDevice, h->st));
    }
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->mci_m = m;
    h->mci_lo = m ? starts[0] : 0;
    h->mci_hi = m ? ends[m - 1] : 0;
    return AD_OK;
}

int ad_preaccept_expiry(ad_handle* h, uint64_t now_hlc, uint64_t pre_accept_timeout, size_t m, const uint64_t* starts,
                        const uint64_t* ends, const uint64_t* msb, const uint64_t* lsb, const int32_t* node) {
    if (!h || (m && (!starts || !ends || !msb || !lsb || !node))) return AD_ERR_ARGUMENT;
    for (size_t i = 0; i < m; ++i) {
        if (!(starts[i] < ends[i])) return set_err(h, AD_ERR_ARGUMENT, "rejectBefore intervals need start < end");
        if (i && starts[i] < ends[i - 1]) return set_err(h, AD_ERR_ARGUMENT, "rejectBefore intervals must be sorted and disjoint");
    }
    hipSetDevice(h->device);
    const size_t c = std::max<size_t>(m, 1);
    CK(dalloc(h, S_RBS, &h->rb_s, c)); CK(dalloc(h, S_RBE, &h->rb_e, c)); CK(dalloc(h, S_RBM, &h->rb_cm, c));
    CK(dalloc(h, S_RBL, &h->rb_cl, c)); CK(dalloc(h, S_RBN, &h->rb_cn, c));
    if (m) {
        HIPCHK(h, hipMemcpyAsync(h->rb_s, starts, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->rb_e, ends, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->rb_cm, msb, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->rb_cl, lsb, m * 8, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipMemcpyAsync(h->rb_cn, node, m * 4, hipMemcpyHostToDevice, h->st));
    }
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->rb_m = m;
    h->rb_clock = pre_accept_timeout != AD_NO_TIMEOUT;
    h->rb_now = now_hlc;
    h->rb_timeout = pre_accept_timeout;
    return AD_OK;
}

int ad_max_conflicts_ts(ad_handle* h, uint64_t* msb, uint64_t* lsb, int32_t* node, uint8_t* fast) {
    if (!h) return AD_ERR_ARGUMENT;
    uint32_t *rank = nullptr, *local = nullptr;
    uint8_t* fst = nullptr;
    CK(run_max_conflicts(h, &rank, &fst, &local));
    const size_t n = h->n, nv = h->cfg.replicas;
    hipStream_t st = h->st;
    uint64_t *om = nullptr, *ol = nullptr;
    int32_t* on = nullptr;
    uint8_t* of = nullptr;
    CK(dalloc(h, S_MCOM, &om, std::max<size_t>(n * nv, 1))); CK(dalloc(h, S_MCOL, &ol, std::max<size_t>(n * nv, 1)));
    CK(dalloc(h, S_MCON, &on, std::max<size_t>(n * nv, 1))); CK(dalloc(h, S_MCOF, &of, std::max<size_t>(n * nv, 1)));
    if (n) {
        McCarryArgs c{};
        c.n = n; c.nv = (int)nv; c.key_off = h->key_off; c.keys = h->keys;
        c.tm = h->tm; c.tl = h->tl; c.tn = h->tn; c.em = h->em; c.el = h->el; c.en = h->en;
        // the batch row holding each answer: the range fold updates `local` only on sharded / history batches
        const bool gid = h->sharded || h->hist_active;
        c.local_rank = (gid || h->Q == 0) ? local : rank;
        if (h->Q > 0) { c.range_off = h->range_off; c.rs = h->range_s; c.re = h->range_e; }
        c.iv = McIntervals{h->mci_m, h->mci_s, h->mci_e, h->mci_cm, h->mci_cl, h->mci_cn};
        c.m = h->mc_m; c.ck = h->mc_ck; c.cm = h->mc_cm; c.cl = h->mc_cl; c.cn = h->mc_cn;
        c.om = om; c.ol = ol; c.on = on; c.fast = of;
        KScope ks(K_MAX_CONFLICTS);
        k_mc_carry<<<ceil_div((long)n, 256), 256, 0, st>>>(c);
        apply_preaccept_rules(h, of);
        HIPCHK(h, hipGetLastError());
        h->mc_fast = of;
        if (msb) HIPCHK(h, hipMemcpyAsync(msb, om, n * nv * 8, hipMemcpyDeviceToHost, st));
        if (lsb) HIPCHK(h, hipMemcpyAsync(lsb, ol, n * nv * 8, hipMemcpyDeviceToHost, st));
        if (node) HIPCHK(h, hipMemcpyAsync(node, on, n * nv * 4, hipMemcpyDeviceToHost, st));
        if (fast) HIPCHK(h, hipMemcpyAsync(fast, of, n * nv, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    h->tracer.resolve();
    return AD_OK;
}

int ad_max_conflicts_export(ad_handle* h, size_t* m_out, uint64_t* keys, uint64_t* msb, uint64_t* lsb, int32_t* node) {
    if (!h || !m_out) return AD_ERR_ARGUMENT;
    if (!h->mc_ready) return set_err(h, AD_ERR_STATE, "ad_max_conflicts_export: run ad_max_conflicts(_ts) on this batch first");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const uint32_t U = h->P ? h->hprm.n_keys_u : 0;
    const size_t S = (size_t)U + h->mc_m;
    uint64_t *sk, *sm, *sl, *ok_, *om_, *ol_;
    int32_t *sn, *on_;
    uint8_t* su;
    uint32_t *sp, *tot;
    CK(dalloc(h, S_MCSK, &sk, std::max<size_t>(S, 1))); CK(dalloc(h, S_MCSM, &sm, std::max<size_t>(S, 1)));
    CK(dalloc(h, S_MCSL, &sl, std::max<size_t>(S, 1))); CK(dalloc(h, S_MCSN, &sn, std::max<size_t>(S, 1)));
    CK(dalloc(h, S_MCSU, &su, std::max<size_t>(S, 1))); CK(dalloc(h, S_MCSP, &sp, std::max<size_t>(S, 1) + 16));
    CK(dalloc(h, S_MCEK, &ok_, std::max<size_t>(S, 1))); CK(dalloc(h, S_MCEM, &om_, std::max<size_t>(S, 1)));
    CK(dalloc(h, S_MCEN, &on_, std::max<size_t>(S, 1))); CK(dalloc(h, S_MCEL, &ol_, std::max<size_t>(S, 1)));
    tot = sp + std::max<size_t>(S, 1);
    uint32_t count = 0;
    if (S) {
        HIPCHK(h, hipMemsetAsync(su, 0, S, st));
        k_mc_export_slots<<<ceil_div((long)S, 256), 256, 0, st>>>(U, h->ukey, h->useg, (const uint64_t*)h->bufs[S_MCPE].p,
                                                                   (const uint32_t*)h->bufs[S_MCPR].p, h->em, h->el, h->en,
                                                                   h->mc_m, h->mc_ck, h->mc_cm, h->mc_cl, h->mc_cn, sk, sm, sl, sn, su);
        CK(ensure_scratch(h, std::max(h->scratch_cap, device_scan_scratch<CompactFlagOp>(S))));
        device_scan(CompactFlagOp{su, sp, tot, S}, S, (uint32_t*)h->scratch, st);
        HIPCHK(h, hipMemcpyAsync(&count, tot, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
    }
    *m_out = count;
    if (!keys) return AD_OK;
    if (count) {
        // CompactFlagOp wrote out[rank] = slot: gather the used slots in order
        k_mc_export_gather<<<ceil_div((long)count, 256), 256, 0, st>>>(count, sp, sk, sm, sl, sn, ok_, om_, ol_, on_);
        HIPCHK(h, hipMemcpyAsync(keys, ok_, count * 8, hipMemcpyDeviceToHost, st));
        if (msb) HIPCHK(h, hipMemcpyAsync(msb, om_, count * 8, hipMemcpyDeviceToHost, st));
        if (lsb) HIPCHK(h, hipMemcpyAsync(lsb, ol_, count * 8, hipMemcpyDeviceToHost, st));
        if (node) HIPCHK(h, hipMemcpyAsync(node, on_, count * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    return AD_OK;
}

// The interval part of the map after the batch (conflict_kernels.h k_mci_*): breakpoints of the carried intervals and
// the batch's range entries, LSD-sorted and made unique; per elementary segment the max of what contains it; runs
// of one value compacted into pieces.  Two calls as ad_max_conflicts_export (starts == NULL: *m only).
int ad_max_conflicts_export_ranges(ad_handle* h, size_t* m_out, uint64_t* starts, uint64_t* ends, uint64_t* msb,
                                   uint64_t* lsb, int32_t* node) {
    if (!h || !m_out) return AD_ERR_ARGUMENT;
    if (!h->mc_ready) return set_err(h, AD_ERR_STATE, "ad_max_conflicts_export_ranges: run ad_max_conflicts(_ts) on this batch first");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    hipStream_t st = h->st;
    const size_t mi = h->mci_m, Q = h->Q, N = 2 * (mi + Q);
    *m_out = 0;
    if (N == 0) return AD_OK;
    if (N >= (1ull << 31)) return set_err(h, AD_ERR_UNSUPPORTED, "ad_max_conflicts_export_ranges: too many intervals");
    // breakpoint spread: carried [mci_lo, mci_hi], batch [rbase, rbase + 2^range_bits)
    uint64_t lo = ~0ull, hi = 0;
    if (mi) { lo = std::min<uint64_t>(lo, h->mci_lo); hi = std::max<uint64_t>(hi, h->mci_hi); }
    if (Q) {
        lo = std::min<uint64_t>(lo, h->rbase);
        const uint64_t span = h->range_bits >= 64 ? ~0ull : ((1ull << h->range_bits) - 1);
        hi = std::max<uint64_t>(hi, h->rbase + std::min<uint64_t>(span, ~0ull - h->rbase));
    }
    int bits = 0;
    for (uint64_t d = hi - lo; d; d >>= 1) ++bits;
    const size_t c = N + 16;
    uint64_t *x, *xu, *vm, *vl, *os, *oe, *om, *ol;
    uint32_t *k0, *v0, *k1, *v1, *rows, *ps, *pe;
    int32_t *vn, *on;
    uint8_t *fl, *has, *fs, *fe;
    CK(dalloc(h, S_MXX, &x, c)); CK(dalloc(h, S_MXK0, &k0, c)); CK(dalloc(h, S_MXV0, &v0, c)); CK(dalloc(h, S_MXK1, &k1, c));
    CK(dalloc(h, S_MXV1, &v1, c)); CK(dalloc(h, S_MXF, &fl, c)); CK(dalloc(h, S_MXR, &rows, c + 1)); CK(dalloc(h, S_MXU, &xu, c));
    CK(dalloc(h, S_MXVM, &vm, c)); CK(dalloc(h, S_MXVL, &vl, c)); CK(dalloc(h, S_MXVN, &vn, c)); CK(dalloc(h, S_MXH, &has, c));
    CK(dalloc(h, S_MXFS, &fs, c)); CK(dalloc(h, S_MXFE, &fe, c)); CK(dalloc(h, S_MXPS, &ps, c + 1)); CK(dalloc(h, S_MXPE, &pe, c + 1));
    CK(dalloc(h, S_MXOS, &os, c)); CK(dalloc(h, S_MXOE, &oe, c)); CK(dalloc(h, S_MXOM, &om, c)); CK(dalloc(h, S_MXOL, &ol, c));
    CK(dalloc(h, S_MXON, &on, c));
    CK(ensure_scratch(h, std::max(h->scratch_cap, std::max((size_t)(3 * (radix_hist_len(N) + 128) + 64 * 1024) * 4,
                                                           device_scan_scratch<CompactFlagOp>(N)))));
    const int gN = ceil_div((long)N, 256);
    uint32_t S = 0, cnt = 0;
    {
        KScope ks(K_MAX_CONFLICTS, N);
        k_mci_points<<<gN, 256, 0, st>>>(mi, h->mci_s, h->mci_e, Q, h->es, h->ee, lo, x, k0, v0);
        uint32_t *k = k0, *v = v0, *ko = k1, *vo = v1;
        if (radix_sort_pairs(k, v, ko, vo, N, std::min(bits, 32), radix_scratch(h, N), st)) { std::swap(k, ko); std::swap(v, vo); }
        if (bits > 32) {
            k_mci_hi<<<gN, 256, 0, st>>>(N, x, v, lo, k);
            if (radix_sort_pairs(k, v, ko, vo, N, bits - 32, radix_scratch(h, N), st)) { std::swap(k, ko); std::swap(v, vo); }
        }
        k_mci_unique<<<gN, 256, 0, st>>>(N, x, v, fl);
        device_scan(CompactFlagOp{fl, rows, rows + c, N}, N, (uint32_t*)h->scratch, st);
        HIPCHK(h, hipMemcpyAsync(&S, rows + c, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        if (S >= 2) {
            const uint32_t nseg = S - 1;
            k_mci_gather_points<<<ceil_div((long)S, 256), 256, 0, st>>>(S, rows, x, v, xu);
            MciSegArgs a{};
            a.S = S; a.xu = xu;
            a.iv = McIntervals{mi, h->mci_s, h->mci_e, h->mci_cm, h->mci_cl, h->mci_cn};
            a.Q = Q; a.es = h->es; a.ee = h->ee; a.eown = h->eown; a.ix = h->ix; a.meta = h->meta;
            a.em = h->em; a.el = h->el; a.en = h->en;
            a.vm = vm; a.vl = vl; a.vn = vn; a.has = has;
            k_mci_segments<<<ceil_div((long)nseg * WAVE, 256), 256, 0, st>>>(a);
            k_mci_pieces<<<ceil_div((long)nseg, 256), 256, 0, st>>>(nseg, vm, vl, vn, has, fs, fe);
            device_scan(CompactFlagOp{fs, ps, ps + c, nseg}, nseg, (uint32_t*)h->scratch, st);
            device_scan(CompactFlagOp{fe, pe, pe + c, nseg}, nseg, (uint32_t*)h->scratch, st);
            HIPCHK(h, hipMemcpyAsync(&cnt, ps + c, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(h, hipStreamSynchronize(st));
            if (cnt) k_mci_emit<<<ceil_div((long)cnt, 256), 256, 0, st>>>(cnt, ps, pe, xu, vm, vl, vn, os, oe, om, ol, on);
        }
    }
    HIPCHK(h, hipGetLastError());
    *m_out = cnt;
    if (starts && cnt) {
        HIPCHK(h, hipMemcpyAsync(starts, os, cnt * 8, hipMemcpyDeviceToHost, st));
        if (ends) HIPCHK(h, hipMemcpyAsync(ends, oe, cnt * 8, hipMemcpyDeviceToHost, st));
        if (msb) HIPCHK(h, hipMemcpyAsync(msb, om, cnt * 8, hipMemcpyDeviceToHost, st));
        if (lsb) HIPCHK(h, hipMemcpyAsync(lsb, ol, cnt * 8, hipMemcpyDeviceToHost, st));
        if (node) HIPCHK(h, hipMemcpyAsync(node, on, cnt * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    h->tracer.resolve();
    return AD_OK;
}

// BeginRecovery's store queries (recovery_kernels.h) for nq recovering rows, over the merged Deps on the handle:
// count pass, one scan for the six outputs' offsets, fill pass.  The outputs stay on the device for
// ad_fetch_recovery / ad_fetch_recovery_flags.
int ad_recover(ad_handle* h, const uint32_t* rows, size_t nq, size_t* entries) {
    if (!h || (nq && !rows)) return AD_ERR_ARGUMENT;
    if (!h->have_deps || !h->have_merged)
        return set_err(h, AD_ERR_STATE, "ad_recover needs the batch's deps and merged Deps (ad_merge_deps / _fast / ad_merge_host)");
    for (size_t q = 0; q < nq; ++q)
        if (rows[q] >= h->n) return set_err(h, AD_ERR_ARGUMENT, "ad_recover: row " + std::to_string(rows[q]) + " out of range");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    CK(complete_entries(h));
    CK(merged_ready(h));
    hipStream_t st = h->st;
    h->rc_ready = false;
    uint32_t *drows = nullptr, *cnt = nullptr, *off = nullptr;
    CK(dalloc(h, S_RCROWS, &drows, std::max<size_t>(nq, 1)));
    CK(dalloc(h, S_RCCNT, &cnt, std::max<size_t>(RC_OUT * nq, 1)));
    CK(dalloc(h, S_RCOFF, &off, RC_OUT * (nq + 1)));
    CK(dalloc(h, S_RCREJ, &h->rc_rej, std::max<size_t>(nq, 1)));
    h->rc_off = off;
    h->rc_nq = nq;
    RecoverArgs a{};
    a.nq = nq; a.rows = drows;
    a.meta = h->meta; a.tx_ts = h->tx_ts; a.ex1 = h->ex1; a.key_off = h->key_off; a.keys = h->keys;
    a.range_off = h->range_off; a.rs = h->range_s; a.re = h->range_e;
    a.ukey = h->ukey; a.useg = h->useg; a.U = h->P ? h->hprm.n_keys_u : 0;
    a.e_txn = h->e_txn; a.e_meta = h->e_meta; a.e_exec1 = h->e_exec1; a.sval = h->sval;
    a.Q = h->Q; a.es = h->es; a.ee = h->ee; a.eown = h->eown; a.ix = h->ix;
    const int ncls = (h->Q > 0 && h->merged_has_range) ? 3 : 2;
    for (int c = 0; c < ncls; ++c) {
        const Csr& m = h->merged[c];
        a.m_key_off[c] = m.key_off; a.m_keys[c] = m.keys; a.m_k2t_off[c] = m.k2t_off; a.m_k2t[c] = m.k2t;
        a.m_ent_off[c] = m.ent_off; a.m_tcnt[c] = m.tcnt; a.m_txns[c] = m.txns;
    }
    a.cnt = cnt; a.off = off; a.reject = h->rc_rej;
    std::array<uint32_t, RC_OUT> tot{};
    if (nq) {
        HIPCHK(h, hipMemcpyAsync(drows, rows, nq * 4, hipMemcpyHostToDevice, st));
        const int grid = ceil_div((long)nq * WAVE, 256);
        KScope ks(K_RECOVER, nq);
        k_recover<false><<<grid, 256, 0, st>>>(a);
        CK(ensure_scratch(h, std::max(h->scratch_cap, device_scan_scratch<RecoverOffsetsOp>(nq))));
        device_scan(RecoverOffsetsOp{cnt, off, nq}, nq, (RecoverOffsetsOp::S*)h->scratch, st);
        for (int o = 0; o < RC_OUT; ++o)
            HIPCHK(h, hipMemcpyAsync(&tot[o], off + (size_t)o * (nq + 1) + nq, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        for (int o = 0; o < RC_OUT; ++o) {
            const int kw = o % 3 == AD_CLASS_RANGE ? 2 : 1;
            CK(dalloc(h, S_RCK0 + o, &h->rc_keys[o], std::max<size_t>((size_t)tot[o] * kw, 1)));
            CK(dalloc(h, S_RCT0 + o, &h->rc_txn[o], std::max<size_t>(tot[o], 1)));
            a.okeys[o] = h->rc_keys[o]; a.otxn[o] = h->rc_txn[o];
        }
        k_recover<true><<<grid, 256, 0, st>>>(a);
        HIPCHK(h, hipGetLastError());
    } else {
        HIPCHK(h, hipMemsetAsync(off, 0, RC_OUT * 4, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    h->tracer.resolve();
    if (entries)
        for (int o = 0; o < RC_OUT; ++o) entries[o] = tot[o];
    h->rc_ready = true;
    return AD_OK;
}

int ad_fetch_recovery(ad_handle* h, uint32_t which, uint32_t cls, uint32_t* off, uint64_t* keys, uint32_t* txns) {
    if (!h || which > 1 || cls >= AD_NUM_CLASSES) return AD_ERR_ARGUMENT;
    if (!h->rc_ready) return set_err(h, AD_ERR_STATE, "no ad_recover result for this batch");
    hipSetDevice(h->device);
    const int o = (int)(which * 3 + cls);
    const size_t nq = h->rc_nq;
    hipStream_t st = h->st;
    uint32_t total = 0;
    HIPCHK(h, hipMemcpyAsync(&total, h->rc_off + (size_t)o * (nq + 1) + nq, 4, hipMemcpyDeviceToHost, st));
    if (off) HIPCHK(h, hipMemcpyAsync(off, h->rc_off + (size_t)o * (nq + 1), (nq + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    const int kw = cls == AD_CLASS_RANGE ? 2 : 1;
    if (total && keys) HIPCHK(h, hipMemcpyAsync(keys, h->rc_keys[o], (size_t)total * kw * 8, hipMemcpyDeviceToHost, st));
    if (total && txns) HIPCHK(h, hipMemcpyAsync(txns, h->rc_txn[o], (size_t)total * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    return AD_OK;
}

int ad_fetch_recovery_flags(ad_handle* h, uint8_t* reject_fast_path) {
    if (!h) return AD_ERR_ARGUMENT;
    if (!h->rc_ready) return set_err(h, AD_ERR_STATE, "no ad_recover result for this batch");
    hipSetDevice(h->device);
    if (h->rc_nq && reject_fast_path) {
        HIPCHK(h, hipMemcpyAsync(reject_fast_path, h->rc_rej, h->rc_nq, hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
    }
    return AD_OK;
}

int ad_fetch_deps(ad_handle* h, uint32_t view, uint32_t cls, ad_csr_out* out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "no deps computed");
    if (view >= h->cfg.replicas || cls >= AD_NUM_CLASSES) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (cls == AD_CLASS_RANGE) return h->Q ? fetch_csr(h, h->rdeps[view], 2, out) : fetch_empty(h, out);
    return fetch_csr(h, h->deps[2 * view + cls], 1, out);
}

int ad_merge_deps(ad_handle* h, ad_csr_sizes* sizes) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    hipSetDevice(h->device);
    CK(stage_merge(h));
    h->merged_has_range = h->Q > 0;
    if (sizes) {
        CK(merged_ready(h));
        CK(csr_sizes(h, h->merged[0], &sizes[0]));
        CK(csr_sizes(h, h->merged[1], &sizes[1]));
        if (h->Q) CK(csr_sizes(h, h->merged[2], &sizes[2]));
        else sizes[2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
    }
    return AD_OK;
}

static __global__ void k_fast_rows(size_t n, int nv, const uint8_t* __restrict__ fast, int32_t* __restrict__ rows) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < n * (size_t)nv) rows[x] = fast[x] == 1 ? (int32_t)(x % n) : -1;     // not AD_FAST_REJECTED
}

// The coordinator's fast-path merge (CoordinateTransaction.onPreAccepted :75): per txn, only the replies whose
// witnessedAt == TxnId — the fast flags of the last ad_max_conflicts(_ts) on this batch.
int ad_merge_deps_fast(ad_handle* h, ad_csr_sizes* sizes) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_merge_deps_fast before ad_preaccept_deps");
    if (!h->mc_fast) return set_err(h, AD_ERR_STATE, "ad_merge_deps_fast: run ad_max_conflicts(_ts) on this batch first");
    hipSetDevice(h->device);
    StageScope sc(h, STAGE_MERGE);
    const size_t n = h->n;
    const int nv = (int)h->cfg.replicas;
    int32_t* rows = nullptr;
    CK(dalloc(h, S_FASTROWS, &rows, std::max<size_t>(n * nv, 1)));
    if (n) k_fast_rows<<<ceil_div((long)(n * nv), 256), 256, 0, h->st>>>(n, nv, h->mc_fast, rows);
    const Csr* parts[3][MAXV] = {};
    const int32_t* vr[MAXV] = {};
    for (int v = 0; v < nv; ++v) {
        parts[0][v] = &h->deps[2 * v];
        parts[1][v] = &h->deps[2 * v + 1];
        parts[2][v] = &h->rdeps[v];
        vr[v] = rows + (size_t)v * n;
    }
    h->merge_heavy = true;
    CK(merge_parts(h, parts, nv, h->Q > 0, vr, h->deps_direct));
    h->merged_has_range = h->Q > 0;
    if (sizes) {
        CK(csr_sizes(h, h->merged[0], &sizes[0]));
        CK(csr_sizes(h, h->merged[1], &sizes[1]));
        if (h->Q) CK(csr_sizes(h, h->merged[2], &sizes[2]));
        else sizes[2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
    }
    return AD_OK;
}

// Union-view merged Deps (capacity regions + per-txn unique counts) compacted ON THE DEVICE into exact per-txn
// TxnId lists, once per batch, so the fetch is straight DMA into the caller's (pinned) buffers as for exact merges:
// one exclusive scan of the counts and one copy pass per class, then one small read of the totals.
static __global__ void k_compact_rows(size_t n, const uint32_t* __restrict__ ent_off, const uint32_t* __restrict__ tcnt,
                                      const uint32_t* __restrict__ xoff, const uint32_t* __restrict__ txns,
                                      uint32_t* __restrict__ out) {
    // one wave per 64 txns, lanes over one txn's entries at a time (rows are short: coalesced within a row)
    const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
    const int lane = threadIdx.x % WAVE;
    const size_t t0 = w * WAVE;
    for (size_t t = t0; t < t0 + WAVE && t < n; ++t) {
        const uint32_t c = tcnt[t], src = ent_off[t], dst = xoff[t];
        for (uint32_t j = lane; j < c; j += WAVE) out[dst + j] = txns[src + j];
    }
}
static int merged_compact(ad_handle* h) {
    if (h->merged_exact || h->merged_compacted) return AD_OK;
    const size_t n = h->n;
    hipStream_t st = h->st;
    uint32_t* totals = nullptr;
    CK(dalloc(h, S_MXS, &totals, 4));
    CK(ensure_scratch(h, device_scan_scratch<SumOp<uint32_t>>(n)));
    for (int c = 0; c < 3; ++c) {
        h->mx_tot[c] = 0;
        const Csr& m = h->merged[c];
        if (c == AD_CLASS_RANGE && !h->merged_has_range) continue;
        CK(dalloc(h, S_MXO0 + c, &h->mx_off[c], n + 1));
        CK(dalloc(h, S_MXT0 + c, &h->mx_txns[c], std::max<size_t>(m.ncap, 1)));
        if (n == 0 || m.ncap == 0) {
            HIPCHK(h, hipMemsetAsync(h->mx_off[c], 0, (n + 1) * 4, st));
        } else {
            SumOp<uint32_t> op{m.tcnt, h->mx_off[c], n};
            device_scan(op, n, (uint32_t*)h->scratch, st);
            k_compact_rows<<<ceil_div((long)ceil_div((long)n, WAVE) * WAVE, 256), 256, 0, st>>>(
                n, m.ent_off, m.tcnt, h->mx_off[c], m.txns, h->mx_txns[c]);
        }
        HIPCHK(h, hipMemcpyAsync(totals + c, h->mx_off[c] + n, 4, hipMemcpyDeviceToDevice, st));
    }
    uint32_t tot[3] = {0, 0, 0};
    HIPCHK(h, hipMemcpyAsync(tot, totals, 12, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    for (int c = 0; c < 3; ++c)
        if (!(c == AD_CLASS_RANGE && !h->merged_has_range)) h->mx_tot[c] = tot[c];
    h->merged_compacted = true;
    return AD_OK;
}

int ad_fetch_merged(ad_handle* h, uint32_t cls, ad_csr_out* out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "no merged deps");
    if (cls >= AD_NUM_CLASSES) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (cls == AD_CLASS_RANGE && !h->merged_has_range) return fetch_empty(h, out);
    CK(merged_ready(h));
    if (h->merged_exact) return fetch_csr(h, h->merged[cls], cls == AD_CLASS_RANGE ? 2 : 1, out);
    CK(merged_compact(h));               // union view: the device-compacted lists, straight DMA
    const Csr& m = h->merged[cls];
    const size_t n = h->n;
    const int kw = cls == AD_CLASS_RANGE ? 2 : 1;
    hipStream_t st = h->st;
    HIPCHK(h, hipMemcpyAsync(out->key_off, m.key_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(out->k2t_off, m.k2t_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(out->txn_off, h->mx_off[cls], (n + 1) * 4, hipMemcpyDeviceToHost, st));
    if (m.nkeys) HIPCHK(h, hipMemcpyAsync(out->keys, m.keys, m.nkeys * 8 * kw, hipMemcpyDeviceToHost, st));
    if (m.nk2t) HIPCHK(h, hipMemcpyAsync(out->k2t, m.k2t, m.nk2t * 4, hipMemcpyDeviceToHost, st));
    if (h->mx_tot[cls]) HIPCHK(h, hipMemcpyAsync(out->txns, h->mx_txns[cls], h->mx_tot[cls] * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    return AD_OK;
}

// The merged Deps of every class in one call: Deps.merge's outputs carry exact per-txn TxnId offsets
// (MultiOffsetsOp), so every array goes straight from HBM into the caller's buffers (pinned: DMA) with one stream
// sync and no host-side compaction.  out[c] sized by ad_merged_sizes.  Merged Deps built as the deps stage's union
// view (ad_run_pipeline) hold per-txn capacity regions like the replies: those go through fetch_csr's compaction.
int ad_merged_sizes(ad_handle* h, ad_csr_sizes* sizes /* [3] */) {
    if (!h || !sizes) return AD_ERR_ARGUMENT;
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "no merged deps");
    hipSetDevice(h->device);
    CK(merged_ready(h));
    if (!h->merged_exact) {
        hipSetDevice(h->device);
        CK(merged_compact(h));
        for (int c = 0; c < 3; ++c) {
            const Csr& m = h->merged[c];
            if (c == AD_CLASS_RANGE && !h->merged_has_range) { sizes[c] = ad_csr_sizes{h->n, 0, 0, 0, 0}; continue; }
            sizes[c] = ad_csr_sizes{h->n, m.nkeys, m.nk2t, h->mx_tot[c], h->mx_tot[c]};   // the compacted lists
        }
        return AD_OK;
    }
    for (int c = 0; c < 3; ++c) {
        const Csr& m = h->merged[c];
        const bool empty = c == AD_CLASS_RANGE && !h->merged_has_range;
        sizes[c] = empty ? ad_csr_sizes{h->n, 0, 0, 0, 0} : ad_csr_sizes{h->n, m.nkeys, m.nk2t, m.ncap, m.ncap};
    }
    return AD_OK;
}

int ad_fetch_merged_all(ad_handle* h, ad_csr_out* out /* [3] */) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "no merged deps");
    hipSetDevice(h->device);
    CK(merged_ready(h));
    CK(merged_compact(h));
    hipStream_t st = h->st;
    const size_t n = h->n;
    for (int c = 0; c < 3; ++c) {
        const Csr& m = h->merged[c];
        ad_csr_out& o = out[c];
        if (c == AD_CLASS_RANGE && !h->merged_has_range) {
            for (size_t i = 0; i <= n; ++i) { o.key_off[i] = 0; o.k2t_off[i] = 0; o.txn_off[i] = 0; }
            continue;
        }
        const int kw = c == AD_CLASS_RANGE ? 2 : 1;
        const uint32_t* toff = h->merged_exact ? m.ent_off : h->mx_off[c];
        const uint32_t* tx = h->merged_exact ? m.txns : h->mx_txns[c];
        const size_t nt = h->merged_exact ? m.ncap : h->mx_tot[c];
        HIPCHK(h, hipMemcpyAsync(o.key_off, m.key_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(o.k2t_off, m.k2t_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(o.txn_off, toff, (n + 1) * 4, hipMemcpyDeviceToHost, st));
        if (m.nkeys) HIPCHK(h, hipMemcpyAsync(o.keys, m.keys, m.nkeys * 8 * kw, hipMemcpyDeviceToHost, st));
        if (m.nk2t) HIPCHK(h, hipMemcpyAsync(o.k2t, m.k2t, m.nk2t * 4, hipMemcpyDeviceToHost, st));
        if (nt) HIPCHK(h, hipMemcpyAsync(o.txns, tx, nt * 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipStreamSynchronize(st));
    return AD_OK;
}

// The merged Deps (3 classes) and the levels / order of the batch, paged out while the device goes on: on the main
// stream they are copied into a device staging buffer (after the previous page-out from it has finished), then a
// copy stream pages the staging buffer out into the caller's (pinned) buffers.  The next ad_run_pipeline may start at
// once; ad_fetch_wait returns when the host buffers hold the results.
int ad_fetch_results_async(ad_handle* h, ad_csr_out* out /* [3] */, uint32_t* level_out, uint32_t* order_out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "no merged deps");
    if ((level_out || order_out) && !h->have_levels) return set_err(h, AD_ERR_STATE, "no levels computed for this batch");
    hipSetDevice(h->device);
    CK(merged_ready(h));
    CK(merged_compact(h));
    hipStream_t st = h->st;
    if (!h->fst) {
        HIPCHK(h, hipStreamCreateWithFlags(&h->fst, hipStreamNonBlocking));
        HIPCHK(h, hipEventCreateWithFlags(&h->fev0, hipEventDisableTiming));
        HIPCHK(h, hipEventCreateWithFlags(&h->fev1, hipEventDisableTiming));
    }
    const size_t n = h->n;
    struct Piece { void* host; const void* dev; size_t bytes; };
    std::vector<Piece> ps;
    for (int c = 0; c < 3; ++c) {
        const Csr& m = h->merged[c];
        ad_csr_out& o = out[c];
        if (c == AD_CLASS_RANGE && !h->merged_has_range) {
            for (size_t i = 0; i <= n; ++i) { o.key_off[i] = 0; o.k2t_off[i] = 0; o.txn_off[i] = 0; }
            continue;
        }
        const int kw = c == AD_CLASS_RANGE ? 2 : 1;
        const uint32_t* toff = h->merged_exact ? m.ent_off : h->mx_off[c];
        const uint32_t* tx = h->merged_exact ? m.txns : h->mx_txns[c];
        const size_t nt = h->merged_exact ? m.ncap : h->mx_tot[c];
        ps.push_back({o.key_off, m.key_off, (n + 1) * 4});
        ps.push_back({o.k2t_off, m.k2t_off, (n + 1) * 4});
        ps.push_back({o.txn_off, toff, (n + 1) * 4});
        if (m.nkeys) ps.push_back({o.keys, m.keys, m.nkeys * 8 * kw});
        if (m.nk2t) ps.push_back({o.k2t, m.k2t, m.nk2t * 4});
        if (nt) ps.push_back({o.txns, tx, nt * 4});
    }
    if (level_out && n) ps.push_back({level_out, h->lvl, n * 4});
    if (order_out && n) ps.push_back({order_out, h->order, n * 4});
    size_t tot = 0;
    for (auto& p : ps) tot += (p.bytes + 255) & ~size_t(255);
    // the staging buffer is reused: the previous page-out from it must be done before it is overwritten (device-side)
    if (h->fetch_pending) HIPCHK(h, hipStreamWaitEvent(st, h->fev1, 0));
    uint8_t* stage = nullptr;
    CK(dalloc(h, S_FSTAGE, &stage, std::max<size_t>(tot, 256)));
    size_t at = 0;
    for (auto& p : ps) {
        HIPCHK(h, hipMemcpyAsync(stage + at, p.dev, p.bytes, hipMemcpyDeviceToDevice, st));
        at += (p.bytes + 255) & ~size_t(255);
    }
    HIPCHK(h, hipEventRecord(h->fev0, st));
    HIPCHK(h, hipStreamWaitEvent(h->fst, h->fev0, 0));
    at = 0;
    for (auto& p : ps) {
        HIPCHK(h, hipMemcpyAsync(p.host, stage + at, p.bytes, hipMemcpyDeviceToHost, h->fst));
        at += (p.bytes + 255) & ~size_t(255);
    }
    HIPCHK(h, hipEventRecord(h->fev1, h->fst));
    h->fetch_pending = true;
    return AD_OK;
}

int ad_fetch_wait(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    if (!h->fetch_pending) return AD_OK;
    hipSetDevice(h->device);
    HIPCHK(h, hipEventSynchronize(h->fev1));
    h->fetch_pending = false;
    return AD_OK;
}

int ad_fetch_rows(ad_handle* h, uint32_t view, uint32_t cls, size_t lo, size_t hi, ad_csr_sizes* sizes, ad_csr_out* out) {
    if (!h || !sizes) return AD_ERR_ARGUMENT;
    if (cls >= AD_NUM_CLASSES || view > h->cfg.replicas) return set_err(h, AD_ERR_ARGUMENT, "view/class out of range");
    if (lo > hi || hi > h->n) return set_err(h, AD_ERR_ARGUMENT, "row range outside the batch");
    hipSetDevice(h->device);
    const Csr* c;
    if (view == h->cfg.replicas) {
        if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_fetch_rows of the merged Deps before ad_merge_deps");
        CK(merged_ready(h));
        c = &h->merged[cls];
    } else {
        if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_fetch_rows before ad_preaccept_deps");
        c = cls == AD_CLASS_RANGE ? &h->rdeps[view] : &h->deps[2 * view + cls];
    }
    if (c->ncap == 0 && c->nkeys == 0) {          // empty class: offsets are zero
        sizes->n = hi - lo; sizes->keys = sizes->k2t = sizes->txn_cap = sizes->txns = 0;
        if (out) for (size_t i = 0; i <= hi - lo; ++i) out->key_off[i] = out->k2t_off[i] = out->txn_off[i] = 0;
        return AD_OK;
    }
    return fetch_rows(h, *c, cls == AD_CLASS_RANGE ? 2 : 1, lo, hi, sizes, out);
}

int ad_merge_host(ad_handle* h, const ad_csr_in* parts, uint32_t r, ad_csr_sizes* sizes) {
    if (h) h->merge_heavy = true;      // caller-supplied replies: any shape
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "no batch loaded");
    if (!parts || r < 1 || r > (uint32_t)MAXV) return set_err(h, AD_ERR_ARGUMENT, "ad_merge_host: 1..8 replies");
    hipSetDevice(h->device);
    const size_t n = h->n;
    hipStream_t st = h->st;
    bool has_range = false;
    const Csr* ptr[3][MAXV] = {};
    for (uint32_t v = 0; v < r; ++v) {
        for (int cls = 0; cls < 3; ++cls) {
            const ad_csr_in& in = parts[v * AD_NUM_CLASSES + cls];
            const int kw = cls == AD_CLASS_RANGE ? 2 : 1;
            size_t nk = 0, nm = 0, nt = 0;
            std::string why;
            if (!valid_part(in, n, kw, &nk, &nm, &nt, why))
                return set_err(h, AD_ERR_ARGUMENT, "ad_merge_host: reply " + std::to_string(v) + " class " + std::to_string(cls) + ": " + why);
            if (cls == AD_CLASS_RANGE && nk > 0) has_range = true;
            Csr& c = h->hparts[cls][v];
            const size_t block = CSR_HOST0 + cls * MAXV + v;
            CK(alloc_csr(h, block, c, n));
            dirty_csr(h, block);
            c.nkeys = nk; c.nk2t = nm; c.ncap = nt;
            CK(alloc_csr_data(h, block, c, kw));
            HIPCHK(h, hipMemcpyAsync(c.key_off, in.key_off, (n + 1) * 4, hipMemcpyHostToDevice, st));
            HIPCHK(h, hipMemcpyAsync(c.k2t_off, in.k2t_off, (n + 1) * 4, hipMemcpyHostToDevice, st));
            HIPCHK(h, hipMemcpyAsync(c.ent_off, in.txn_off, (n + 1) * 4, hipMemcpyHostToDevice, st));
            if (nk) HIPCHK(h, hipMemcpyAsync(c.keys, in.keys, nk * 8 * kw, hipMemcpyHostToDevice, st));
            if (nm) HIPCHK(h, hipMemcpyAsync(c.k2t, in.k2t, nm * 4, hipMemcpyHostToDevice, st));
            if (nt) HIPCHK(h, hipMemcpyAsync(c.txns, in.txns, nt * 4, hipMemcpyHostToDevice, st));
            if (n) k_tcnt_from_off<<<ceil_div((long)n, 256), 256, 0, st>>>(n, c.ent_off, c.tcnt);
            ptr[cls][v] = &c;
        }
    }
    CK(merge_parts(h, ptr, (int)r, has_range));
    h->merged_has_range = has_range;
    if (sizes) {
        CK(csr_sizes(h, h->merged[0], &sizes[0]));
        CK(csr_sizes(h, h->merged[1], &sizes[1]));
        if (has_range) CK(csr_sizes(h, h->merged[2], &sizes[2]));
        else sizes[2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
    }
    return AD_OK;
}

int ad_exec_levels(ad_handle* h, uint32_t* level_out, uint32_t* order_out, uint32_t* iterations_out) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    hipSetDevice(h->device);
    CK(stage_levels(h, order_out != nullptr));
    hipStream_t st = h->st;
    HIPCHK(h, hipStreamSynchronize(st));
    CK(finish_order(h));
    if (level_out && h->n) HIPCHK(h, hipMemcpyAsync(level_out, h->lvl, h->n * 4, hipMemcpyDeviceToHost, st));
    if (order_out && h->n) HIPCHK(h, hipMemcpyAsync(order_out, h->order, h->n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (iterations_out) *iterations_out = h->level_iters;
    return AD_OK;
}

int ad_fetch_levels(ad_handle* h, uint32_t* level_out, uint32_t* order_out) {
    if (!h) return AD_ERR_ARGUMENT;
    if (!h->have_levels) return set_err(h, AD_ERR_STATE, "no levels computed for this batch");
    hipSetDevice(h->device);
    if (level_out && h->n) HIPCHK(h, hipMemcpyAsync(level_out, h->lvl, h->n * 4, hipMemcpyDeviceToHost, h->st));
    if (order_out && h->n) HIPCHK(h, hipMemcpyAsync(order_out, h->order, h->n * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

// The pipeline's final wait: poll the event instead of hipEventSynchronize's blocking wait (its wake-up was most
// of the ~37 us the GPU sat idle between consecutive batches)
static int spin_event(ad_handle* h, hipEvent_t e) {
    for (uint64_t k = 0;; ++k) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return AD_OK;
        if (q != hipErrorNotReady) { HIPCHK(h, q); }
        if (k > (1u << 22)) { HIPCHK(h, hipEventSynchronize(e)); return AD_OK; }   // a long batch: block instead
    }
}

int ad_run_pipeline(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "no batch loaded");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    h->ht.clear();
    host_mark(h, "start");
    HIPCHK(h, hipEventRecord(h->ev[0], st));
    // the merged Deps: k_merge_cap over the R replies (stage_merge); ad_set_pipeline_union(h, 1) instead builds them
    // as the deps stage's union view, a shortcut only a generator that holds every view's inputs can take
    h->want_union = h->pipeline_union;
    h->in_pipeline = true;                       // stage_prepare: k_seg_fuse may build the pull pass's chains
    const int rc_prep = stage_prepare(h);
    h->in_pipeline = false;
    CK(rc_prep);
    host_mark(h, "prepare returned");
    HIPCHK(h, hipEventRecord(h->ev[1], st));
    CK(stage_sort(h));
    HIPCHK(h, hipEventRecord(h->ev[2], st));
    host_mark(h, "sort enqueued");
    h->xdefer = true;                            // k_txn_finish_ovf's side stream joins where its rows are read
    const int rc_deps = stage_deps(h);            // (joins the side stream itself on an error)
    h->xdefer = false;
    if (rc_deps != AD_OK) { side_join(h); return rc_deps; }
    HIPCHK(h, hipEventRecord(h->ev[3], st));
    host_mark(h, "deps returned");
    h->merge_side = true;                        // a merge of identical-shape replies may run beside the levels
    h->merge_sided = false;
    int rc = stage_merge(h);
    h->merge_side = false;
    host_mark(h, "merge returned");
    if (rc == AD_OK) {
        h->merged_has_range = h->Q > 0;
        if (!h->merge_sided) HIPCHK(h, hipEventRecord(h->ev[4], st));
        rc = stage_levels(h, true);
    }
    host_mark(h, "levels returned");
    side_join(h);                                // also on an error: nothing may read the CSRs before the side rows
    CK(rc);
    HIPCHK(h, hipEventRecord(h->ev[5], st));
    CK(spin_event(h, h->ev[5]));
    if (order_failed(h)) {                       // optimistic order failed its check: general path, timed in
        CK(finish_order(h));
        HIPCHK(h, hipEventRecord(h->ev[5], st));
        HIPCHK(h, hipEventSynchronize(h->ev[5]));
    }
    h->order_pending = false;
    float ms;
    hipEventElapsedTime(&ms, h->ev[0], h->ev[1]); h->times.prepare = ms;
    hipEventElapsedTime(&ms, h->ev[1], h->ev[2]); h->times.sort = ms;
    hipEventElapsedTime(&ms, h->ev[2], h->ev[3]); h->times.deps = ms;
    // (a merge beside the levels: both timed from the end of the deps stage)
    hipEventElapsedTime(&ms, h->ev[3], h->ev[4]); h->times.merge = ms;
    hipEventElapsedTime(&ms, h->ev[h->merge_sided ? 3 : 4], h->ev[5]); h->times.levels = ms;
    hipEventElapsedTime(&ms, h->ev[0], h->ev[5]); h->times.total = ms;
    h->times.deps_entries = h->deps_entries;
    h->times.merged_entries = h->merged_entries;
    h->times.level_iterations = h->level_iters;
    h->times.level_edges = h->P;
    h->times.walk_items = (uint32_t)(h->P - (h->P ? h->hprm.n_keys_u : 0));
    h->times.gather_items = (!h->nh_valid && h->sf_ntiles && h->P) ? h->times.walk_items + h->hprm.n_multi : 0u;
    h->tracer.resolve();
    host_mark(h, "end");
    if (h->host_timers == 1 && h->ht.size() > 1) {
        std::string line = "host_timers";
        for (size_t i = 1; i < h->ht.size(); ++i)
            line += std::string(" | ") + h->ht[i].first + " " +
                    std::to_string(std::chrono::duration<double, std::micro>(h->ht[i].second - h->ht[0].second).count());
        fprintf(stderr, "%s\n", line.c_str());
    }
    return AD_OK;
}

int ad_last_times(ad_handle* h, ad_stage_times* out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (h->mcap_entries_pending) {
        hipSetDevice(h->device);
        CK(merged_entries_resolve(h));
        h->times.merged_entries = h->merged_entries;
    }
    *out = h->times;
    return AD_OK;
}

int ad_kernel_count(void) { return K_COUNT; }

const char* ad_kernel_name(int kid) { return kernel_name(kid); }

int ad_set_level_mode(ad_handle* h, int mode) {
    if (!h || (mode != AD_LEVELS_AUTO && mode != AD_LEVELS_FIXPOINT && mode != AD_LEVELS_BLOCKS && mode != AD_LEVELS_KAHN &&
               mode != AD_LEVELS_PULL_ABORT && mode != AD_LEVELS_BLOCKS_WIDE))
        return AD_ERR_ARGUMENT;
    h->level_mode = mode;
    return AD_OK;
}

int ad_set_pipeline_union(ad_handle* h, int on) {
    if (!h) return AD_ERR_ARGUMENT;
    h->pipeline_union = on != 0;
    return AD_OK;
}

int ad_set_trace(ad_handle* h, uint64_t mask) {
    if (!h) return AD_ERR_ARGUMENT;
    h->tracer.mask = mask;
    return AD_OK;
}

int ad_kernel_stats(ad_handle* h, int kid, const char** name, uint64_t* calls, double* total_ms) {
    if (!h || kid < 0 || kid >= K_COUNT) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->tracer.resolve();
    if (name) *name = kernel_name(kid);
    if (calls) *calls = h->tracer.calls[kid];
    if (total_ms) *total_ms = h->tracer.total_ms[kid];
    return AD_OK;
}

int ad_kernel_units(ad_handle* h, int kid, uint64_t* units) {
    if (!h || !units || kid < 0 || kid >= K_COUNT) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->tracer.resolve();
    *units = h->tracer.units[kid];
    return AD_OK;
}

int ad_reset_kernel_stats(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->tracer.resolve();
    h->tracer.reset_counts();
    return AD_OK;
}

}  // extern "C"
