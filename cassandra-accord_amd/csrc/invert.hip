// invert.hip — ad_fetch_inverse: KeyDeps.txnIdsToKeys / RangeDeps.txnIdsToRanges of a row window of a batched
// Deps CSR (invert_kernels.h; RelationMultiMap.invert, utils/RelationMultiMap.java:907-938).
#include "engine_internal.h"

int ad_fetch_inverse(ad_handle* h, uint32_t view, uint32_t cls, size_t lo, size_t hi, size_t* total, uint32_t* off,
                     int32_t* inv) {
    if (!h || !total) return AD_ERR_ARGUMENT;
    if (cls >= AD_NUM_CLASSES || view > h->cfg.replicas) return set_err(h, AD_ERR_ARGUMENT, "ad_fetch_inverse: view/class out of range");
    if (lo > hi || hi > h->n) return set_err(h, AD_ERR_ARGUMENT, "ad_fetch_inverse: row range outside the batch");
    const Csr* c;
    if (view == h->cfg.replicas) {
        if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_fetch_inverse of the merged Deps before ad_merge_deps");
        CK(merged_ready(h));
        c = &h->merged[cls];
    } else {
        if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_fetch_inverse before ad_preaccept_deps");
        c = cls == AD_CLASS_RANGE ? &h->rdeps[view] : &h->deps[2 * view + cls];
    }
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    const size_t m = hi - lo;
    *total = 0;
    if (m == 0 || (c->ncap == 0 && c->nkeys == 0)) {      // empty window / empty class: every row's inverse is empty
        if (off) for (size_t i = 0; i <= m; ++i) off[i] = 0;
        return AD_OK;
    }
    hipStream_t st = h->st;
    uint32_t* cnt;                                          // nt[m] ne[m] tb[m+1] eb[m+1] bad[1]
    CK(dalloc(h, S_IVC, &cnt, 4 * m + 8));
    InvArgs a{};
    a.m = m; a.lo = lo;
    a.key_off = c->key_off; a.k2t_off = c->k2t_off; a.tcnt = c->tcnt; a.k2t = c->k2t;
    a.nt = cnt; a.ne = cnt + m;
    uint32_t* tb = cnt + 2 * m;
    uint32_t* eb = tb + m + 1;
    a.tb = tb; a.eb = eb; a.bad = eb + m + 1;
    CK(ensure_scratch(h, std::max(h->scratch_cap, device_scan_scratch<SumOp<uint32_t>>(m + 1))));
    HIPCHK(h, hipMemsetAsync(a.bad, 0, 4, st));
    k_inv_counts<<<ceil_div((long)m, 256), 256, 0, st>>>(a);
    scan_offsets(h, a.nt, tb, m);      // exclusive: [m + 1]
    scan_offsets(h, a.ne, eb, m);
    std::vector<uint32_t> hcnt(2 * m), htb(m + 1), heb(m + 1);
    HIPCHK(h, hipMemcpyAsync(hcnt.data(), cnt, 2 * m * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(htb.data(), tb, (m + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipMemcpyAsync(heb.data(), eb, (m + 1) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    // the totals in 64 bits from the per-row counts: the u32 prefix sums above wrap past 2^32
    uint64_t NT64 = 0, E64 = 0;
    for (size_t i = 0; i < m; ++i) { NT64 += hcnt[i]; E64 += hcnt[m + i]; }
    if (NT64 + E64 >= (uint64_t)1 << 31)
        return set_err(h, AD_ERR_UNSUPPORTED, "ad_fetch_inverse: the window's inverse exceeds 2^31 ints (page a smaller row window)");
    const size_t NT = htb[m], E = heb[m];
    if (NT != NT64 || E != E64) return set_err(h, AD_ERR_DEVICE, "ad_fetch_inverse: device prefix sums disagree with the counts");
    *total = NT + E;
    if (off) for (size_t i = 0; i <= m; ++i) off[i] = htb[i] + heb[i];
    if (!inv) return AD_OK;
    uint32_t *k0, *v0, *k1, *v1;
    int32_t* out;
    CK(dalloc(h, S_IVK0, &k0, E)); CK(dalloc(h, S_IVV0, &v0, E));
    CK(dalloc(h, S_IVK1, &k1, E)); CK(dalloc(h, S_IVV1, &v1, E));
    CK(dalloc(h, S_IVOUT, &out, NT + E));
    a.skey = k0; a.sval = v0; a.out = out; a.total_nt = NT; a.E = E;
    k_inv_expand<<<ceil_div((long)m * WAVE, 256), 256, 0, st>>>(a);
    uint32_t hbad = 0;
    HIPCHK(h, hipMemcpyAsync(&hbad, a.bad, 4, hipMemcpyDeviceToHost, st));
    const int bits = NT > 1 ? bits_of(NT - 1) : 0;
    bool flip = false;
    if (E > 0 && bits > 0) {
        CK(ensure_scratch(h, std::max(h->scratch_cap, (size_t)(3 * (radix_hist_len(E) + 128) + 64 * 1024) * 4)));
        flip = radix_sort_pairs(k0, v0, k1, v1, E, bits, radix_scratch(h, E), st);
    }
    const uint32_t* sk = flip ? k1 : k0;
    const uint32_t* sv = flip ? v1 : v0;
    if (E) k_inv_body<<<ceil_div((long)E, 256), 256, 0, st>>>(a, sk, sv);
    if (NT) k_inv_header<<<ceil_div((long)NT, 256), 256, 0, st>>>(a, sk);
    HIPCHK(h, hipMemcpyAsync(inv, out, (NT + E) * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (hbad) return set_err(h, AD_ERR_ARGUMENT, "ad_fetch_inverse: a keysToTxnIds entry is outside its TxnId list");
    return AD_OK;
}
