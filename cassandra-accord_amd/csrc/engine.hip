// engine.hip — host orchestration + C-ABI (include/accord_deps.h) of the gfx950 deps engine.
//
// One ad_handle = one CommandStore shard on one GPU: a HIP stream, a device arena and the loaded
// batch.  Stages:
//   prepare   batch statistics, timestamp packing (ts64), pair owners       (deps_kernels.h)
//   sort      stable LSD radix sort of (key, pair)                          (radix_sort.h)
//   deps      CFK elision scans, per-pair walk (count/fill), per-txn layout and TxnId union
//   merge     Deps.merge of the R replica views per txn                     (merge_kernels.h)
//   levels    execution levels over key chains + deps                       (level_kernels.h)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "deps_kernels.h"
#include "level_kernels.h"
#include "merge_kernels.h"
#include "radix_sort.h"

using namespace ad;

namespace {

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
};

using Csr = ad::DevCsr;

}  // namespace

struct ad_handle {
    int device = 0;
    ad_config cfg{};
    hipStream_t st = nullptr;
    std::string err;
    std::vector<DBuf> bufs;
    // loaded batch
    size_t n = 0, P = 0, Q = 0;
    bool loaded = false;
    uint64_t *tm = nullptr, *tl = nullptr, *em = nullptr, *el = nullptr, *keys = nullptr;
    int32_t *tn = nullptr, *en = nullptr;
    uint8_t* status = nullptr;
    uint32_t *key_off = nullptr, *range_off = nullptr;
    uint64_t *range_s = nullptr, *range_e = nullptr;
    // derived
    Params* prm = nullptr;
    Params hprm{};
    TsPack pack{};
    int key_bits = 0;
    uint64_t *tx_ts = nullptr, *ex1 = nullptr;
    uint8_t* meta = nullptr;
    uint32_t *pair_txn = nullptr, *ka = nullptr, *va = nullptr, *kb = nullptr, *vb = nullptr;
    uint32_t *skey = nullptr, *sval = nullptr;           // sorted (alias ka/kb)
    uint32_t *e_txn = nullptr, *spos = nullptr;
    uint8_t* e_meta = nullptr;
    uint64_t *e_exec1 = nullptr, *pm_w = nullptr, *pm_c = nullptr;
    int32_t *seg_start = nullptr, *ud_prev = nullptr;
    uint32_t *cnt = nullptr, *dst = nullptr, *nk = nullptr, *ne = nullptr;
    void* scratch = nullptr;
    size_t scratch_cap = 0;
    std::vector<Csr> deps;           // [view * 2 + class]  (key, direct)
    Csr merged[2];
    bool have_deps = false, have_merged = false, have_levels = false;
    // levels
    uint32_t *lvl = nullptr, *order = nullptr;
    uint32_t level_iters = 0;
    LevelState ls{};
    // timing
    hipEvent_t ev[8]{};
    ad_stage_times times{};
    Tracer tracer;
    uint64_t deps_entries = 0, merged_entries = 0;
};

namespace {

#define HIPCHK(h, x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            (h)->err = std::string(#x) + ": " + hipGetErrorString(e_);                 \
            return AD_ERR_DEVICE;                                                      \
        }                                                                              \
    } while (0)

int set_err(ad_handle* h, int code, const std::string& msg) {
    h->err = msg;
    return code;
}

// Grow-only device allocation slot `slot` of at least `bytes`.
template <class T>
int dalloc(ad_handle* h, size_t slot, T** out, size_t count) {
    if (h->bufs.size() <= slot) h->bufs.resize(slot + 1);
    DBuf& b = h->bufs[slot];
    size_t bytes = std::max<size_t>(count * sizeof(T), 256);
    if (b.cap < bytes) {
        if (b.p) { HIPCHK(h, hipStreamSynchronize(h->st)); HIPCHK(h, hipFree(b.p)); }
        size_t nb = std::max(bytes, b.cap + b.cap / 4);
        HIPCHK(h, hipMalloc(&b.p, nb));
        b.cap = nb;
    }
    *out = (T*)b.p;
    return AD_OK;
}

enum Slot : size_t {
    S_TM, S_TL, S_TN, S_EM, S_EL, S_EN, S_ST, S_KOFF, S_KEYS, S_ROFF, S_RS, S_RE,
    S_PRM, S_TXTS, S_EX1, S_META, S_PTXN, S_KA, S_VA, S_KB, S_VB, S_ETXN, S_SPOS, S_EMETA, S_EEXEC,
    S_PMW, S_PMC, S_SEG, S_UD, S_CNT, S_DST, S_NK, S_NE, S_SCRATCH,
    S_LVL, S_ORDER, S_LEVEL0,
    S_CSR0 = 100
};

#define CK(x) do { int rc_ = (x); if (rc_ != AD_OK) return rc_; } while (0)

inline int bits_of(uint64_t x) { return x == 0 ? 0 : 64 - __builtin_clzll(x); }

int ensure_scratch(ad_handle* h, size_t bytes) {
    void* p;
    CK(dalloc(h, S_SCRATCH, (uint8_t**)&p, bytes));
    h->scratch = p;
    h->scratch_cap = bytes;
    return AD_OK;
}

int alloc_csr(ad_handle* h, size_t slot_base, Csr& c, size_t n) {
    CK(dalloc(h, slot_base + 0, &c.key_off, n + 1));
    CK(dalloc(h, slot_base + 1, &c.k2t_off, n + 1));
    CK(dalloc(h, slot_base + 2, &c.ent_off, n + 1));
    CK(dalloc(h, slot_base + 3, &c.tcnt, n));
    return AD_OK;
}
int alloc_csr_data(ad_handle* h, size_t slot_base, Csr& c) {
    CK(dalloc(h, slot_base + 4, &c.keys, c.nkeys));
    CK(dalloc(h, slot_base + 5, &c.k2t, c.nk2t));
    CK(dalloc(h, slot_base + 6, &c.txns, c.ncap));
    return AD_OK;
}

template <class T>
void scan_offsets(ad_handle* h, const T* in, T* out, size_t n) {
    if (n == 0) { hipMemsetAsync(out, 0, sizeof(T), h->st); return; }
    device_scan(SumOp<T>{in, out, n}, n, (T*)h->scratch, h->st);
}

// ---------------------------------------------------------------------------------------------------
// prepare + sort
// ---------------------------------------------------------------------------------------------------
int stage_prepare(ad_handle* h) {
    const size_t n = h->n, P = h->P;
    hipStream_t st = h->st;
    k_params_init<<<1, 1, 0, st>>>(h->prm);
    const int g = (int)std::min<size_t>(1024, std::max<size_t>(1, (std::max(n, P) + 255) / 256));
    { KScope ks(K_MINMAX); k_minmax<<<g, 256, 0, st>>>(n, h->tm, h->tl, h->tn, h->em, h->el, h->en, h->key_off, h->keys, P, h->range_off, h->prm); }
    HIPCHK(h, hipMemcpyAsync(&h->hprm, h->prm, sizeof(Params), hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    const Params& p = h->hprm;
    if (p.err & ERR_RANGE) return set_err(h, AD_ERR_UNSUPPORTED, "range-domain transactions are not supported by this build's device path");
    if (p.max_keys > (unsigned)KMAX) return set_err(h, AD_ERR_UNSUPPORTED, "more than 16 keys in one transaction");
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
    h->key_bits = P ? bits_of(p.key_max - p.key_min) : 0;
    if (h->key_bits > 32) return set_err(h, AD_ERR_UNSUPPORTED, "key spread exceeds 32 bits");
    KScope ks(K_PACK);
    k_pack<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->pack, P ? p.key_min : 0, h->tm, h->tl, h->tn, h->em, h->el, h->en,
                                                    h->status, h->key_off, h->keys, h->tx_ts, h->ex1, h->meta, h->pair_txn,
                                                    h->ka, h->va, h->prm);
    return AD_OK;
}

int stage_sort(ad_handle* h) {
    const size_t P = h->P;
    if (P == 0) return AD_OK;
    RadixScratch rs;
    const size_t hl = radix_hist_len(P);
    uint8_t* base = (uint8_t*)h->scratch;
    rs.hist = (uint32_t*)base;
    rs.offs = rs.hist + hl + 64;
    rs.agg = rs.offs + hl + 64;
    bool flip = radix_sort_pairs(h->ka, h->va, h->kb, h->vb, P, h->key_bits, rs, h->st);
    h->skey = flip ? h->kb : h->ka;
    h->sval = flip ? h->vb : h->va;
    return AD_OK;
}

// ---------------------------------------------------------------------------------------------------
// deps
// ---------------------------------------------------------------------------------------------------
template <int NV>
void launch_walk(const WalkArgs& a, bool fill, hipStream_t st) {
    const int g = ceil_div((long)a.P, 256);
    KScope ks(fill ? K_WALK_FILL : K_WALK_COUNT);
    if (fill) k_deps_walk<NV, true><<<g, 256, 0, st>>>(a);
    else k_deps_walk<NV, false><<<g, 256, 0, st>>>(a);
}
void walk(const WalkArgs& a, int nv, bool fill, hipStream_t st) {
    switch (nv) {
        case 1: launch_walk<1>(a, fill, st); break;
        case 2: launch_walk<2>(a, fill, st); break;
        case 3: launch_walk<3>(a, fill, st); break;
        case 4: launch_walk<4>(a, fill, st); break;
        case 5: launch_walk<5>(a, fill, st); break;
        case 6: launch_walk<6>(a, fill, st); break;
        case 7: launch_walk<7>(a, fill, st); break;
        default: launch_walk<8>(a, fill, st); break;
    }
}

int stage_deps(ad_handle* h) {
    const size_t n = h->n, P = h->P;
    const int nv = (int)h->cfg.replicas, nvc = 2 * nv;
    hipStream_t st = h->st;
    h->deps.resize(nvc);
    for (int vc = 0; vc < nvc; ++vc) CK(alloc_csr(h, S_CSR0 + 10 * vc, h->deps[vc], n));
    if (P > 0) {
        { KScope ks(K_GATHER); k_gather_entries<<<ceil_div((long)P, 256), 256, 0, st>>>(P, h->sval, h->pair_txn, h->meta, h->ex1, h->e_txn, h->e_meta,
                                                                   h->e_exec1, h->spos); }
        ElideOp eop{h->skey, h->e_meta, h->e_exec1, h->seg_start, h->ud_prev, h->pm_w, h->pm_c};
        KScope ks(K_SCAN_ELIDE);
        device_scan(eop, P, (ElideOp::S*)h->scratch, st);
    }
    WalkArgs wa{};
    wa.e_txn = h->e_txn; wa.e_meta = h->e_meta; wa.e_exec1 = h->e_exec1; wa.seg_start = h->seg_start;
    wa.ud_prev = h->ud_prev; wa.pm_w = h->pm_w; wa.pm_c = h->pm_c; wa.tx_ts = h->tx_ts; wa.P = P;
    wa.window = h->cfg.window; wa.thresh = ad_drop_threshold(h->cfg.drop_p); wa.seed = h->cfg.seed;
    wa.cnt = h->cnt; wa.dst = h->dst;
    if (P > 0) walk(wa, nv, false, st);
    TxnArgs ta{};
    ta.n = n; ta.P = P; ta.nvc = nvc; ta.key_off = h->key_off; ta.keys = h->keys; ta.spos = h->spos; ta.cnt = h->cnt;
    ta.nk = h->nk; ta.ne = h->ne; ta.dst = h->dst; ta.prm = h->prm;
    if (n > 0) { KScope ks(K_TXN_COUNTS); k_txn_counts<<<ceil_div((long)n, 256), 256, 0, st>>>(ta); }
    for (int vc = 0; vc < nvc; ++vc) {
        KScope ks(K_SCAN_OFFSETS);
        Csr& c = h->deps[vc];
        scan_offsets(h, h->nk + (size_t)vc * n, c.key_off, n);
        scan_offsets(h, h->ne + (size_t)vc * n, c.ent_off, n);
        if (n) device_scan(Sum2Op<uint32_t>{h->nk + (size_t)vc * n, h->ne + (size_t)vc * n, c.k2t_off, n}, n, (uint32_t*)h->scratch, st);
        else hipMemsetAsync(c.k2t_off, 0, 4, st);
    }
    // sizes -> host (one sync), allocate outputs
    std::vector<uint32_t> tot(3 * nvc);
    for (int vc = 0; vc < nvc; ++vc) {
        HIPCHK(h, hipMemcpyAsync(&tot[3 * vc + 0], h->deps[vc].key_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(&tot[3 * vc + 1], h->deps[vc].k2t_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(&tot[3 * vc + 2], h->deps[vc].ent_off + n, 4, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(h, hipMemcpyAsync(&h->hprm, h->prm, sizeof(Params), hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (h->hprm.err & ERR_UNSORTED) return set_err(h, AD_ERR_UNSORTED, "batch TxnIds are not strictly ascending");
    if (h->hprm.err & ERR_KEYS) return set_err(h, AD_ERR_UNSUPPORTED, "more than 16 keys in one transaction");
    h->deps_entries = 0;
    for (int vc = 0; vc < nvc; ++vc) {
        Csr& c = h->deps[vc];
        c.nkeys = tot[3 * vc]; c.nk2t = tot[3 * vc + 1]; c.ncap = tot[3 * vc + 2];
        h->deps_entries += c.ncap;
        CK(alloc_csr_data(h, S_CSR0 + 10 * vc, c));
        ta.out_key_off[vc] = c.key_off; ta.out_k2t_off[vc] = c.k2t_off; ta.out_keys[vc] = c.keys; ta.out_k2t[vc] = c.k2t;
        wa.k2t[vc] = c.k2t;
    }
    if (n > 0) { KScope ks(K_TXN_LAYOUT); k_txn_layout<<<ceil_div((long)n, 256), 256, 0, st>>>(ta); }
    if (P > 0) walk(wa, nv, true, st);
    UnionArgs ua{};
    ua.n = n; ua.nvc = nvc;
    for (int vc = 0; vc < nvc; ++vc) {
        Csr& c = h->deps[vc];
        ua.key_off[vc] = c.key_off; ua.k2t_off[vc] = c.k2t_off; ua.ent_off[vc] = c.ent_off; ua.k2t[vc] = c.k2t;
        ua.txns[vc] = c.txns; ua.tcnt[vc] = c.tcnt;
    }
    if (n > 0) { KScope ks(K_TXN_UNION); k_txn_union<<<ceil_div((long)n, 256), 256, 0, st>>>(ua); }
    h->have_deps = true;
    return AD_OK;
}

// ---------------------------------------------------------------------------------------------------
// merge
// ---------------------------------------------------------------------------------------------------
int stage_merge(ad_handle* h) {
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_merge_deps before ad_preaccept_deps");
    const size_t n = h->n;
    const int nv = (int)h->cfg.replicas;
    hipStream_t st = h->st;
    h->merged_entries = 0;
    for (int cls = 0; cls < 2; ++cls) {
        Csr& m = h->merged[cls];
        CK(alloc_csr(h, S_CSR0 + 10 * (NVC_MAX + cls), m, n));
        MergeArgs ma{};
        ma.n = n; ma.nv = nv;
        for (int v = 0; v < nv; ++v) {
            const Csr& c = h->deps[2 * v + cls];
            ma.key_off[v] = c.key_off; ma.keys[v] = c.keys; ma.k2t_off[v] = c.k2t_off; ma.k2t[v] = c.k2t;
            ma.ent_off[v] = c.ent_off; ma.txns[v] = c.txns; ma.tcnt[v] = c.tcnt;
        }
        ma.mk = h->nk; ma.me = h->ne; ma.mu = h->nk + n;   // scratch counters (n each)
        if (n > 0) merge_launch(ma, nv, false, st);
        {
            KScope ks(K_SCAN_OFFSETS);
            scan_offsets(h, ma.mk, m.key_off, n);
            scan_offsets(h, ma.mu, m.ent_off, n);
            if (n) device_scan(Sum2Op<uint32_t>{ma.mk, ma.me, m.k2t_off, n}, n, (uint32_t*)h->scratch, st);
            else hipMemsetAsync(m.k2t_off, 0, 4, st);
        }
        uint32_t tot[3];
        HIPCHK(h, hipMemcpyAsync(&tot[0], m.key_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(&tot[1], m.k2t_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipMemcpyAsync(&tot[2], m.ent_off + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(h, hipStreamSynchronize(st));
        m.nkeys = tot[0]; m.nk2t = tot[1]; m.ncap = tot[2];
        h->merged_entries += m.nk2t - m.nkeys;
        CK(alloc_csr_data(h, S_CSR0 + 10 * (NVC_MAX + cls), m));
        ma.o_key_off = m.key_off; ma.o_keys = m.keys; ma.o_k2t_off = m.k2t_off; ma.o_k2t = m.k2t;
        ma.o_ent_off = m.ent_off; ma.o_txns = m.txns; ma.o_tcnt = m.tcnt;
        if (n > 0) merge_launch(ma, nv, true, st);
    }
    h->have_merged = true;
    return AD_OK;
}

// ---------------------------------------------------------------------------------------------------
// levels
// ---------------------------------------------------------------------------------------------------
int stage_levels(ad_handle* h, bool want_order) {
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_exec_levels before ad_merge_deps");
    LevelInputs li{};
    li.n = h->n; li.P = h->P; li.skey = h->skey; li.e_txn = h->e_txn; li.e_meta = h->e_meta; li.e_exec1 = h->e_exec1;
    li.seg_start = h->seg_start; li.meta = h->meta; li.ex1 = h->ex1; li.lvl = h->lvl; li.order = h->order;
    li.scratch = h->scratch; li.scratch_cap = h->scratch_cap;
    li.merged_direct = &h->merged[1];
    li.exec_bits = h->pack.total_bits;
    int iters = 0;
    int rc = run_levels(h->ls, li, want_order, h->st, &iters, h->err);
    if (rc != AD_OK) return rc;
    h->level_iters = (uint32_t)iters;
    h->have_levels = true;
    return AD_OK;
}

int fetch_csr(ad_handle* h, const Csr& c, ad_csr_out* out) {
    const size_t n = h->n;
    hipStream_t st = h->st;
    std::vector<uint32_t> ent(n + 1), cnt(n);
    HIPCHK(h, hipMemcpyAsync(out->key_off, c.key_off, (n + 1) * 4, hipMemcpyDeviceToHost, st));
    if (c.nkeys) HIPCHK(h, hipMemcpyAsync(out->keys, c.keys, c.nkeys * 8, hipMemcpyDeviceToHost, st));
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
        std::memcpy(out->txns + o, tx.data() + ent[i], cnt[i] * 4);
        o += cnt[i];
        out->txn_off[i + 1] = o;
    }
    return AD_OK;
}

int csr_sizes(ad_handle* h, const Csr& c, ad_csr_sizes* s) {
    s->n = h->n; s->keys = c.nkeys; s->k2t = c.nk2t; s->txn_cap = c.ncap;
    std::vector<uint32_t> cnt(h->n);
    if (h->n) {
        HIPCHK(h, hipMemcpyAsync(cnt.data(), c.tcnt, h->n * 4, hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
    }
    size_t t = 0;
    for (uint32_t x : cnt) t += x;
    s->txns = t;
    return AD_OK;
}

}  // namespace

// =====================================================================================================
// C-ABI
// =====================================================================================================
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
    h->cfg = *cfg;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return AD_ERR_DEVICE;
    }
    for (auto& e : h->ev) hipEventCreate(&e);
    h->tracer.st = h->st;
    *out = h;
    return AD_OK;
}

void ad_close(ad_handle* h) {
    if (!h) return;
    hipSetDevice(h->device);
    if (h->st) hipStreamSynchronize(h->st);
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
    const size_t n = b->n;
    if (n >= (1ull << 31)) return set_err(h, AD_ERR_ARGUMENT, "batch too large");
    const size_t P = n ? b->key_off[n] : 0;
    const size_t Q = (n && b->range_off) ? b->range_off[n] : 0;
    h->n = n; h->P = P; h->Q = Q;
    h->have_deps = h->have_merged = h->have_levels = false;
    CK(dalloc(h, S_TM, &h->tm, n)); CK(dalloc(h, S_TL, &h->tl, n)); CK(dalloc(h, S_TN, &h->tn, n));
    CK(dalloc(h, S_EM, &h->em, n)); CK(dalloc(h, S_EL, &h->el, n)); CK(dalloc(h, S_EN, &h->en, n));
    CK(dalloc(h, S_ST, &h->status, n)); CK(dalloc(h, S_KOFF, &h->key_off, n + 1)); CK(dalloc(h, S_KEYS, &h->keys, P));
    hipStream_t st = h->st;
    if (n) {
        HIPCHK(h, hipMemcpyAsync(h->tm, b->txn_msb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->tl, b->txn_lsb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->tn, b->txn_node, n * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->em, b->exec_msb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->el, b->exec_lsb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->en, b->exec_node, n * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->status, b->status, n, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->key_off, b->key_off, (n + 1) * 4, hipMemcpyHostToDevice, st));
        if (P) HIPCHK(h, hipMemcpyAsync(h->keys, b->keys, P * 8, hipMemcpyHostToDevice, st));
    } else {
        HIPCHK(h, hipMemsetAsync(h->key_off, 0, 4, st));
    }
    h->range_off = nullptr;
    if (Q) {
        CK(dalloc(h, S_ROFF, &h->range_off, n + 1)); CK(dalloc(h, S_RS, &h->range_s, Q)); CK(dalloc(h, S_RE, &h->range_e, Q));
        HIPCHK(h, hipMemcpyAsync(h->range_off, b->range_off, (n + 1) * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->range_s, b->range_start, Q * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(h->range_e, b->range_end, Q * 8, hipMemcpyHostToDevice, st));
    }
    // working buffers
    const int nvc = 2 * (int)h->cfg.replicas;
    CK(dalloc(h, S_PRM, &h->prm, 1));
    CK(dalloc(h, S_TXTS, &h->tx_ts, n)); CK(dalloc(h, S_EX1, &h->ex1, n)); CK(dalloc(h, S_META, &h->meta, n));
    CK(dalloc(h, S_PTXN, &h->pair_txn, P));
    CK(dalloc(h, S_KA, &h->ka, P)); CK(dalloc(h, S_VA, &h->va, P)); CK(dalloc(h, S_KB, &h->kb, P)); CK(dalloc(h, S_VB, &h->vb, P));
    CK(dalloc(h, S_ETXN, &h->e_txn, P)); CK(dalloc(h, S_SPOS, &h->spos, P)); CK(dalloc(h, S_EMETA, &h->e_meta, P));
    CK(dalloc(h, S_EEXEC, &h->e_exec1, P)); CK(dalloc(h, S_PMW, &h->pm_w, P)); CK(dalloc(h, S_PMC, &h->pm_c, P));
    CK(dalloc(h, S_SEG, &h->seg_start, P)); CK(dalloc(h, S_UD, &h->ud_prev, P));
    CK(dalloc(h, S_CNT, &h->cnt, (size_t)nvc * P)); CK(dalloc(h, S_DST, &h->dst, (size_t)nvc * P));
    CK(dalloc(h, S_NK, &h->nk, (size_t)nvc * n + n)); CK(dalloc(h, S_NE, &h->ne, (size_t)nvc * n + n));
    CK(dalloc(h, S_LVL, &h->lvl, n + 1)); CK(dalloc(h, S_ORDER, &h->order, n + 1));
    size_t sc = std::max<size_t>(1 << 20, 3 * (radix_hist_len(std::max(P, n)) + 128) * 4 + 64 * 1024);
    sc = std::max(sc, device_scan_scratch<ElideOp>(std::max(P, n)) + 4096);
    sc = std::max(sc, level_scratch_bytes(n, P));
    CK(ensure_scratch(h, sc));
    HIPCHK(h, hipStreamSynchronize(st));
    h->loaded = true;
    return AD_OK;
}

int ad_preaccept_deps(ad_handle* h, ad_csr_sizes* sizes) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "no batch loaded");
    hipSetDevice(h->device);
    CK(stage_prepare(h));
    CK(stage_sort(h));
    CK(stage_deps(h));
    if (sizes) {
        const int nv = (int)h->cfg.replicas;
        for (int v = 0; v < nv; ++v) {
            CK(csr_sizes(h, h->deps[2 * v], &sizes[v * AD_NUM_CLASSES + 0]));
            CK(csr_sizes(h, h->deps[2 * v + 1], &sizes[v * AD_NUM_CLASSES + 1]));
            sizes[v * AD_NUM_CLASSES + 2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
        }
    }
    return AD_OK;
}

static int fetch_empty(ad_handle* h, ad_csr_out* out) {
    for (size_t i = 0; i <= h->n; ++i) { out->key_off[i] = 0; out->k2t_off[i] = 0; out->txn_off[i] = 0; }
    return AD_OK;
}

int ad_fetch_deps(ad_handle* h, uint32_t view, uint32_t cls, ad_csr_out* out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "no deps computed");
    if (view >= h->cfg.replicas || cls >= AD_NUM_CLASSES) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (cls == AD_CLASS_RANGE) return fetch_empty(h, out);
    return fetch_csr(h, h->deps[2 * view + cls], out);
}

int ad_merge_deps(ad_handle* h, ad_csr_sizes* sizes) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    hipSetDevice(h->device);
    CK(stage_merge(h));
    if (sizes) {
        CK(csr_sizes(h, h->merged[0], &sizes[0]));
        CK(csr_sizes(h, h->merged[1], &sizes[1]));
        sizes[2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
    }
    return AD_OK;
}

int ad_fetch_merged(ad_handle* h, uint32_t cls, ad_csr_out* out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "no merged deps");
    if (cls >= AD_NUM_CLASSES) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (cls == AD_CLASS_RANGE) return fetch_empty(h, out);
    return fetch_csr(h, h->merged[cls], out);
}

int ad_merge_host(ad_handle* h, const ad_csr_in*, uint32_t, ad_csr_sizes*) {
    return h ? set_err(h, AD_ERR_UNSUPPORTED, "ad_merge_host: not in this build") : AD_ERR_ARGUMENT;
}

int ad_exec_levels(ad_handle* h, uint32_t* level_out, uint32_t* order_out, uint32_t* iterations_out) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    hipSetDevice(h->device);
    CK(stage_levels(h, order_out != nullptr));
    hipStream_t st = h->st;
    if (level_out && h->n) HIPCHK(h, hipMemcpyAsync(level_out, h->lvl, h->n * 4, hipMemcpyDeviceToHost, st));
    if (order_out && h->n) HIPCHK(h, hipMemcpyAsync(order_out, h->order, h->n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (iterations_out) *iterations_out = h->level_iters;
    return AD_OK;
}

int ad_run_pipeline(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "no batch loaded");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    HIPCHK(h, hipEventRecord(h->ev[0], st));
    CK(stage_prepare(h));
    HIPCHK(h, hipEventRecord(h->ev[1], st));
    CK(stage_sort(h));
    HIPCHK(h, hipEventRecord(h->ev[2], st));
    CK(stage_deps(h));
    HIPCHK(h, hipEventRecord(h->ev[3], st));
    CK(stage_merge(h));
    HIPCHK(h, hipEventRecord(h->ev[4], st));
    CK(stage_levels(h, true));
    HIPCHK(h, hipEventRecord(h->ev[5], st));
    HIPCHK(h, hipEventSynchronize(h->ev[5]));
    float ms;
    hipEventElapsedTime(&ms, h->ev[0], h->ev[1]); h->times.prepare = ms;
    hipEventElapsedTime(&ms, h->ev[1], h->ev[2]); h->times.sort = ms;
    hipEventElapsedTime(&ms, h->ev[2], h->ev[3]); h->times.deps = ms;
    hipEventElapsedTime(&ms, h->ev[3], h->ev[4]); h->times.merge = ms;
    hipEventElapsedTime(&ms, h->ev[4], h->ev[5]); h->times.levels = ms;
    hipEventElapsedTime(&ms, h->ev[0], h->ev[5]); h->times.total = ms;
    h->times.deps_entries = h->deps_entries;
    h->times.merged_entries = h->merged_entries;
    h->times.level_iterations = h->level_iters;
    h->times.level_edges = h->P;
    h->tracer.resolve();
    return AD_OK;
}

int ad_last_times(ad_handle* h, ad_stage_times* out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    *out = h->times;
    return AD_OK;
}

int ad_kernel_count(void) { return K_COUNT; }

const char* ad_kernel_name(int kid) { return kernel_name(kid); }

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

int ad_reset_kernel_stats(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    HIPCHK(h, hipStreamSynchronize(h->st));
    h->tracer.resolve();
    h->tracer.reset_counts();
    return AD_OK;
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
