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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "conflict_kernels.h"
#include "level_kernels.h"
#include "history_kernels.h"
#include "recovery_kernels.h"
#include "merge_kernels.h"
#include "radix_sort.h"
#include "shard_kernels.h"
#include "validate.h"

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
    uint32_t* totd = nullptr;          // device: gathered CSR totals (read_totals_params)
    int level_mode = AD_LEVELS_AUTO;
    bool order_pending = false;          // optimistic order issued; order_bad valid after a stream sync
    uint32_t order_bad = 0;
    size_t mrange_zero_n = ~(size_t)0;   // merged RangeDeps offsets known zero for this n / buffer
    const uint32_t* mrange_zero_p = nullptr;
    TsPack pack{};
    int key_bits = 0, range_bits = 0;
    uint64_t rbase = 0, wmax = 0;
    uint32_t n_large = 0;
    uint32_t n_special = 0;          // key-domain txns other than Read/Write (unmanaged execution)
    uint64_t *tx_ts = nullptr, *ex1 = nullptr;
    uint8_t* meta = nullptr;
    PairRec* prec = nullptr;
    uint32_t *ka = nullptr, *va = nullptr, *kb = nullptr, *vb = nullptr;
    uint32_t *skey = nullptr, *sval = nullptr;           // sorted (alias ka/kb)
    uint32_t *e_txn = nullptr, *nh = nullptr, *useg = nullptr;   // nh: non-head entries
    uint64_t* ukey = nullptr;
    uint8_t* e_meta = nullptr;
    uint64_t *e_exec1 = nullptr, *pm_w = nullptr, *pm_c = nullptr;
    int32_t *seg_start = nullptr, *ud_prev = nullptr;
    uint32_t *cnt = nullptr, *dst = nullptr, *nk = nullptr, *ne = nullptr;
    // virtual items (large txns)
    size_t V = 0;
    uint32_t *vn = nullptr, *voff = nullptr, *vi_txn = nullptr, *vi_pos = nullptr, *vi_u = nullptr;
    uint32_t* vcnt = nullptr;        // per (item, view x class): counts, rewritten in place into fill slots
    // range entries sorted by (start, end, owner)
    uint32_t *rowner = nullptr, *rk0 = nullptr, *rv0 = nullptr, *rk1 = nullptr, *rv1 = nullptr, *eown = nullptr;
    uint64_t *es = nullptr, *ee = nullptr;
    uint64_t* ri_nodes = nullptr;    // upper levels of the range index (range_index.h)
    RangeIndex ix{};
    uint32_t *rnk = nullptr, *rne = nullptr;
    void* scratch = nullptr;
    size_t scratch_cap = 0;
    std::vector<Csr> deps;           // [view * 2 + class]  (key, direct)
    Csr rdeps[MAXV];                 // RangeDeps per view
    Csr merged[3];
    Csr hparts[3][MAXV];             // ad_merge_host uploads
    // key-range sharding (shard_kernels.h)
    bool sharded = false;
    size_t n_global = 0;
    uint32_t* gid = nullptr;         // local row -> global arrival rank
    uint8_t* home = nullptr;         // local row is homed here (first key in this store's range)
    uint8_t* hstore = nullptr;       // local row -> its home store (destination of its fragment)
    uint32_t self = 0;               // this store's rank
    uint8_t* send = nullptr;         // per-destination blobs, concatenated in destination order
    size_t send_bytes = 0;
    std::vector<uint64_t> send_sizes;
    std::vector<uint64_t> send_hdr;  // host copy of the blob headers (outlives the async upload)
    uint8_t* recv = nullptr;         // per-source blobs (this store's home txns), concatenated
    uint32_t world = 0;
    size_t H = 0;                    // home txns
    uint32_t *home_rows = nullptr, *home_gid = nullptr, *G = nullptr;
    int32_t* src_rows = nullptr;     // [source * H + h]
    std::vector<Csr> src_csr;        // [source * nvc + vc] views into recv
    std::vector<uint32_t*> src_gid;
    std::vector<uint32_t> src_n;
    std::vector<Csr> sdeps;          // home-indexed per (view, class)
    Csr srdeps[MAXV];                // home-indexed RangeDeps per view (sources with range classes)
    Csr smerged[3];
    std::vector<uint8_t> src_ranges; // per source: its blob carries RangeDeps classes
    bool shard_ranges = false;       // the home merge produced RangeDeps (some source carried them)
    int32_t* none_rows = nullptr;    // [H] all -1: a source without RangeDeps classes
    ncclComm_t comm = nullptr;
    // delta level exchange (ad_shard_set_holders): per-row holder masks, per-destination send regions
    uint8_t* holders = nullptr;
    uint32_t *dbase_dev = nullptr, *dcnt_dev = nullptr;
    uint64_t* dout = nullptr;
    std::vector<uint32_t> dbase, dcnt;   // [world + 1] region starts; [world] last round's pair counts
    // MaxConflicts carried from earlier batches (ad_max_conflicts_carry): sorted keys + timestamps on the device
    size_t mc_m = 0;
    uint64_t *mc_ck = nullptr, *mc_cm = nullptr, *mc_cl = nullptr;
    int32_t* mc_cn = nullptr;
    bool mc_ready = false;           // the MaxConflicts scan of the current batch is on the device (export)
    const uint8_t* mc_fast = nullptr;  // [replicas * n] fast-path flags of the last ad_max_conflicts(_ts)
    bool have_deps = false, have_merged = false, have_levels = false, merged_has_range = false;
    int stage = 0;                   // STAGE_* while a stage allocates (what an allocation failure may evict)
    bool evicting = false;
    bool merge_heavy = true;         // Deps.merge may meet heavy txns (false: the deps stage saw none)
    bool accept = false;             // the deps stage runs with bound = executeAt (ad_accept_deps)
    // CFK history (history_kernels.h): kept rows of earlier batches, prepended to the next loaded batch
    bool hist_valid = false;         // ad_cfk_retain ran: the next ad_load_batch prepends hist_n rows
    size_t hist_n = 0, hist_p = 0;   // kept rows / their keys
    uint64_t hist_next = 0;          // global arrival rank of the next batch's first txn
    bool hist_active = false;        // the loaded batch's rows [0, hist_rows) are history; gid = global ranks
    size_t hist_rows = 0;
    uint32_t* qpos = nullptr;        // [n] arrival position of each txn's executeAt (accept bound)
    // BeginRecovery queries (recovery_kernels.h): outputs of the last ad_recover
    size_t rc_nq = 0;
    bool rc_ready = false;
    uint32_t* rc_off = nullptr;      // [RC_OUT][nq + 1]
    uint8_t* rc_rej = nullptr;
    uint64_t* rc_keys[RC_OUT] = {};
    uint32_t* rc_txn[RC_OUT] = {};
    // levels
    uint32_t *lvl = nullptr, *order = nullptr;
    uint32_t level_iters = 0;
    LevelState ls{};
    // host-mapped publish buffer (read_totals_params): small results written by a kernel, polled by the host
    uint32_t* pub_host = nullptr;    // hipHostMalloc(mapped, coherent): [0] sequence, totals, Params
    uint32_t* pub_dev = nullptr;     // its device address
    uint32_t pub_seq = 0;
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

enum Stage { STAGE_NONE = 0, STAGE_DEPS, STAGE_MERGE };
void release_dead(ad_handle* h);

// Grow-only device allocation slot `slot` of at least `bytes`.  When HBM is exhausted, the buffers the
// running stage makes dead (release_dead) are given back once and the allocation retried.
template <class T>
int dalloc(ad_handle* h, size_t slot, T** out, size_t count) {
    if (h->bufs.size() <= slot) h->bufs.resize(slot + 1);
    size_t bytes = std::max<size_t>(count * sizeof(T), 256);
    if (h->bufs[slot].cap < bytes) {
        DBuf& b = h->bufs[slot];
        if (b.p) { HIPCHK(h, hipStreamSynchronize(h->st)); HIPCHK(h, hipFree(b.p)); b.p = nullptr; b.cap = 0; }
        size_t nb = std::max(bytes, b.cap + b.cap / 4);
        void* p = nullptr;
        if (hipMalloc(&p, nb) != hipSuccess) {
            (void)hipGetLastError();
            if (h->stage != STAGE_NONE && !h->evicting) {
                h->evicting = true;
                release_dead(h);
                h->evicting = false;
                if (hipMalloc(&p, nb) != hipSuccess) { (void)hipGetLastError(); p = nullptr; }
            } else {
                p = nullptr;
            }
            if (!p) return set_err(h, AD_ERR_NOMEM, "device allocation of " + std::to_string(nb) + " bytes failed");
        }
        h->bufs[slot].p = p;
        h->bufs[slot].cap = nb;
    }
    *out = (T*)h->bufs[slot].p;
    return AD_OK;
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

enum Slot : size_t {
    S_TM, S_TL, S_TN, S_EM, S_EL, S_EN, S_ST, S_KOFF, S_KEYS, S_ROFF, S_RS, S_RE,
    S_PRM, S_TXTS, S_EX1, S_META, S_PTXN, S_KA, S_VA, S_KB, S_VB, S_ETXN, S_SPOS, S_EMETA, S_EEXEC,
    S_PMW, S_PMC, S_SEG, S_UD, S_CNT, S_DST, S_NK, S_NE, S_SCRATCH,
    S_LVL, S_ORDER, S_UIDX, S_UKEY, S_USEG, S_VN, S_VOFF, S_VTXN, S_VPOS, S_VSEG, S_VCNT,
    S_ROWN, S_RK0, S_RV0, S_RK1, S_RV1, S_ES, S_EE, S_EOWN, S_RNK, S_RNE, S_MSCR,
    S_GID, S_HOME, S_SEND, S_RECV, S_HROWS, S_HGID, S_G, S_SROWS, S_TOT, S_HSTORE, S_XRANK, S_XLIST, S_XOFF,
    S_XBND, S_XSEC, S_OVF, S_OVFL, S_OVFT, S_OVFN, S_OVFG, S_OVFO, S_MHL,
    S_MCPE, S_MCPR, S_MCINV, S_MCRANK, S_MCFAST, S_MCLOCAL, S_MCCK, S_MCCM, S_MCCL, S_MCCN,
    S_MCOM, S_MCOL, S_MCON, S_MCOF, S_MCSK, S_MCSM, S_MCSL, S_MCSN, S_MCSU, S_MCSP,
    S_MCEK, S_MCEM, S_MCEL, S_MCEN, S_FASTROWS, S_HOLD, S_DBASE, S_DCNT, S_DOUT, S_DMAT, S_DRECV, S_QPOS,
    S_HTM, S_HTL, S_HTN, S_HEM, S_HEL, S_HEN, S_HST, S_HKOFF, S_HKEYS, S_HGIDS, S_HSEGM, S_HKEEP, S_HROWS2, S_HCNT,
    S_RCROWS, S_RCCNT, S_RCOFF, S_RCREJ, S_RCK0, S_RCT0 = S_RCK0 + RC_OUT, S_RCEND = S_RCT0 + RC_OUT,
    S_RIDX = S_RCEND, S_NONEROWS, S_LROWS, S_UMEDC, S_UMED,
    S_NUM_FIXED,
    S_CSR0 = 160
};
static_assert(S_NUM_FIXED <= S_CSR0, "fixed device slots overlap the CSR slot blocks");
// CSR slot blocks (10 slots each): key-class CSRs [0, NVC_MAX), range CSRs [NVC_MAX, NVC_MAX + MAXV),
// merged [NVC_MAX + MAXV, +3)
constexpr size_t CSR_RANGE0 = NVC_MAX, CSR_MERGED0 = NVC_MAX + MAXV, CSR_HOST0 = CSR_MERGED0 + 3;
constexpr size_t CSR_SHARD0 = CSR_HOST0 + 3 * MAXV, CSR_SMERGED0 = CSR_SHARD0 + NVC_MAX, CSR_SRANGE0 = CSR_SMERGED0 + 3;

#define CK(x) do { int rc_ = (x); if (rc_ != AD_OK) return rc_; } while (0)

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
        h->mrange_zero_p = nullptr;
        h->mrange_zero_n = ~(size_t)0;
    }
    free_level_state(h->ls);
    h->have_levels = false;
}

inline int bits_of(uint64_t x) { return x == 0 ? 0 : 64 - __builtin_clzll(x); }

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

// Device-wide scan over h->scratch (scan.h: tile reduce, aggregate scan, apply).  A single-pass decoupled
// look-back variant measured slower on MI355X (ElideOp over 4M entries: 0.119 vs 0.092 ms; the radix
// digit scans 16 vs 12 us): the per-tile status must be read coherently across the 8 XCDs' L2s, so
// every look-back hop is a memory round trip.
template <class Op>
void scan_any(ad_handle* h, const Op& op, size_t n) {
    device_scan(op, n, (typename Op::S*)h->scratch, h->st);
}

template <class T>
void scan_offsets(ad_handle* h, const T* in, T* out, size_t n) {
    if (n == 0) { hipMemsetAsync(out, 0, sizeof(T), h->st); return; }
    scan_any(h, SumOp<T>{in, out, n}, n);
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
constexpr int MAX_TOTALS = 96;
constexpr int PUB_PRM = 4;                                  // Params words start here
constexpr int PUB_TOT = PUB_PRM + (int)(sizeof(Params) + 3) / 4;
constexpr int PUB_WORDS = PUB_TOT + MAX_TOTALS;
struct TotTable { const uint32_t* src[MAX_TOTALS]; int count; };
__global__ void k_collect_totals(TotTable t, uint32_t* out) {
    const int i = threadIdx.x;
    if (i < t.count) out[i] = *t.src[i];
}
__global__ __launch_bounds__(128) void k_publish(TotTable t, const Params* __restrict__ prm, uint32_t* pub, uint32_t seq) {
    const int i = threadIdx.x;
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
int read_totals_params(ad_handle* h, const TotTable& t, uint32_t* host) {
    if (pub_ready(h) != AD_OK) {        // no mapped memory: copy + stream sync
        if (t.count > 0) {
            k_collect_totals<<<1, MAX_TOTALS, 0, h->st>>>(t, h->totd);
            HIPCHK(h, hipMemcpyAsync(host, h->totd, (size_t)t.count * 4, hipMemcpyDeviceToHost, h->st));
        }
        HIPCHK(h, hipMemcpyAsync(&h->hprm, h->prm, sizeof(Params), hipMemcpyDeviceToHost, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
        return AD_OK;
    }
    const uint32_t seq = ++h->pub_seq;
    k_publish<<<1, 128, 0, h->st>>>(t, h->prm, h->pub_dev, seq);
    HIPCHK(h, hipGetLastError());
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
    if (t.count > 0) std::memcpy(host, h->pub_host + PUB_TOT, (size_t)t.count * 4);
    std::memcpy(&h->hprm, h->pub_host + PUB_PRM, sizeof(Params));
    return AD_OK;
}
// the level stage's flag read-backs share the handle's mapped buffer (the totals region)
static void set_level_pub(ad_handle* h) {
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
    return AD_OK;
}

// ---------------------------------------------------------------------------------------------------
// prepare + sort
// ---------------------------------------------------------------------------------------------------
int stage_prepare(ad_handle* h) {
    const size_t n = h->n, P = h->P, Q = h->Q;
    hipStream_t st = h->st;
    k_params_init<<<1, 1, 0, st>>>(h->prm);
    const int g = (int)std::min<size_t>(1024, std::max<size_t>(1, (std::max(std::max(n, P), Q) + 255) / 256));
    {
        KScope ks(K_MINMAX, n);
        unsigned long long* partial = (unsigned long long*)h->scratch;
        k_minmax<<<g, 256, 0, st>>>(n, h->tm, h->tl, h->tn, h->em, h->el, h->en, h->key_off, h->keys, P, h->range_s, h->range_e, Q, partial);
        k_minmax_final<<<1, 256, 0, st>>>(g, partial, h->prm);
    }
    CK(read_params(h));
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
    KScope ks(K_PACK, n);
    k_pack<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->pack, P ? p.key_min : 0, h->tm, h->tl, h->tn, h->em, h->el, h->en,
                                                    h->status, h->key_off, h->keys, Q ? h->range_off : nullptr, h->range_s,
                                                    h->range_e, h->tx_ts, h->ex1, h->meta, h->prec, h->ka, h->va, h->prm);
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

// ---------------------------------------------------------------------------------------------------
// deps
// ---------------------------------------------------------------------------------------------------
template <int NV>
void launch_walk(const WalkArgs& a, bool fill, hipStream_t st) {
    if (a.P > 0) {
        const int g = ceil_div((long)a.P, 256);
        KScope ks(fill ? K_WALK_FILL : K_WALK_COUNT, a.P);
        if (fill) k_deps_walk<NV, true><<<g, 256, 0, st>>>(a);
        else k_deps_walk<NV, false><<<g, 256, 0, st>>>(a);
    }
    if (a.V > 0) {
        const int g = ceil_div((long)a.V, 256);
        KScope ks(K_VITEMS);
        if (fill) k_vitem_walk<NV, true><<<g, 256, 0, st>>>(a);
        else k_vitem_walk<NV, false><<<g, 256, 0, st>>>(a);
    }
}
template <int NV>
void launch_range(const RangeArgs& a, bool fill, hipStream_t st) {
    const int g = ceil_div((long)a.n * WAVE, 256);
    KScope ks(K_RANGE);
    if (fill) k_range_deps<NV, true><<<g, 256, 0, st>>>(a);
    else k_range_deps<NV, false><<<g, 256, 0, st>>>(a);
}
#define NV_DISPATCH(nv, F, ...)                      \
    switch (nv) {                                    \
        case 1: F<1>(__VA_ARGS__); break;            \
        case 2: F<2>(__VA_ARGS__); break;            \
        case 3: F<3>(__VA_ARGS__); break;            \
        case 4: F<4>(__VA_ARGS__); break;            \
        case 5: F<5>(__VA_ARGS__); break;            \
        case 6: F<6>(__VA_ARGS__); break;            \
        case 7: F<7>(__VA_ARGS__); break;            \
        default: F<8>(__VA_ARGS__); break;           \
    }

// Capacity (elements) of CSR block `block`'s data buffers as currently allocated (0 if none).
size_t csr_cap(ad_handle* h, size_t block, int which, size_t elem) {
    const size_t slot = S_CSR0 + 10 * block + which;
    return slot < h->bufs.size() ? h->bufs[slot].cap / elem : 0;
}

// Offsets of every key-class CSR in one scan; with buffers left by an earlier batch, also the per-txn
// layout (fused; *overflow reports rows that did not fit, then k_txn_layout runs after sizing).
template <int NV>
void launch_offsets(ad_handle* h, const TxnArgs& ta, uint32_t* overflow) {
    OffsetsOp<2 * NV> op{};
    op.n = h->n; op.meta = h->meta; op.key_off = h->key_off; op.cnt = h->cnt;
    op.layout = 1;
    op.keys = h->keys; op.dst = h->dst; op.overflow = overflow;
    op.lsum_k = h->nk; op.lsum_e = h->ne; op.heavy = overflow - 1;
    for (int c = 0; c < 2 * NV; ++c) {
        op.o_key_off[c] = h->deps[c].key_off; op.o_ent_off[c] = h->deps[c].ent_off; op.o_k2t_off[c] = h->deps[c].k2t_off;
        const size_t base = S_CSR0 + 10 * (size_t)c;
        const size_t ck = csr_cap(h, c, 4, 8), cm = csr_cap(h, c, 5, 4);
        op.out_keys[c] = ck ? (uint64_t*)h->bufs[base + 4].p : nullptr;
        op.out_k2t[c] = cm ? (int32_t*)h->bufs[base + 5].p : nullptr;
        op.cap_keys[c] = (uint32_t)std::min<size_t>(ck, 0xFFFFFFFFu);
        op.cap_k2t[c] = (uint32_t)std::min<size_t>(cm, 0xFFFFFFFFu);
    }
    scan_any(h, op, h->n);
    (void)ta;
}

__global__ void k_ovf_sizes(uint32_t count, const uint2* items, const uint32_t* const* key_off, const uint32_t* const* k2t_off,
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

template <int NV>
void launch_large_sums(const TxnArgs& ta, hipStream_t st) {
    k_large_sums<2 * NV><<<ceil_div((long)ta.n * WAVE, 256), 256, 0, st>>>(ta);
}
template <int NV>
void launch_large_layout(const TxnArgs& ta, hipStream_t st) {
    k_large_layout<2 * NV><<<ceil_div((long)ta.n * WAVE, 256), 256, 0, st>>>(ta);
}

template <int NV>
void launch_union(const UnionArgs& ua, hipStream_t st) {
    k_txn_union<2 * NV><<<ceil_div((long)ua.n, 256), 256, 0, st>>>(ua);
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

struct StageScope {
    ad_handle* h;
    StageScope(ad_handle* x, int st) : h(x) { h->stage = st; }
    ~StageScope() { h->stage = STAGE_NONE; }
};

// Accept / GetDeps bound: per txn the number of batch TxnIds below its executeAt (TxnIds and executeAts share
// one packed order; tx_ts ascends with the batch).
__global__ __launch_bounds__(256) void k_query_pos(size_t n, const uint64_t* __restrict__ tx_ts, const uint64_t* __restrict__ ex1,
                                                   uint32_t* __restrict__ qpos) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t e = ex1[i] - 1;
    size_t lo = i, hi = n;              // executeAt >= TxnId
    while (lo < hi) { const size_t m = (lo + hi) >> 1; if (tx_ts[m] < e) lo = m + 1; else hi = m; }
    qpos[i] = (uint32_t)lo;
}

int stage_deps(ad_handle* h) {
    StageScope sc(h, STAGE_DEPS);
    const size_t n = h->n, P = h->P, Q = h->Q;
    const int nv = (int)h->cfg.replicas, nvc = 2 * nv;
    hipStream_t st = h->st;
    h->deps.resize(nvc);
    for (int vc = 0; vc < nvc; ++vc) CK(alloc_csr(h, vc, h->deps[vc], n));
    for (int v = 0; v < nv; ++v) CK(alloc_csr(h, CSR_RANGE0 + v, h->rdeps[v], n));
    if (P > 0) {
        { KScope ks(K_GATHER, P); k_gather_entries<<<ceil_div((long)P, 256), 256, 0, st>>>(P, h->sval, h->prec, h->e_txn, h->e_meta, h->e_exec1); }
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
        if (n) k_query_pos<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->tx_ts, h->ex1, h->qpos);
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
        CK(dalloc(h, S_VCNT, &h->vcnt, (size_t)V * nvc));
        va.vi_txn = h->vi_txn; va.vi_pos = h->vi_pos; va.vi_u = h->vi_u;
        if (V > 0) k_vitems<true><<<ceil_div((long)n, 256), 256, 0, st>>>(va);
    }
    // ---- walk (count)
    WalkArgs wa{};
    wa.e_txn = h->e_txn; wa.e_meta = h->e_meta; wa.e_exec1 = h->e_exec1; wa.seg_start = h->seg_start;
    wa.ud_prev = h->ud_prev; wa.pm_w = h->pm_w; wa.pm_c = h->pm_c; wa.tx_ts = h->tx_ts; wa.meta = h->meta; wa.P = P;
    wa.window = h->cfg.window; wa.thresh = ad_drop_threshold(h->cfg.drop_p); wa.seed = h->cfg.seed;
    wa.gid = (h->sharded || h->hist_active) ? h->gid : nullptr;
    wa.nh = h->nh; wa.prm = h->prm;
    wa.sval = h->sval; wa.cnt = h->cnt; wa.dst = h->dst;
    wa.V = h->V; wa.vi_txn = h->vi_txn; wa.vi_pos = h->vi_pos; wa.vi_u = h->vi_u; wa.useg = h->useg;
    wa.vcnt = h->vcnt; wa.vdst = h->vcnt;
    wa.qpos = qpos; wa.ex1 = h->ex1;
    if (P > 0) HIPCHK(h, hipMemsetAsync(h->cnt, 0, (size_t)nvc * P * 4, st));   // segment heads keep zero counts
    NV_DISPATCH(nv, launch_walk, wa, false, st);
    TxnArgs ta{};
    ta.n = n; ta.P = P; ta.nvc = nvc; ta.key_off = h->key_off; ta.keys = h->keys; ta.meta = h->meta; ta.cnt = h->cnt;
    ta.nk = h->nk; ta.ne = h->ne; ta.dst = h->dst; ta.prm = h->prm;
    ta.voff = h->voff; ta.vcnt = h->vcnt; ta.vdst = h->vcnt; ta.vi_u = h->vi_u; ta.ukey = h->ukey;
    uint32_t* overflow = h->totd + MAX_TOTALS - 1;       // fused-layout overflow flag (read with the totals)
    if (n > 0 && h->V > 0) {
        KScope ks(K_VITEMS);
        NV_DISPATCH(nv, launch_large_sums, ta, st);
    }
    if (n > 0) {
        HIPCHK(h, hipMemsetAsync(overflow - 1, 0, 8, st));     // [heavy-merge hint, layout overflow]
        KScope ks(K_SCAN_OFFSETS, n);
        NV_DISPATCH(nv, launch_offsets, h, ta, overflow);
    } else {
        for (int vc = 0; vc < nvc; ++vc) csr_offsets(h, h->deps[vc], h->nk, h->ne);
    }
    // ---- RangeDeps (count)
    RangeArgs ra{};
    ra.n = n; ra.Q = Q; ra.key_off = h->key_off; ra.keys = h->keys; ra.range_off = h->range_off; ra.rs = h->range_s;
    ra.re = h->range_e; ra.meta = h->meta; ra.es = h->es; ra.ee = h->ee; ra.eown = h->eown; ra.ix = h->ix;
    ra.window = h->cfg.window; ra.thresh = wa.thresh; ra.seed = h->cfg.seed; ra.rnk = h->rnk; ra.rne = h->rne;
    ra.qpos = qpos;
    ra.gid = wa.gid;
    if (Q > 0 && n > 0) {
        NV_DISPATCH(nv, launch_range, ra, false, st);
        for (int v = 0; v < nv; ++v) csr_offsets(h, h->rdeps[v], h->rnk + (size_t)v * n, h->rne + (size_t)v * n);
    }
    // ---- sizes -> host (one sync), allocate outputs
    const int ncsr = nvc + nv;
    std::vector<uint32_t> tot(3 * ncsr, 0);
    auto csr_at = [&](int c) -> Csr& { return c < nvc ? h->deps[c] : h->rdeps[c - nvc]; };
    TotTable tt{};
    for (int c = 0; c < (Q > 0 ? ncsr : nvc); ++c) {
        Csr& x = csr_at(c);
        tt.src[3 * c + 0] = x.key_off + n; tt.src[3 * c + 1] = x.k2t_off + n; tt.src[3 * c + 2] = x.ent_off + n;
        tt.count = 3 * c + 3;
    }
    const int ncol = tt.count;
    tt.src[tt.count++] = overflow;
    tt.src[tt.count++] = overflow - 1;
    std::vector<uint32_t> got(tt.count, 0);
    CK(read_totals_params(h, tt, got.data()));
    std::copy(got.begin(), got.begin() + ncol, tot.begin());
    const bool fused_layout = n > 0 && got[ncol] == 0;
    h->merge_heavy = n == 0 || got[ncol + 1] != 0 || h->n_large > 0 || Q > 0;
    CK(check_params(h));
    h->deps_entries = 0;
    for (int c = 0; c < ncsr; ++c) {
        Csr& x = csr_at(c);
        x.nkeys = tot[3 * c]; x.nk2t = tot[3 * c + 1]; x.ncap = tot[3 * c + 2];
        h->deps_entries += x.ncap;
        if (c < nvc) {
            CK(alloc_csr_data(h, c, x, 1));
            ta.out_key_off[c] = x.key_off; ta.out_k2t_off[c] = x.k2t_off; ta.out_keys[c] = x.keys; ta.out_k2t[c] = x.k2t;
            wa.k2t[c] = x.k2t;
        } else {
            CK(alloc_csr_data(h, CSR_RANGE0 + (c - nvc), x, 2));
            const int v = c - nvc;
            ra.key_off_v[v] = x.key_off; ra.k2t_off_v[v] = x.k2t_off; ra.keys_v[v] = x.keys; ra.k2t_v[v] = x.k2t;
        }
    }
    // ---- fill
    if (n > 0 && !fused_layout) { KScope ks(K_TXN_LAYOUT, P); k_txn_layout<<<ceil_div((long)n, 256), 256, 0, st>>>(ta); }
    if (n > 0 && h->V > 0) { KScope ks(K_VITEMS); NV_DISPATCH(nv, launch_large_layout, ta, st); }
    NV_DISPATCH(nv, launch_walk, wa, true, st);
    if (Q > 0 && n > 0) NV_DISPATCH(nv, launch_range, ra, true, st);
    UnionArgs ua{};
    ua.n = n; ua.nvc = nvc; ua.meta = h->meta;
    for (int vc = 0; vc < nvc; ++vc) {
        Csr& c = h->deps[vc];
        ua.key_off[vc] = c.key_off; ua.k2t_off[vc] = c.k2t_off; ua.ent_off[vc] = c.ent_off; ua.k2t[vc] = c.k2t;
        ua.txns[vc] = c.txns; ua.tcnt[vc] = c.tcnt;
    }
    if (n > 0) { KScope ks(K_TXN_UNION, n); NV_DISPATCH(nv, launch_union, ua, st); }
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
            la.ncsr = nvc; la.csr_base = 0; la.only_large = 1;
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
            k_union_lds<<<dim3((unsigned)h->n_large, (unsigned)nvc), UB, 0, st>>>(la);
            la.rows = nullptr; la.rows_total = nullptr;
        }
        if (Q > 0) {
            la.ncsr = nv; la.csr_base = nvc; la.only_large = 0;
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
            k_union_lds_small<<<dim3((unsigned)n, (unsigned)nv), US_T, 0, st>>>(la);
            k_union_lds_list<<<8192, UB, 0, st>>>(la);
        }
        CK(union_overflow(h, la, ovf_count, ovf, Q > 0));
    }
    // Virtual-item work arrays are dead once the CSRs are filled; they stay allocated for the next batch
    // (re-allocating C4's ~90 GB of them every batch cost more than the walks) unless the merge runs out of
    // HBM, when release_dead gives them back (STAGE_MERGE).
    h->have_deps = true;
    h->ls.chains_ready = false;
    h->times.deps_entries = h->deps_entries;
    h->times.level_edges = h->P;
    h->times.walk_items = (uint32_t)(h->P - (h->P ? h->hprm.n_keys_u : 0));
    return AD_OK;
}

// ---------------------------------------------------------------------------------------------------
// merge
// ---------------------------------------------------------------------------------------------------
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
    if (n > 0) HIPCHK(h, hipMemsetAsync(hc, 0, (size_t)K * 4, st));
    std::vector<MergeArgs> ma(K);
    for (int k = 0; k < K; ++k) {
        CK(alloc_csr(h, out_block[k], *out[k], n));
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
        if (h->merge_heavy) { a.hlist = hl + (size_t)k * n; a.hcount = hc + k; }
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
    CK(read_totals_params(h, tt, tot.data()));
    CK(check_params(h));
    for (int k = 0; k < K; ++k) {
        Csr& m = *out[k];
        m.nkeys = tot[3 * k]; m.nk2t = tot[3 * k + 1]; m.ncap = tot[3 * k + 2];
        if (entries) *entries += m.nk2t - m.nkeys;
        CK(alloc_csr_data(h, out_block[k], m, kw[k]));
        MergeArgs& a = ma[k];
        a.o_key_off = m.key_off; a.o_keys = m.keys; a.o_k2t_off = m.k2t_off; a.o_k2t = m.k2t;
        a.o_ent_off = m.ent_off; a.o_txns = m.txns; a.o_tcnt = m.tcnt;
        if (n > 0) merge_launch(a, np, true, kw[k], st);
    }
    return AD_OK;
}

// Deps.merge of `np` parts per class into h->merged.  parts[cls][v] are batched per-txn CSRs over the loaded batch;
// view_rows[v] (nullable) maps txn -> row of part v, -1 = leave that reply out for the txn.
int merge_parts(ad_handle* h, const Csr* const parts[3][MAXV], int np, bool has_range, const int32_t* const* view_rows = nullptr) {
    const size_t n = h->n;
    h->merged_entries = 0;
    Csr* out[3];
    size_t blocks[3];
    int kw[3];
    const Csr* in[3][MAXV] = {};
    const int32_t* rows[3][MAXV] = {};
    int K = 0;
    for (int cls = 0; cls < 3; ++cls) {
        if (cls == AD_CLASS_RANGE && !has_range) {
            Csr& m = h->merged[cls];
            CK(alloc_csr(h, CSR_MERGED0 + cls, m, n));
            m.nkeys = m.nk2t = m.ncap = 0;
            // an empty merged RangeDeps: zero offsets, kept from the previous batch when still valid
            if (h->mrange_zero_n != n || h->mrange_zero_p != m.key_off) {
                HIPCHK(h, hipMemsetAsync(m.key_off, 0, (n + 1) * 4, h->st));
                HIPCHK(h, hipMemsetAsync(m.ent_off, 0, (n + 1) * 4, h->st));
                HIPCHK(h, hipMemsetAsync(m.k2t_off, 0, (n + 1) * 4, h->st));
                h->mrange_zero_n = n;
                h->mrange_zero_p = m.key_off;
            }
            continue;
        }
        if (cls == AD_CLASS_RANGE) h->mrange_zero_p = nullptr;     // about to be written
        out[K] = &h->merged[cls];
        blocks[K] = CSR_MERGED0 + cls;
        kw[K] = cls == AD_CLASS_RANGE ? 2 : 1;
        for (int v = 0; v < np; ++v) { in[K][v] = parts[cls][v]; rows[K][v] = view_rows ? view_rows[v] : nullptr; }
        ++K;
    }
    CK(merge_multi(h, n, K, out, blocks, kw, in, view_rows ? rows : nullptr, np, &h->merged_entries));
    h->have_merged = true;
    return AD_OK;
}

int stage_merge(ad_handle* h) {
    StageScope sc(h, STAGE_MERGE);
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_merge_deps before ad_preaccept_deps");
    const int nv = (int)h->cfg.replicas;
    const Csr* parts[3][MAXV] = {};
    for (int v = 0; v < nv; ++v) {
        parts[0][v] = &h->deps[2 * v];
        parts[1][v] = &h->deps[2 * v + 1];
        parts[2][v] = &h->rdeps[v];
    }
    return merge_parts(h, parts, nv, h->Q > 0);
}

// ---------------------------------------------------------------------------------------------------
// levels
// ---------------------------------------------------------------------------------------------------
int stage_levels(ad_handle* h, bool want_order) {
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_exec_levels before ad_merge_deps");
    if (h->hist_active)
        return set_err(h, AD_ERR_UNSUPPORTED, "ad_exec_levels: the batch carries CFK history rows (already ordered in their own batch)");
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_exec_levels needs ad_preaccept_deps on this batch (its key chains)");
    LevelInputs li{};
    li.n = h->n; li.P = h->P; li.e_txn = h->e_txn; li.e_meta = h->e_meta; li.e_exec1 = h->e_exec1;
    li.seg_start = h->seg_start; li.sval = h->sval; li.nh = h->nh; li.prm = h->prm; li.key_off = h->key_off; li.meta = h->meta; li.ex1 = h->ex1;
    li.lvl = h->lvl; li.order = h->order;
    li.merged_key = &h->merged[AD_CLASS_KEY];
    li.merged_direct = &h->merged[AD_CLASS_DIRECT_KEY];
    li.ukey = h->ukey; li.useg = h->useg; li.U = h->P ? h->hprm.n_keys_u : 0;
    li.merged_range = &h->merged[AD_CLASS_RANGE];
    li.n_large = h->n_large;
    li.n_special = h->n_special;
    li.exec_bits = h->pack.total_bits;
    li.kahn_ok = h->level_mode != AD_LEVELS_FIXPOINT ? 1 : 0;
    li.force_blocks = h->level_mode == AD_LEVELS_BLOCKS ? 1 : 0;
    h->ls.pull_off = h->level_mode == AD_LEVELS_KAHN;
    h->ls.bl_rounds = 0;
    h->ls.bl_used = false;
    h->order_pending = false;
    h->order_bad = 0;
    li.order_verify = &h->order_bad;
    li.order_pending = &h->order_pending;
    int iters = 0;
    set_level_pub(h);
    int rc = run_levels(h->ls, li, want_order, h->st, &iters, h->err);
    if (rc != AD_OK) return rc;
    h->level_iters = (uint32_t)iters;
    h->times.level_rounds = h->ls.bl_rounds;
    h->times.level_blocks = h->ls.bl_used ? h->ls.bl.nblocks : 0;
    h->have_levels = true;
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
    if (h->comm) ncclCommDestroy(h->comm);
    if (h->st) hipStreamSynchronize(h->st);
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
    // working buffers
    const int nv = (int)h->cfg.replicas, nvc = 2 * nv;
    CK(dalloc(h, S_PRM, &h->prm, 1)); CK(dalloc(h, S_TOT, &h->totd, MAX_TOTALS));
    CK(dalloc(h, S_TXTS, &h->tx_ts, n)); CK(dalloc(h, S_EX1, &h->ex1, n)); CK(dalloc(h, S_META, &h->meta, n));
    CK(dalloc(h, S_PTXN, &h->prec, P));
    CK(dalloc(h, S_KA, &h->ka, P)); CK(dalloc(h, S_VA, &h->va, P)); CK(dalloc(h, S_KB, &h->kb, P)); CK(dalloc(h, S_VB, &h->vb, P));
    CK(dalloc(h, S_ETXN, &h->e_txn, P)); CK(dalloc(h, S_EMETA, &h->e_meta, P));
    CK(dalloc(h, S_EEXEC, &h->e_exec1, P)); CK(dalloc(h, S_PMW, &h->pm_w, P)); CK(dalloc(h, S_PMC, &h->pm_c, P));
    CK(dalloc(h, S_SEG, &h->seg_start, P)); CK(dalloc(h, S_UD, &h->ud_prev, P));
    CK(dalloc(h, S_UIDX, &h->nh, P)); CK(dalloc(h, S_UKEY, &h->ukey, P)); CK(dalloc(h, S_USEG, &h->useg, P + 1));
    CK(dalloc(h, S_CNT, &h->cnt, (size_t)nvc * P)); CK(dalloc(h, S_DST, &h->dst, (size_t)nvc * P));
    CK(dalloc(h, S_NK, &h->nk, (size_t)nvc * n + n)); CK(dalloc(h, S_NE, &h->ne, (size_t)nvc * n + n));
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
    HIPCHK(h, hipStreamSynchronize(st));
    h->loaded = true;
    return AD_OK;
}

static int run_deps(ad_handle* h, ad_csr_sizes* sizes, bool accept) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->loaded) return set_err(h, AD_ERR_STATE, "no batch loaded");
    if (accept && h->sharded) return set_err(h, AD_ERR_UNSUPPORTED, "ad_accept_deps: sharded stores answer PreAccept deps only");
    if (accept && h->hist_active) return set_err(h, AD_ERR_UNSUPPORTED, "ad_accept_deps: not over a CFK history batch");
    hipSetDevice(h->device);
    h->accept = accept;
    int rc = stage_prepare(h);
    if (rc == AD_OK) rc = stage_sort(h);
    if (rc == AD_OK) rc = stage_deps(h);
    h->accept = false;
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

static int fetch_empty(ad_handle* h, ad_csr_out* out) {
    for (size_t i = 0; i <= h->n; ++i) { out->key_off[i] = 0; out->k2t_off[i] = 0; out->txn_off[i] = 0; }
    return AD_OK;
}

// CommandStore.preaccept's maxConflicts.get(keys) per view (conflict_kernels.h), over the sorted entries the
// deps stage left on the device: leaves max_rank / fast (and the batch-local rank) in their slots.
static int run_max_conflicts(ad_handle* h, uint32_t** rank_out, uint8_t** fast_out, uint32_t** local_out) {
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "no deps computed");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
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

int ad_max_conflicts_ts(ad_handle* h, uint64_t* msb, uint64_t* lsb, int32_t* node, uint8_t* fast) {
    if (!h) return AD_ERR_ARGUMENT;
    if (h->Q > 0) return set_err(h, AD_ERR_UNSUPPORTED, "ad_max_conflicts_ts: the carried MaxConflicts map is per key (key batches)");
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
        c.local_rank = local; c.m = h->mc_m; c.ck = h->mc_ck; c.cm = h->mc_cm; c.cl = h->mc_cl; c.cn = h->mc_cn;
        c.om = om; c.ol = ol; c.on = on; c.fast = of;
        KScope ks(K_MAX_CONFLICTS);
        k_mc_carry<<<ceil_div((long)n, 256), 256, 0, st>>>(c);
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
    if (h->Q > 0) return set_err(h, AD_ERR_UNSUPPORTED, "ad_max_conflicts_export: the carried MaxConflicts map is per key (key batches)");
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

// BeginRecovery's store queries (recovery_kernels.h) for nq recovering rows, over the merged Deps on the handle:
// count pass, one scan for the six outputs' offsets, fill pass.  The outputs stay on the device for
// ad_fetch_recovery / ad_fetch_recovery_flags.
int ad_recover(ad_handle* h, const uint32_t* rows, size_t nq, size_t* entries) {
    if (!h || (nq && !rows)) return AD_ERR_ARGUMENT;
    if (!h->have_deps || !h->have_merged)
        return set_err(h, AD_ERR_STATE, "ad_recover needs the batch's deps and merged Deps (ad_merge_deps / _fast / ad_merge_host)");
    if (h->sharded) return set_err(h, AD_ERR_UNSUPPORTED, "ad_recover: not in sharded mode");
    for (size_t q = 0; q < nq; ++q)
        if (rows[q] >= h->n) return set_err(h, AD_ERR_ARGUMENT, "ad_recover: row " + std::to_string(rows[q]) + " out of range");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
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
        CK(csr_sizes(h, h->merged[0], &sizes[0]));
        CK(csr_sizes(h, h->merged[1], &sizes[1]));
        if (h->Q) CK(csr_sizes(h, h->merged[2], &sizes[2]));
        else sizes[2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
    }
    return AD_OK;
}

__global__ void k_fast_rows(size_t n, int nv, const uint8_t* __restrict__ fast, int32_t* __restrict__ rows) {
    const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x < n * (size_t)nv) rows[x] = fast[x] ? (int32_t)(x % n) : -1;
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
    CK(merge_parts(h, parts, nv, h->Q > 0, vr));
    h->merged_has_range = h->Q > 0;
    if (sizes) {
        CK(csr_sizes(h, h->merged[0], &sizes[0]));
        CK(csr_sizes(h, h->merged[1], &sizes[1]));
        if (h->Q) CK(csr_sizes(h, h->merged[2], &sizes[2]));
        else sizes[2] = ad_csr_sizes{h->n, 0, 0, 0, 0};
    }
    return AD_OK;
}

int ad_fetch_merged(ad_handle* h, uint32_t cls, ad_csr_out* out) {
    if (!h || !out) return AD_ERR_ARGUMENT;
    if (!h->have_merged) return set_err(h, AD_ERR_STATE, "no merged deps");
    if (cls >= AD_NUM_CLASSES) return AD_ERR_ARGUMENT;
    hipSetDevice(h->device);
    if (cls == AD_CLASS_RANGE) return h->merged_has_range ? fetch_csr(h, h->merged[2], 2, out) : fetch_empty(h, out);
    return fetch_csr(h, h->merged[cls], 1, out);
}

int ad_fetch_rows(ad_handle* h, uint32_t view, uint32_t cls, size_t lo, size_t hi, ad_csr_sizes* sizes, ad_csr_out* out) {
    if (!h || !sizes) return AD_ERR_ARGUMENT;
    if (cls >= AD_NUM_CLASSES || view > h->cfg.replicas) return set_err(h, AD_ERR_ARGUMENT, "view/class out of range");
    if (lo > hi || hi > h->n) return set_err(h, AD_ERR_ARGUMENT, "row range outside the batch");
    hipSetDevice(h->device);
    const Csr* c;
    if (view == h->cfg.replicas) {
        if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_fetch_rows of the merged Deps before ad_merge_deps");
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

// After a stream sync: if the optimistic execution order failed its verification, redo it on the
// general path (radix sort by executeAt) and wait for it.
int finish_order(ad_handle* h) {
    if (!h->order_pending) return AD_OK;
    h->order_pending = false;
    if (!h->order_bad) return AD_OK;
    order_rows(h->ls, h->n, nullptr, h->ex1, h->lvl, h->pack.total_bits, h->order, h->st);
    HIPCHK(h, hipStreamSynchronize(h->st));
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
    h->merged_has_range = h->Q > 0;
    HIPCHK(h, hipEventRecord(h->ev[4], st));
    CK(stage_levels(h, true));
    HIPCHK(h, hipEventRecord(h->ev[5], st));
    HIPCHK(h, hipEventSynchronize(h->ev[5]));
    if (h->order_pending && h->order_bad) {      // optimistic order failed its check: general path, timed in
        CK(finish_order(h));
        HIPCHK(h, hipEventRecord(h->ev[5], st));
        HIPCHK(h, hipEventSynchronize(h->ev[5]));
    }
    h->order_pending = false;
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
    h->times.walk_items = (uint32_t)(h->P - (h->P ? h->hprm.n_keys_u : 0));
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

int ad_set_level_mode(ad_handle* h, int mode) {
    if (!h || (mode != AD_LEVELS_AUTO && mode != AD_LEVELS_FIXPOINT && mode != AD_LEVELS_BLOCKS && mode != AD_LEVELS_KAHN))
        return AD_ERR_ARGUMENT;
    h->level_mode = mode;
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

// ---------------------------------------------------------------------------------------------------
// Key-range sharding across GPUs (shard_kernels.h)
// ---------------------------------------------------------------------------------------------------
static size_t align8(size_t x) { return (x + 7) & ~(size_t)7; }

int ad_cfk_retain(ad_handle* h, size_t* retained) {
    if (!h) return AD_ERR_ARGUMENT;
    if (!h->have_deps) return set_err(h, AD_ERR_STATE, "ad_cfk_retain: run ad_preaccept_deps on the batch first");
    if (h->sharded) return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_retain: not in sharded mode");
    if (h->Q) return set_err(h, AD_ERR_UNSUPPORTED, "ad_cfk_retain: key batches only (no range txns)");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
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
    hipStream_t st = h->st;
    const size_t n = h->n;
    // Unmanaged txns (range txns, key-domain sync points / ephemeral reads) and the key txns depending on range
    // txns also wait on their merged deps: rules (b) and (c).  Every such constraint is local to one store — a
    // dependency edge T -> D comes from a key or range slice both hold, a (c) bound from one key's chain — so
    // each store applies the ones it holds from the Deps.merge of its own replica views (the global merged
    // deps restricted to its keys), computed once per batch.
    const bool mixed = h->Q > 0 || h->n_special > 0 || h->n_large > 0;
    if (first && mixed) CK(stage_merge(h));
    CK(dalloc(h, S_G, &h->G, h->n_global + 1));
    uint32_t* flag = nullptr;
    CK(dalloc(h, S_NE, &flag, 16));
    if (first) HIPCHK(h, hipMemsetAsync(h->G, 0, (h->n_global + 1) * 4, st));
    else if (n) k_levels_gather<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->gid, h->G, h->lvl);
    LevelInputs li{};
    li.n = n; li.P = h->P; li.e_txn = h->e_txn; li.e_meta = h->e_meta; li.e_exec1 = h->e_exec1;
    li.seg_start = h->seg_start; li.sval = h->sval; li.nh = h->nh; li.prm = h->prm; li.key_off = h->key_off; li.meta = h->meta; li.ex1 = h->ex1;
    li.lvl = h->lvl; li.order = h->order;
    li.ukey = h->ukey; li.useg = h->useg; li.U = h->P ? h->hprm.n_keys_u : 0;
    if (mixed) {
        if (!h->have_merged) return set_err(h, AD_ERR_STATE, "ad_shard_levels_round: first round missing");
        li.merged_key = &h->merged[AD_CLASS_KEY];
        li.merged_direct = &h->merged[AD_CLASS_DIRECT_KEY];
        li.merged_range = &h->merged[AD_CLASS_RANGE];
    }
    li.n_large = mixed ? h->n_large : 0;
    li.n_special = mixed ? h->n_special : 0;
    li.exec_bits = h->pack.total_bits;
    li.keep_levels = first ? 0 : 1;
    int iters = 0;
    set_level_pub(h);
    CK(run_levels(h->ls, li, false, st, &iters, h->err));
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
    if (!h || !h->G || h->sdeps.empty()) return set_err(h, AD_ERR_STATE, "ad_shard_order: levels rounds + ad_shard_merge first");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    hipStream_t st = h->st;
    const size_t H = h->H, n = h->n;
    if (H == 0) return AD_OK;
    if (n) k_levels_gather<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->gid, h->G, h->lvl);
    uint32_t *ord, *tmp;
    CK(dalloc(h, S_ORDER, &ord, std::max(n, H) + 1));
    CK(dalloc(h, S_MSCR, &tmp, 2 * H + 2));
    order_rows(h->ls, H, h->home_rows, h->ex1, h->lvl, h->pack.total_bits, ord, st);
    k_home_gid<<<ceil_div((long)H, 256), 256, 0, st>>>(H, ord, h->home_gid, tmp);           // order -> global ids
    k_home_gid<<<ceil_div((long)H, 256), 256, 0, st>>>(H, h->home_rows, h->lvl, tmp + H);  // home levels
    if (order_out) HIPCHK(h, hipMemcpyAsync(order_out, tmp, H * 4, hipMemcpyDeviceToHost, st));
    if (level_out) HIPCHK(h, hipMemcpyAsync(level_out, tmp + H, H * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
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
