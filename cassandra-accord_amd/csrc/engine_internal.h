// engine_internal.h — the handle and the host-side helpers shared by the engine translation units
// (engine.hip: C-ABI, prepare/sort, fetch; deps.hip; merge.hip; levels.hip; shard.hip).
//
// One ad_handle = one CommandStore shard on one GPU: a HIP stream, a device arena and the loaded batch.
//   prepare   batch statistics, timestamp packing (ts64), pair owners, footprint checks   (deps_kernels.h)
//   sort      stable LSD radix sort of (key, pair); range entries by (start, end, owner)  (radix_sort.h)
//   deps      CFK elision scan, per-pair / per-virtual-item walks (count, fill), per-txn KeyDeps
//             layout, TxnId unions; RangeDeps interval join                               (deps/union/range)
//   merge     Deps.merge of the R replica views per txn, all three classes                (merge_kernels.h)
//   levels    execution levels over key chains + deps                                     (level_kernels.h)
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "conflict_kernels.h"
#include "level_kernels.h"
#include "history_kernels.h"
#include "invert_kernels.h"
#include "notify_kernels.h"
#include "cfk_store_kernels.h"
#include "seg_fuse_kernels.h"
#include "recovery_kernels.h"
#include "merge_kernels.h"
#include "radix_sort.h"
#include "shard_kernels.h"
#include "validate.h"


using namespace ad;

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
};

using Csr = ad::DevCsr;

constexpr size_t CSR_BLOCKS_MAX = 96;

// The handle's query model: replicas from ad_config; window / drop_p / seed from ad_replica_model (0: the snapshot)
struct ModelCfg {
    uint32_t window = 0;
    uint32_t replicas = 1;
    float drop_p = 0.0f;
    uint64_t seed = 0;
};

struct ad_handle {
    int device = 0;
    ModelCfg cfg{};                  // replicas (ad_config) + the replica model (ad_replica_model)
    hipStream_t st = nullptr;
    std::string err;
    // AD_HOST_TIMERS=1: host-side timestamps at marked points of ad_run_pipeline, printed to stderr per call
    // (where the host, not the device, sets the pace: the launch gaps in the kernel trace)
    int host_timers = -1;
    std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> ht;
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
    bool order_pending = false;          // optimistic order issued; its check (pub_host[1]) valid after a stream sync
    // CSRs whose offsets are known to be all zero (an empty class: directKeyDeps without sync points,
    // RangeDeps without range txns), per CSR block: valid while the buffer, n and the allocation
    // generation are unchanged, so steady-state batches skip re-zeroing them
    const uint32_t* zero_p[CSR_BLOCKS_MAX] = {};
    size_t zero_n[CSR_BLOCKS_MAX] = {};
    uint64_t zero_gen[CSR_BLOCKS_MAX] = {};
    uint64_t alloc_gen = 0;              // bumped by every device (re)allocation
    bool deps_direct = true;             // the last deps stage computed directKeyDeps classes
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
    uint8_t *cnt8 = nullptr, *dfr = nullptr;             // per (pair, class) byte counts; per txn deferred flag
    uint32_t *cntx = nullptr, *inl = nullptr;            // saturated counts; the walk's inline ids
    uint32_t *dst = nullptr, *nk = nullptr, *ne = nullptr;
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
    // one-exchange sharded levels (global_levels.h): this store's constraint edges, the gathered ones
    uint64_t* gl_edges = nullptr;
    size_t gl_m = 0;
    bool gl_ready = false;
    // delta level exchange (ad_shard_set_holders): per-row holder masks, per-destination send regions
    uint8_t* holders = nullptr;
    uint32_t *dbase_dev = nullptr, *dcnt_dev = nullptr;
    uint64_t* dout = nullptr;
    std::vector<uint32_t> dbase, dcnt;   // [world + 1] region starts; [world] last round's pair counts
    // distributed Kahn levels (ad_shard_kahn_*, kahn_shard_kernels.h)
    std::vector<uint8_t> home_host, holders_host;   // local row -> home store / holder mask (host copies)
    std::vector<uint32_t> ks_base;   // [2 * (MAX_STORES + 1)]: READY then RELEASE region starts per destination
    uint32_t *ks_base_dev = nullptr, *ks_cnt_dev = nullptr, *ks_rem = nullptr, *ks_rcnt = nullptr, *ks_flag = nullptr;
    uint32_t* ks_xs = nullptr;
    uint64_t *ks_out = nullptr, *ks_in = nullptr, *ks_xoff = nullptr;
    size_t ks_in_m = 0, ks_unreleased = 0;
    uint64_t ks_sent = 0;            // messages this batch sent to other stores
    uint32_t *ks_lacc = nullptr, *ks_plv = nullptr;   // per row: greatest READY level bound seen, predecessors' bound
    uint32_t* ks_head_dev = nullptr;  // per destination: READYs sent (ks_cnt_dev: appended)
    std::vector<uint32_t> ks_head_host;
    unsigned long long* ks_sent_dev = nullptr;         // ad_shard_kahn_run's READYs to other stores
    int ks_phase = -1;               // 0 after ad_shard_kahn_begin: the outbox holds the next wave's READYs
    bool ks_levels = false;          // lvl holds this batch's levels from the Kahn waves (ad_shard_order reads them)
    // MaxConflicts carried from earlier batches (ad_max_conflicts_carry): sorted keys + timestamps on the device
    size_t mc_m = 0;
    uint64_t *mc_ck = nullptr, *mc_cm = nullptr, *mc_cl = nullptr;
    int32_t* mc_cn = nullptr;
    size_t mci_m = 0;                // ... and its intervals (s, e] from range txns (ad_max_conflicts_carry_ranges)
    uint64_t *mci_s = nullptr, *mci_e = nullptr, *mci_cm = nullptr, *mci_cl = nullptr;
    int32_t* mci_cn = nullptr;
    uint64_t mci_lo = 0, mci_hi = 0;  // smallest start / greatest end
    // the rest of CommandStore.preaccept (ad_preaccept_expiry): rejectBefore intervals + the clock's timeout test
    size_t rb_m = 0;
    uint64_t *rb_s = nullptr, *rb_e = nullptr, *rb_cm = nullptr, *rb_cl = nullptr;
    int32_t* rb_cn = nullptr;
    int rb_clock = 0;
    uint64_t rb_now = 0, rb_timeout = 0;
    bool mc_ready = false;           // the MaxConflicts scan of the current batch is on the device (export)
    const uint8_t* mc_fast = nullptr;  // [replicas * n] fast-path flags of the last ad_max_conflicts(_ts)
    bool have_deps = false, have_merged = false, have_levels = false, merged_has_range = false;
    bool entries_partial = false;    // the deps stage skipped the lone entries' gather (complete_entries)
    bool seg_long = false;           // the loaded batch has a key segment too long for k_seg_fuse's tiles
    int cnt8_cleared = 0;            // count bytes per pair k_pack cleared for the next deps stage (0: none)
    bool want_union = false;         // ad_run_pipeline: the deps stage also builds the union view (the merged Deps)
    bool deps_union = false;         // the last deps stage did: deps[2R], deps[2R + 1] are the merged key classes
    bool pack_enqueued = false;      // stage_prepare: k_pack launched on the device Params (PackPlan)
    bool small_cleared = false;      // k_pack zeroed the deps stage's small counters (pack_clear_list)
    bool chains_pending = false;     // k_pack zeroed the pull pass's succ words and flags (ad_run_pipeline)
    bool chains_prebuilt = false;    // k_seg_fuse built the pull pass's chains (LevelInputs.chains_prebuilt)
    bool no_fused_chains = getenv("AD_NO_FUSED_CHAINS") != nullptr;   // A/B switch
    bool merged_exact = true;        // merged TxnId lists exact (k_merge); false: capacity regions + tcnt (union view)
    bool merged_compacted = false;   // !merged_exact: the exact offsets / lists below are built (merged_compact)
    bool in_pipeline = false;        // ad_run_pipeline's stage_prepare is running
    bool pipeline_union = false;     // ad_set_pipeline_union: ad_run_pipeline takes the union view (a generator shortcut)
    bool merged_cap = false;         // merged key classes as k_merge_ref's references + merged rows (merged_ready compacts)
    bool mcap_direct = false;        //   ... the directKeyDeps class too
    MergeCapArgs mcap_args[2] = {};  //   the last merge's references / merged-row region per class (merged_ready)
    uint32_t* mcap_part[2] = {};
    unsigned mcap_blocks = 0;
    int mcap_phase = 0;              //   which of the two counter sets this call uses
    bool mcap_entries_pending = false;   // merged_entries = the sum of mcap_part (read lazily)
    uint32_t* mx_off[3] = {};        //   per class: exact TxnId offsets [n + 1]
    uint32_t* mx_txns[3] = {};       //   and the compacted TxnId lists
    size_t mx_tot[3] = {};
    bool nh_valid = false;           // nh holds the batch's non-head entries (not after k_seg_fuse)
    bool keys_partial = false;       // k_seg_fuse left ukey / useg to complete_entries (from its tiles)
    bool state_partial = false;      // ... and the entry state (complete_entries: gather + ElideOp scan)
    size_t sf_ntiles = 0;
    int stage = 0;                   // STAGE_* while a stage allocates (what an allocation failure may evict)
    bool evicting = false;
    bool merge_heavy = true;         // Deps.merge may meet heavy txns (false: the deps stage saw none)
    bool accept = false;             // the deps stage runs with bound = executeAt (ad_accept_deps)
    bool bound_max = false;          // ... with bound = Timestamp.MAX (ad_ephemeral_read_deps)
    // ad_load_batch_async: the next batch's inputs on a copy stream into the staging slots
    hipStream_t cst = nullptr;
    hipStream_t xst = nullptr;       // side stream: k_txn_finish_ovf's latency-bound rows, overlapped with later stages
    hipEvent_t xev0 = nullptr, xev1 = nullptr;
    bool xjoin = false;              // work queued on xst that the main stream has not waited for
    bool merge_side = false;         // ad_run_pipeline: stage_merge may run k_merge_ref on xst beside the levels
    bool merge_sided = false;        // ... and did (ev[4] then marks its end on xst)
    bool xdefer = false;             // ad_run_pipeline: stage_deps leaves the join to the stages that read its CSRs
    hipEvent_t cev = nullptr, sev = nullptr;
    // ad_fetch_results_async: the results copied into a device staging buffer on st (fev0), paged out on fst (fev1)
    hipStream_t fst = nullptr;
    hipEvent_t fev0 = nullptr, fev1 = nullptr;
    bool fetch_pending = false;
    bool stage_pending = false;
    size_t stg_n = 0, stg_p = 0, stg_q = 0;
    // CFK history (history_kernels.h): kept rows of earlier batches, prepended to the next loaded batch
    bool hist_valid = false;         // ad_cfk_retain ran: the next ad_load_batch prepends hist_n rows
    size_t hist_n = 0, hist_p = 0;   // kept rows / their keys
    uint64_t hist_next = 0;          // global arrival rank of the next batch's first txn
    bool hist_active = false;        // the loaded batch's rows [0, hist_rows) are history; gid = global ranks
    size_t hist_rows = 0;
    uint32_t* qpos = nullptr;        // [n] arrival position of each txn's executeAt (accept bound)
    uint32_t* gqpos = nullptr;       // sharded stores: [n] the GLOBAL arrival position of each row's executeAt
    bool gq_ready = false;           // ad_shard_query_positions ran for the loaded batch
    // BeginRecovery queries (recovery_kernels.h): outputs of the last ad_recover
    size_t rc_nq = 0;
    bool rc_ready = false;
    uint32_t* rc_off = nullptr;      // [RC_OUT][nq + 1]
    uint8_t* rc_rej = nullptr;
    uint64_t* rc_keys[RC_OUT] = {};
    uint32_t* rc_txn[RC_OUT] = {};
    // device-resident CommandsForKey states (cfk_store_kernels.h, ad_cfk_store_*): K keys x cap byId rows
    struct CfkStore {
        uint32_t K = 0, cap = 0, words = 0;
        uint32_t ucap = 0;           // the caller's capacity (cap: rounded up to whole 64-slot words)
        uint32_t* cnt = nullptr;
        uint64_t *tm = nullptr, *tl = nullptr, *em = nullptr, *el = nullptr, *bits = nullptr;
        int32_t *tn = nullptr, *en = nullptr;
        uint8_t *st = nullptr, *out = nullptr;
        uint32_t *slot = nullptr, *pre = nullptr, *flags = nullptr;
        uint64_t *pbm = nullptr, *pbl = nullptr, *lpm = nullptr, *lpl = nullptr, *lp_bits = nullptr;  // pruning
        int32_t *pbn = nullptr, *lpn = nullptr;
        uint32_t* lp_cnt = nullptr;
        uint64_t *lp_xm = nullptr, *lp_xl = nullptr;                 // loadingPruned least witness TxnIds
        int32_t* lp_xn = nullptr;
        uint8_t* lp_xh = nullptr;
        uint32_t* um_cnt = nullptr;                                  // unmanaged registry
        uint8_t* um_p = nullptr;
        uint64_t *um_wm = nullptr, *um_wl = nullptr, *um_tm = nullptr, *um_tl = nullptr;
        int32_t *um_wn = nullptr, *um_tn = nullptr;
        uint32_t *nt_base = nullptr, *nt_cnt = nullptr, *nt_ev = nullptr;   // the last apply's notifications
        uint8_t* nt_tag = nullptr;
        uint64_t *nt_tm = nullptr, *nt_tl = nullptr;
        int32_t* nt_tn = nullptr;
        size_t nt_total = 0;
        std::vector<uint32_t> nt_base_host, ev_off_host;
        // the large tier (keys outgrowing cap): capB rows per slot, nbig slots, big_keys[slot] = its key
        uint32_t capB = 0, wordsB = 0, nbig = 0, ucapB = 0;
        uint32_t *kslot = nullptr, *kres = nullptr, *klist = nullptr, *kstart = nullptr, *kslots_new = nullptr;
        std::vector<uint32_t> kslot_host, big_keys;
        uint32_t rows_cap(uint32_t key) const { return kslot_host.empty() || kslot_host[key] == ~0u ? cap : capB; }
        uint32_t words_of(uint32_t key) const { return kslot_host.empty() || kslot_host[key] == ~0u ? words : wordsB; }
        size_t rbase(uint32_t key) const {
            return kslot_host.empty() || kslot_host[key] == ~0u ? (size_t)key * cap : (size_t)K * cap + (size_t)kslot_host[key] * capB;
        }
        size_t bbase(uint32_t key) const {
            return kslot_host.empty() || kslot_host[key] == ~0u ? (size_t)key * cap * words
                                                                : (size_t)K * cap * words + (size_t)kslot_host[key] * capB * wordsB;
        }
    } cs;
    // the last ad_cfk_store_query (cfk_query_kernels.h): capacity-laid outputs per class + exact counts on the host
    struct CfkQueryOut {
        bool ready = false;
        size_t nq = 0, items = 0, lists[2] = {0, 0};
        uint64_t* okeys[2] = {};
        int32_t* ok2t[2] = {};
        uint64_t *otm[2] = {}, *otl[2] = {};
        int32_t* otn[2] = {};
        uint32_t *okc[2] = {}, *oen[2] = {}, *otc[2] = {};
        std::vector<uint32_t> qoff, qe, kc[2], en[2], tc[2];
    } csq;
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

#define HIPCHK(h, x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            (h)->err = std::string(#x) + ": " + hipGetErrorString(e_);                 \
            return AD_ERR_DEVICE;                                                      \
        }                                                                              \
    } while (0)

int set_err(ad_handle* h, int code, const std::string& msg);
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
        ++h->alloc_gen;
    }
    *out = (T*)h->bufs[slot].p;
    return AD_OK;
}

// Releases slot `slot` (its next dalloc allocates afresh).
int drelease(ad_handle* h, size_t slot);

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
    S_GLCT, S_GLCM, S_GLCE, S_GLCP, S_GLLW, S_GLEC, S_GLEO, S_GLXC, S_GLXO, S_GLCONS, S_GLE, S_GLIN,
    S_GLSRC, S_GLDST, S_GLSRC2, S_GLDST2, S_GLDEG, S_GLREM, S_GLXOFF, S_GLFL, S_GLFRONT, S_GLKEY, S_CFKU,
    S_CNTX, S_INL, S_DFR, S_OVI, S_DTX, S_POSOF, S_GQPOS,
    S_MCIS, S_MCIE, S_MCIM, S_MCIL, S_MCIN,                     // carried MaxConflicts intervals
    S_MXX, S_MXK0, S_MXV0, S_MXK1, S_MXV1, S_MXF, S_MXR, S_MXU, S_MXVM, S_MXVL, S_MXVN, S_MXH, S_MXFS, S_MXFE,
    S_MXPS, S_MXPE, S_MXOS, S_MXOE, S_MXOM, S_MXOL, S_MXON,    // their export
    S_MHS,                                                      // heavy merge: identical-replies flags
    S_IVC, S_IVK0, S_IVV0, S_IVK1, S_IVV1, S_IVOUT,             // ad_fetch_inverse (invert_kernels.h)
    S_RBS, S_RBE, S_RBM, S_RBL, S_RBN,                          // rejectBefore intervals (ad_preaccept_expiry)
    S_NF0, S_NF_END = S_NF0 + 14,                               // ad_cfk_notify inputs / scratch / outputs
    S_STG0, S_STG_END = S_STG0 + 12,
    S_KSSRC, S_KSDST, S_KSSRC2, S_KSDST2, S_KSREM, S_KSXOFF, S_KSRCNT, S_KSFL, S_KSBASE, S_KSCNT, S_KSOUT,
    S_KSIN, S_KSMAT,                                            // distributed Kahn levels (ad_shard_kahn_*)
    S_KSLACC, S_KSPLV, S_KSHEAD, S_KSSENT, S_KSSTO, S_KSSTI, S_KSPEND,   // ... READY level bounds, queues, slots
    S_CSKSLOT, S_CSKRES, S_CSKLIST, S_CSKSTART, S_CSKNEW,                // CFK store large tier
    S_FOVFCM,                                                           // k_txn_finish_ovf's rows' classes
    S_FSTAGE,                                                           // ad_fetch_results_async staging
    S_CS0, S_CS_END = S_CS0 + 22,                               // resident CFK store (ad_cfk_store_*)
    S_CSE0, S_CSE_END = S_CSE0 + 14,                            // its event upload
    S_SFLO, S_SFCNT, S_FOVF, S_SFSEC,                                     // k_seg_fuse tiles
    S_MXO0, S_MXO_END = S_MXO0 + 3, S_MXT0, S_MXT_END = S_MXT0 + 3, S_MXS,  // union-view merged Deps compacted for fetch
    S_MCK0, S_MCK1, S_MCE0, S_MCE1, S_MCP0, S_MCP1,                          // k_merge_cap: kcnt, ment, block parts
    S_MCL, S_MCLS0, S_MCLS1,                                                  //   pass-2 list counters, lists
    S_CSQ0, S_CSQ_END = S_CSQ0 + 34,                                           // ad_cfk_store_query
    S_CSU0, S_CSU_END = S_CSU0 + 20,                                           // the store's unmanaged registry
    S_NUM_FIXED,
    S_CSR0 = 400
};
static_assert(S_NUM_FIXED <= S_CSR0, "fixed device slots overlap the CSR slot blocks");
// CSR slot blocks (10 slots each): key-class CSRs [0, NVC_MAX), range CSRs [NVC_MAX, NVC_MAX + MAXV),
// merged [NVC_MAX + MAXV, +3)
constexpr size_t CSR_RANGE0 = NVC_MAX, CSR_MERGED0 = NVC_MAX + MAXV, CSR_HOST0 = CSR_MERGED0 + 3;
constexpr size_t CSR_SHARD0 = CSR_HOST0 + 3 * MAXV, CSR_SMERGED0 = CSR_SHARD0 + NVC_MAX, CSR_SRANGE0 = CSR_SMERGED0 + 3;
constexpr size_t CSR_MCAP0 = CSR_SRANGE0 + MAXV;          // k_merge_cap's capacity-laid merged key classes (2)
static_assert(CSR_MCAP0 + 2 <= CSR_BLOCKS_MAX, "zero-offset cache covers every CSR block");

#define CK(x) do { int rc_ = (x); if (rc_ != AD_OK) return rc_; } while (0)


inline int bits_of(uint64_t x) { return x == 0 ? 0 : 64 - __builtin_clzll(x); }

int ensure_scratch(ad_handle* h, size_t bytes);
// Makes CSR block `block` an empty class over n txns (zero offsets and counts), skipping the memsets when
// the same buffers were zeroed for the same n since the last allocation.
int zero_csr(ad_handle* h, size_t block, Csr& c, size_t n);
inline void dirty_csr(ad_handle* h, size_t block) { if (block < CSR_BLOCKS_MAX) h->zero_p[block] = nullptr; }
int alloc_csr(ad_handle* h, size_t block, Csr& c, size_t n);
int alloc_csr_data(ad_handle* h, size_t block, Csr& c, int kw);

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

constexpr int MAX_TOTALS = 96;
constexpr int PUB_PRM = 4;                                  // Params words start here
constexpr int PUB_TOT = PUB_PRM + (int)(sizeof(Params) + 3) / 4;
constexpr int PUB_WORDS = PUB_TOT + MAX_TOTALS;
struct TotTable { const uint32_t* src[MAX_TOTALS]; int count; };
// key_off / ent_off / k2t_off of one batched CSR from per-txn (keys, entries) counts
void csr_offsets(ad_handle* h, Csr& c, const uint32_t* nk, const uint32_t* ne);
// The [n] totals of several device offset arrays and the batch Params -> host (engine.hip: k_publish)
int read_totals_params(ad_handle* h, const TotTable& t, uint32_t* host);
int publish_totals(ad_handle* h, const TotTable& t, uint32_t* host, uint32_t* seq_out, const PubExtra* ex = nullptr);
int wait_totals(ad_handle* h, uint32_t seq, int count, uint32_t* host);
void set_level_pub(ad_handle* h);
int read_params(ad_handle* h);
int check_params(ad_handle* h);

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
size_t csr_cap(ad_handle* h, size_t block, int which, size_t elem);

inline void host_mark(ad_handle* h, const char* what) {
    if (h->host_timers < 0) { const char* e = getenv("AD_HOST_TIMERS"); h->host_timers = (e && *e == '1') ? 1 : 0; }
    if (h->host_timers) h->ht.emplace_back(what, std::chrono::steady_clock::now());
}

struct StageScope {
    ad_handle* h;
    StageScope(ad_handle* x, int st) : h(x) { h->stage = st; }
    ~StageScope() { h->stage = STAGE_NONE; }
};


// ---- stages and fetch helpers (definitions: engine.hip, deps.hip, merge.hip, levels.hip)
int stage_prepare(ad_handle* h);
int stage_sort(ad_handle* h);
RadixScratch radix_scratch(ad_handle* h, size_t n);
int stage_deps(ad_handle* h);
int complete_entries(ad_handle* h);
int deps_class_plan(const ad_handle* h, bool want_union, bool* uni_out);
int stage_merge(ad_handle* h);
// k_merge_cap's capacity-laid merged classes -> the exact CSRs in h->merged (no-op otherwise); every reader of
// h->merged's keys / lists calls it first
int merged_ready(ad_handle* h);
// the merged entries of the last merge (k_merge_cap: its per-workgroup sums, read here)
int merged_entries_resolve(ad_handle* h);
int stage_levels(ad_handle* h, bool want_order);
int finish_order(ad_handle* h);
bool order_failed(const ad_handle* h);
// K unions computed together; out[k] = Deps.merge over in[k][0..np) per output txn (merge.hip)
int merge_multi(ad_handle* h, size_t n, int K, Csr* const* out, const size_t* out_block, const int* kw,
                const Csr* const (*in)[MAXV], const int32_t* const (*rows)[MAXV], int np, uint64_t* entries);
// has_direct false: every part's directKeyDeps class is empty (a batch without key-domain sync points)
int merge_parts(ad_handle* h, const Csr* const parts[3][MAXV], int np, bool has_range, const int32_t* const* view_rows = nullptr,
                bool has_direct = true);
int fetch_csr(ad_handle* h, const Csr& c, int kw, ad_csr_out* out);
int csr_sizes(ad_handle* h, const Csr& c, ad_csr_sizes* s);
int fetch_rows(ad_handle* h, const Csr& c, int kw, size_t lo, size_t hi, ad_csr_sizes* s, ad_csr_out* out);
int fetch_empty(ad_handle* h, ad_csr_out* out);
// deps_walk.hip: count / fill walks of the key entries and virtual items, and the RangeDeps join
void launch_walk_nv(int nv, const WalkArgs& a, bool fill, bool direct, bool pairs, hipStream_t st);
void launch_seg_fuse_nv(int nv, const SegFuseArgs& f, const WalkArgs& w, bool direct, hipStream_t st);
void launch_range_nv(int nv, const RangeArgs& a, bool fill, hipStream_t st);
// deps_layout.hip: per-txn offsets / layout / unions of the computed key classes
void launch_offsets_nv(ad_handle* h, int nv, bool direct, const int* cls, uint32_t* heavy, uint32_t* dtx, uint32_t* dtx_count,
                       uint32_t* ovf_rows, uint8_t* ovf_cm, uint32_t* ovf_count);
void launch_finish_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st);
void launch_finish_ovf_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st);
// k_txn_finish_ovf on the side stream xst (forked after the finish; joined before anything reads the deps CSRs)
int side_fork(ad_handle* h);
void side_join(ad_handle* h);
void launch_large_sums_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st);
void launch_large_layout_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st);
void launch_union_nv(int nv, const UnionArgs& ua, bool direct, hipStream_t st);
// level passes for the sharded store rounds (levels.hip: keeps the level kernels in one translation unit)
int levels_run(ad_handle* h, const LevelInputs& li, bool want_order, int* iters);
// global_levels.h: the store's execution constraints as explicit edges over global arrival ranks (kept on the
// device: h->gl_edges, *m edges), and the Kahn solve of an edge set (sharded: the gathered edges into h->G)
// global_ranks: edges over h->gid (sharded stores), else over local rows; done_aware: CFK history batches (no
// edge into or out of an APPLIED / INVALID row)
int levels_export_edges(ad_handle* h, size_t* m, bool global_ranks, bool done_aware);
int levels_solve_edges(ad_handle* h, const uint64_t* d_edges, size_t m, size_t N, uint32_t* L, uint32_t* depth);
void levels_order_rows(ad_handle* h, size_t m, const uint32_t* rows, uint32_t* out);

