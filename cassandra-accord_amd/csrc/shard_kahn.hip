// shard_kahn.hip — execution levels of a key-range sharded batch by distributed Kahn wavefronts
// (kahn_shard_kernels.h has the protocol).  Per wave the host moves one message set between the stores: every
// store's READYs to the txns' holders.  RCCL moves them device to device (ad_shard_kahn_exchange: the per-destination
// counts all-gathered -- the wave's one host synchronisation -- then grouped send/recv); host transports use
// ad_shard_kahn_outbox / ad_shard_kahn_inbox.  ad_shard_kahn_step then runs the wave on the device without waiting for
// it; ad_shard_kahn_finish reads the error flags and the released count once, after the last wave.
#include "engine_internal.h"
#include "global_levels.h"
#include "kahn_shard_kernels.h"

#include <algorithm>

using namespace ad;

namespace {

uint32_t* ks_base(ad_handle* h) { return h->ks_base_dev; }

int ks_bad(ad_handle* h, const char* what) {
    uint32_t bad = 0;
    HIPCHK(h, hipMemcpyAsync(&bad, h->ks_flag + 2, 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    if (bad) return set_err(h, AD_ERR_ARGUMENT, what);
    return AD_OK;
}

void ks_launch_step(ad_handle* h, size_t m, uint32_t S, const uint64_t* in, hipStream_t st) {
    k_ks_step<<<ceil_div((long)m, 256), 256, 0, st>>>(m, S, in, h->n, h->gid, h->holders, h->ks_xoff, h->ks_xs, h->ks_rem,
                                                     h->lvl, h->ks_rcnt, h->ks_lacc, h->ks_plv, ks_base(h), h->ks_cnt_dev,
                                                     h->ks_out, h->ks_flag, h->ks_flag + 2);
}

}  // namespace

extern "C" {

// The store's local constraint graph (its key chains' transitive reduction plus its (b)/(c) edges, local rows:
// the same edges ad_shard_level_edges exports), its successor lists, and wave 0's READY messages.
int ad_shard_kahn_begin(ad_handle* h) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (!h->sharded || !h->have_deps) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_begin: sharded deps first");
    if (!h->holders || h->holders_host.size() != h->n)
        return set_err(h, AD_ERR_STATE, "ad_shard_kahn_begin: ad_shard_set_holders first (the RELEASE fan-out)");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const size_t n = h->n;
    const uint32_t W = h->world;
    const bool mixed = h->Q > 0 || h->n_special > 0 || h->n_large > 0;
    if (mixed && !h->have_merged) {
        CK(stage_merge(h));
        h->merged_has_range = h->Q > 0;
    }
    size_t m = 0;
    CK(levels_export_edges(h, &m, false, false));
    const size_t m1 = std::max<size_t>(m, 1), n1 = std::max<size_t>(n, 1);
    uint32_t *src, *dst, *src2, *dst2;
    CK(dalloc(h, S_KSSRC, &src, m1)); CK(dalloc(h, S_KSDST, &dst, m1));
    CK(dalloc(h, S_KSSRC2, &src2, m1)); CK(dalloc(h, S_KSDST2, &dst2, m1));
    CK(dalloc(h, S_KSREM, &h->ks_rem, n1)); CK(dalloc(h, S_KSXOFF, &h->ks_xoff, n + 1));
    CK(dalloc(h, S_KSRCNT, &h->ks_rcnt, n1)); CK(dalloc(h, S_KSFL, &h->ks_flag, 16));
    CK(dalloc(h, S_KSBASE, &h->ks_base_dev, 2 * (MAX_STORES + 1))); CK(dalloc(h, S_KSCNT, &h->ks_cnt_dev, MAX_STORES + 1));
    CK(dalloc(h, S_KSLACC, &h->ks_lacc, n1)); CK(dalloc(h, S_KSPLV, &h->ks_plv, n1));
    CK(dalloc(h, S_KSHEAD, &h->ks_head_dev, MAX_STORES + 1)); CK(dalloc(h, S_KSSENT, &h->ks_sent_dev, 2));
    // outbox regions: READY to d <= the local rows whose txn d holds (each row is ready once)
    std::vector<uint64_t> lc(W, 0);
    for (size_t i = 0; i < n; ++i)
        for (uint32_t d = 0; d < W; ++d) lc[d] += (h->holders_host[i] >> d) & 1u;
    h->ks_base.assign(2 * (MAX_STORES + 1), 0);
    for (uint32_t d = 0; d < W; ++d) h->ks_base[d + 1] = h->ks_base[d] + (uint32_t)lc[d];
    const size_t cap = std::max<size_t>(h->ks_base[W], 1);
    CK(dalloc(h, S_KSOUT, &h->ks_out, cap));
    HIPCHK(h, hipMemcpyAsync(h->ks_base_dev, h->ks_base.data(), 2 * (MAX_STORES + 1) * 4, hipMemcpyHostToDevice, st));
    HIPCHK(h, hipMemsetAsync(h->ks_rem, 0, n1 * 4, st));
    HIPCHK(h, hipMemsetAsync(h->ks_flag, 0, 64, st));
    CK(ensure_scratch(h, std::max(h->scratch_cap, (size_t)(3 * (radix_hist_len(m1) + 128) + 64 * 1024) * 4)));
    // in-degrees (remaining local predecessors) and the successor lists by source
    if (m) k_edges_split<<<ceil_div((long)m, 256), 256, 0, st>>>(m, h->gl_edges, src, dst, h->ks_rem, (uint32_t)n, h->ks_flag + 2);
    h->ks_xs = dst;
    if (m) {
        const int bits = std::max(1, bits_of(n - 1));
        if (radix_sort_pairs(src, dst, src2, dst2, m, bits, radix_scratch(h, m), st)) { std::swap(src, src2); h->ks_xs = dst2; }
        k_xoff_bounds<<<ceil_div((long)n + 1, 256), 256, 0, st>>>(m, src, (uint32_t)n, h->ks_xoff);
    } else {
        HIPCHK(h, hipMemsetAsync(h->ks_xoff, 0, (n + 1) * 8, st));
    }
    HIPCHK(h, hipMemsetAsync(h->ks_cnt_dev, 0, (MAX_STORES + 1) * 4, st));
    HIPCHK(h, hipMemsetAsync(h->ks_head_dev, 0, (MAX_STORES + 1) * 4, st));
    HIPCHK(h, hipMemsetAsync(h->ks_sent_dev, 0, 16, st));
    h->ks_head_host.assign(MAX_STORES + 1, 0);
    if (n) k_ks_init<<<ceil_div((long)n, 256), 256, 0, st>>>(n, h->gid, h->holders, h->ks_rem, h->lvl, h->ks_rcnt, h->ks_lacc,
                                                             h->ks_plv, ks_base(h), h->ks_cnt_dev, h->ks_out);
    HIPCHK(h, hipGetLastError());
    CK(ks_bad(h, "ad_shard_kahn_begin: a level edge out of range or a self edge"));
    h->ks_phase = 0;
    h->ks_unreleased = n;
    h->ks_sent = 0;
    h->ks_in_m = 0;
    h->ks_levels = true;
    h->level_iters = 0;
    return AD_OK;
}

// Host transports: the outbox of the current phase, per destination (counts[world]) and, if msgs is given, the
// messages in destination order (counts' sum of them).
int ad_shard_kahn_outbox(ad_handle* h, uint32_t* counts, uint64_t* msgs) {
    if (!h || !counts) return AD_ERR_ARGUMENT;
    if (h->ks_phase < 0) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_outbox: ad_shard_kahn_begin first");
    hipSetDevice(h->device);
    const uint32_t W = h->world;
    uint32_t tail[MAX_STORES + 1];
    HIPCHK(h, hipMemcpyAsync(tail, h->ks_cnt_dev, W * 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    for (uint32_t d = 0; d < W; ++d) counts[d] = tail[d] - h->ks_head_host[d];
    if (msgs) {                                  // every queued READY; the queues' heads move past them
        const uint32_t* b = h->ks_base.data();
        size_t at = 0;
        for (uint32_t d = 0; d < W; ++d) {
            if (counts[d])
                HIPCHK(h, hipMemcpyAsync(msgs + at, h->ks_out + b[d] + h->ks_head_host[d], (size_t)counts[d] * 8,
                                         hipMemcpyDeviceToHost, h->st));
            at += counts[d];
            if (d != h->self) h->ks_sent += counts[d];
            h->ks_head_host[d] = tail[d];
        }
        HIPCHK(h, hipMemcpyAsync(h->ks_head_dev, h->ks_head_host.data(), W * 4, hipMemcpyHostToDevice, h->st));
        HIPCHK(h, hipStreamSynchronize(h->st));
    }
    return AD_OK;
}

// Host transports: the messages this store received (every source's region for it, any order).
int ad_shard_kahn_inbox(ad_handle* h, const uint64_t* msgs, size_t m) {
    if (!h || (m && !msgs)) return AD_ERR_ARGUMENT;
    if (h->ks_phase < 0) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_inbox: ad_shard_kahn_begin first");
    hipSetDevice(h->device);
    for (size_t i = 0; i < m; ++i)
        if ((uint32_t)msgs[i] >= h->n_global) return set_err(h, AD_ERR_ARGUMENT, "ad_shard_kahn_inbox: global rank out of range");
    CK(dalloc(h, S_KSIN, &h->ks_in, std::max<size_t>(m, 1)));
    if (m) HIPCHK(h, hipMemcpyAsync(h->ks_in, msgs, m * 8, hipMemcpyHostToDevice, h->st));
    h->ks_in_m = m;
    return AD_OK;
}

// RCCL: this wave's per-destination counts (the queues' lengths) all-gathered (a world x (world + 1) matrix; the last
// column is unused), a host synchronisation, then the queued READYs by grouped point-to-point send/recv into the inbox
// (this store's own by a device copy).  *any_status: some store sent something (else the waves are over; `status` is
// ignored).  (ad_shard_kahn_run drives the waves without the synchronisation.)
int ad_shard_kahn_exchange(ad_handle* h, uint32_t status, uint32_t* any_status) {
    if (!h || !any_status) return AD_ERR_ARGUMENT;
    if (!h->comm || h->ks_phase < 0) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_exchange: ad_comm_init + ad_shard_kahn_begin first");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const uint32_t W = h->world, self = h->self;
    uint32_t *mat = nullptr, *wcnt = nullptr;
    CK(dalloc(h, S_KSMAT, &mat, (size_t)MAX_STORES * (MAX_STORES + 1)));
    CK(dalloc(h, S_KSPEND, &wcnt, 64));
    (void)status;
    k_ks_lengths<<<1, 64, 0, st>>>(W, h->ks_cnt_dev, h->ks_head_dev, wcnt);
    ncclResult_t r = ncclAllGather(wcnt, mat, W + 1, ncclUint32, h->comm, st);
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclAllGather (Kahn counts): ") + ncclGetErrorString(r));
    std::vector<uint32_t> M((size_t)W * (W + 1));
    HIPCHK(h, hipMemcpyAsync(M.data(), mat, M.size() * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    uint64_t recv_total = 0, sent_any = 0;
    for (uint32_t s = 0; s < W; ++s) {
        recv_total += M[(size_t)s * (W + 1) + self];
        for (uint32_t d = 0; d < W; ++d) sent_any += M[(size_t)s * (W + 1) + d];
    }
    *any_status = sent_any ? 1u : 0u;
    CK(dalloc(h, S_KSIN, &h->ks_in, std::max<uint64_t>(recv_total, 1)));
    const uint32_t* b = h->ks_base.data();
    if (ncclGroupStart() != ncclSuccess) return set_err(h, AD_ERR_DEVICE, "ncclGroupStart");
    ncclResult_t first = ncclSuccess;
    std::string what;
    size_t ro = 0;
    for (uint32_t p = 0; p < W && first == ncclSuccess; ++p) {
        const uint32_t sn = M[(size_t)self * (W + 1) + p], rn = M[(size_t)p * (W + 1) + self];
        const uint64_t* src = h->ks_out + b[p] + h->ks_head_host[p];
        if (p == self) {
            if (sn) HIPCHK(h, hipMemcpyAsync(h->ks_in + ro, src, (size_t)sn * 8, hipMemcpyDeviceToDevice, st));
        } else {
            if (sn) {
                ncclResult_t e = ncclSend(src, (size_t)sn * 8, ncclUint8, (int)p, h->comm, st);
                if (e != ncclSuccess) { first = e; what = "ncclSend (Kahn) to " + std::to_string(p); }
                h->ks_sent += sn;
            }
            if (first == ncclSuccess && rn) {
                ncclResult_t e = ncclRecv(h->ks_in + ro, (size_t)rn * 8, ncclUint8, (int)p, h->comm, st);
                if (e != ncclSuccess) { first = e; what = "ncclRecv (Kahn) from " + std::to_string(p); }
            }
        }
        h->ks_head_host[p] += sn;
        ro += rn;
    }
    r = ncclGroupEnd();
    if (first != ncclSuccess) return set_err(h, AD_ERR_DEVICE, what + ": " + ncclGetErrorString(first));
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclGroupEnd (Kahn): ") + ncclGetErrorString(r));
    HIPCHK(h, hipMemcpyAsync(h->ks_head_dev, h->ks_head_host.data(), W * 4, hipMemcpyHostToDevice, st));
    h->ks_in_m = recv_total;
    return AD_OK;
}

// One wave on the device (no host synchronisation): the received READYs counted, rows every holder reported released
// (at the greatest level bound of their READYs), their successors' READYs queued for the next exchange.  `level` is
// not used (the levels ride in the READYs).
int ad_shard_kahn_step(ad_handle* h, uint32_t level) {
    if (!h) return AD_ERR_ARGUMENT;
    g_tracer = &h->tracer;
    if (h->ks_phase != 0) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_step: ad_shard_kahn_begin first");
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    const size_t m = h->ks_in_m;
    if (m) ks_launch_step(h, m, 0, h->ks_in, st);
    HIPCHK(h, hipGetLastError());
    if (m) h->level_iters = level + 1;
    h->ks_in_m = 0;
    return AD_OK;
}

// The whole wave loop over RCCL with fixed exchange slots (kahn_shard_kernels.h): per wave the slots packed from the
// queues, one grouped send/recv of (slot + 1) words per peer, the step; every `check_every` waves the READYs still
// queued on every store summed by an all-reduce into a pinned word, which the host reads `lag` checks later (no wait
// between waves: the device has those waves queued).  The slot size is the largest proposal over the stores
// (`slot`, or from the queues' capacities when 0): one all-reduce before the loop.  *waves: waves run; returns
// AD_ERR_UNSUPPORTED (nothing left to raise: the caller falls back) past wave_cap waves.
int ad_shard_kahn_run(ad_handle* h, uint32_t slot, uint32_t check_every, uint32_t lag, uint32_t wave_cap, uint32_t* waves) {
    if (!h || !waves) return AD_ERR_ARGUMENT;
    if (!h->comm || h->ks_phase != 0) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_run: ad_comm_init + ad_shard_kahn_begin first");
    hipSetDevice(h->device);
    g_tracer = &h->tracer;
    hipStream_t st = h->st;
    const uint32_t W = h->world, self = h->self;
    check_every = std::max<uint32_t>(check_every, 1);
    // the slot: every store's proposal (its largest queue capacity / 16, within [1024, 65536]) maxed over the stores
    uint32_t prop = slot;
    if (!prop) {
        uint32_t cap = 0;
        for (uint32_t d = 0; d < W; ++d) cap = std::max(cap, h->ks_base[d + 1] - h->ks_base[d]);
        prop = std::min<uint32_t>(65536, std::max<uint32_t>(1024, cap / 16));
    }
    uint32_t* wv = nullptr;
    CK(dalloc(h, S_KSPEND, &wv, 64));
    HIPCHK(h, hipMemcpyAsync(wv, &prop, 4, hipMemcpyHostToDevice, st));
    ncclResult_t r = ncclAllReduce(wv, wv + 1, 1, ncclUint32, ncclMax, h->comm, st);
    if (r != ncclSuccess) return set_err(h, AD_ERR_DEVICE, std::string("ncclAllReduce (Kahn slot): ") + ncclGetErrorString(r));
    uint32_t S = 0;
    HIPCHK(h, hipMemcpyAsync(&S, wv + 1, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));                   // (once, before the waves)
    const size_t sw = (size_t)W * (S + 1);
    uint64_t *sto = nullptr, *sti = nullptr;
    CK(dalloc(h, S_KSSTO, &sto, sw)); CK(dalloc(h, S_KSSTI, &sti, sw));
    unsigned long long* pend = reinterpret_cast<unsigned long long*>(wv + 8);   // [0] this store's, [1] the sum
    // pinned check words: one per check, read lag checks later
    const uint32_t max_checks = wave_cap / check_every + lag + 2;
    unsigned long long* pin = nullptr;
    HIPCHK(h, hipHostMalloc(&pin, (size_t)max_checks * 8, hipHostMallocDefault));
    std::vector<hipEvent_t> evs(max_checks, nullptr);
    int rc = AD_OK;
    uint32_t w = 0, checks = 0, read = 0;
    bool done = false;
    while (!done) {
        if (w >= wave_cap) { rc = set_err(h, AD_ERR_UNSUPPORTED, "ad_shard_kahn_run: waves still releasing past the cap"); break; }
        k_ks_pack<<<W, 256, 0, st>>>(S, self, ks_base(h), h->ks_cnt_dev, h->ks_head_dev, h->ks_out, sto, h->ks_sent_dev);
        bool fail = ncclGroupStart() != ncclSuccess;
        for (uint32_t p = 0; p < W && !fail; ++p) {
            if (p == self) {
                fail = hipMemcpyAsync(sti + (size_t)p * (S + 1), sto + (size_t)p * (S + 1), (S + 1) * 8, hipMemcpyDeviceToDevice, st) != hipSuccess;
                continue;
            }
            fail = ncclSend(sto + (size_t)p * (S + 1), (S + 1) * 8, ncclUint8, (int)p, h->comm, st) != ncclSuccess ||
                   ncclRecv(sti + (size_t)p * (S + 1), (S + 1) * 8, ncclUint8, (int)p, h->comm, st) != ncclSuccess;
        }
        fail = (ncclGroupEnd() != ncclSuccess) || fail;
        if (fail) { rc = set_err(h, AD_ERR_DEVICE, "ad_shard_kahn_run: slot exchange failed"); break; }
        ks_launch_step(h, sw - W, S, sti, st);            // W sources x S slots (their count words skipped by index)
        ++w;
        if (w % check_every == 0) {
            k_ks_pending<<<1, 64, 0, st>>>(W, h->ks_cnt_dev, h->ks_head_dev, pend);
            if (ncclAllReduce(pend, pend + 1, 1, ncclUint64, ncclSum, h->comm, st) != ncclSuccess) {
                rc = set_err(h, AD_ERR_DEVICE, "ad_shard_kahn_run: pending all-reduce failed");
                break;
            }
            HIPCHK(h, hipMemcpyAsync(pin + checks, pend + 1, 8, hipMemcpyDeviceToHost, st));
            HIPCHK(h, hipEventCreateWithFlags(&evs[checks], hipEventDisableTiming));
            HIPCHK(h, hipEventRecord(evs[checks], st));
            ++checks;
            // the check `lag` behind the front: every store reads the same sum at the same wave, so all stop together
            if (checks > lag) {
                HIPCHK(h, hipEventSynchronize(evs[read]));
                done = pin[read] == 0;
                ++read;
            }
        }
    }
    HIPCHK(h, hipStreamSynchronize(st));
    for (uint32_t c = 0; c < checks; ++c) hipEventDestroy(evs[c]);
    hipHostFree(pin);
    unsigned long long sent = 0;
    HIPCHK(h, hipMemcpy(&sent, h->ks_sent_dev, 8, hipMemcpyDeviceToHost));
    h->ks_sent = sent;
    h->level_iters = w;
    *waves = w;
    return rc;
}

// The batch's depth (the greatest level + 1) after the waves.
int ad_shard_kahn_depth(ad_handle* h, uint32_t* depth) {
    if (!h || !depth) return AD_ERR_ARGUMENT;
    if (h->ks_phase != 0) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_depth: ad_shard_kahn_begin first");
    hipSetDevice(h->device);
    HIPCHK(h, hipMemcpyAsync(depth, h->ks_flag + 3, 4, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    return AD_OK;
}

// After the last wave: the error flag and the rows still unreleased (a cycle if any).
int ad_shard_kahn_finish(ad_handle* h, uint64_t* unreleased) {
    if (!h || !unreleased) return AD_ERR_ARGUMENT;
    if (h->ks_phase != 0) return set_err(h, AD_ERR_STATE, "ad_shard_kahn_finish: ad_shard_kahn_begin first");
    hipSetDevice(h->device);
    uint32_t f[3] = {0, 0, 0};
    HIPCHK(h, hipMemcpyAsync(f, h->ks_flag, 12, hipMemcpyDeviceToHost, h->st));
    HIPCHK(h, hipStreamSynchronize(h->st));
    if (f[2]) return set_err(h, AD_ERR_ARGUMENT, "ad_shard_kahn: a READY for a txn this store does not hold, or already released");
    *unreleased = h->n - std::min<size_t>(h->n, f[1]);
    return AD_OK;
}

// Messages this batch's waves sent to other stores (8 bytes each).
int ad_shard_kahn_sent(ad_handle* h, uint64_t* sent) {
    if (!h || !sent) return AD_ERR_ARGUMENT;
    *sent = h->ks_sent;
    return AD_OK;
}

}  // extern "C"
