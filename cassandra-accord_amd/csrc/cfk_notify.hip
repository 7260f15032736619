// cfk_notify.hip — ad_cfk_notify: CommandsForKey.notifyManaged's release rule over CFK states (notify_kernels.h).
#include "engine_internal.h"

int ad_cfk_notify(ad_handle* h, const ad_cfk_state* s, uint8_t* not_waiting) {
    if (!h || !s) return AD_ERR_ARGUMENT;
    const size_t K = s->keys, n = s->rows;
    if (K && (!s->row_off || !not_waiting)) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: row_off / not_waiting missing");
    if (n && (!s->txn_msb || !s->txn_lsb || !s->txn_node || !s->exec_msb || !s->exec_lsb || !s->exec_node || !s->status || !s->miss_off))
        return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: a row array is missing");
    if (K && (s->row_off[0] != 0 || s->row_off[K] != n)) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: row_off must span [0, rows]");
    for (size_t k = 0; k < K; ++k)
        if (s->row_off[k + 1] < s->row_off[k]) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: row_off must be non-decreasing");
    const size_t nm = n ? s->miss_off[n] : 0;
    if (n && s->miss_off[0] != 0) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: miss_off must start at 0");
    for (size_t i = 0; i < n; ++i)          // every row's missing run inside [0, miss_off[n]]: no read past the array
        if (s->miss_off[i + 1] < s->miss_off[i] || s->miss_off[i + 1] > nm)
            return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: miss_off must be non-decreasing and end at the missing count");
    if (nm && !s->missing) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: missing entries without an array");
    if (K == 0) return AD_OK;
    hipSetDevice(h->device);
    hipStream_t st = h->st;
    uint32_t *roff, *moff, *miss, *pre, *flags;
    uint64_t *tm, *tl, *em, *el;
    int32_t *tn, *en;
    uint8_t *sts, *out;
    const size_t c = std::max<size_t>(n, 1);
    CK(dalloc(h, S_NF0 + 0, &roff, K + 1)); CK(dalloc(h, S_NF0 + 1, &tm, c)); CK(dalloc(h, S_NF0 + 2, &tl, c));
    CK(dalloc(h, S_NF0 + 3, &tn, c)); CK(dalloc(h, S_NF0 + 4, &em, c)); CK(dalloc(h, S_NF0 + 5, &el, c));
    CK(dalloc(h, S_NF0 + 6, &en, c)); CK(dalloc(h, S_NF0 + 7, &sts, c)); CK(dalloc(h, S_NF0 + 8, &moff, n + 1));
    CK(dalloc(h, S_NF0 + 9, &miss, std::max<size_t>(nm, 1))); CK(dalloc(h, S_NF0 + 10, &pre, 2 * c));
    CK(dalloc(h, S_NF0 + 11, &out, c)); CK(dalloc(h, S_NF0 + 12, &flags, 2));
    HIPCHK(h, hipMemcpyAsync(roff, s->row_off, (K + 1) * 4, hipMemcpyHostToDevice, st));
    if (n) {
        HIPCHK(h, hipMemcpyAsync(tm, s->txn_msb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(tl, s->txn_lsb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(tn, s->txn_node, n * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(em, s->exec_msb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(el, s->exec_lsb, n * 8, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(en, s->exec_node, n * 4, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(sts, s->status, n, hipMemcpyHostToDevice, st));
        HIPCHK(h, hipMemcpyAsync(moff, s->miss_off, (n + 1) * 4, hipMemcpyHostToDevice, st));
        if (nm) HIPCHK(h, hipMemcpyAsync(miss, s->missing, nm * 4, hipMemcpyHostToDevice, st));
    }
    HIPCHK(h, hipMemsetAsync(flags, 0, 8, st));
    NotifyArgs a{};
    a.K = K; a.row_off = roff; a.tm = tm; a.tl = tl; a.tn = tn; a.em = em; a.el = el; a.en = en; a.st = sts;
    a.miss_off = moff; a.miss = miss; a.pre = pre; a.out = out; a.bad_order = flags; a.bad_miss = flags + 1;
    k_cfk_notify<<<(unsigned)K, NF_T, 0, st>>>(a);
    HIPCHK(h, hipGetLastError());
    uint32_t hf[2] = {0, 0};
    HIPCHK(h, hipMemcpyAsync(hf, flags, 8, hipMemcpyDeviceToHost, st));
    if (n) HIPCHK(h, hipMemcpyAsync(not_waiting, out, n, hipMemcpyDeviceToHost, st));
    HIPCHK(h, hipStreamSynchronize(st));
    if (hf[0]) return set_err(h, AD_ERR_UNSORTED, "ad_cfk_notify: a key's TxnIds are not strictly ascending (byId order)");
    if (hf[1]) return set_err(h, AD_ERR_ARGUMENT, "ad_cfk_notify: a missing entry indexes outside its key's rows");
    return AD_OK;
}
