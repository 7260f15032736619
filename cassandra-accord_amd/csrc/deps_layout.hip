// deps_layout.hip — the deps stage's per-txn kernels (offsets scan with the fused KeyDeps layout, large-txn
// sums and layout, TxnId unions), one instantiation per class count; compiled in parallel with deps.hip.
#include "engine_internal.h"

// Offsets of every computed key-class CSR in one scan (OffsetsOp: one count dword per pair for <= 4 classes);
// the scan also marks the small txns k_txn_finish cannot finish from the walk's inline ids.  Computed class k
// is CSR cls[k] (every class, or the keyDeps class of each view when the batch has no directKeyDeps).
template <int NC>
void launch_offsets_nc(ad_handle* h, const int* cls, uint32_t* heavy, uint32_t* dtx, uint32_t* dtx_count,
                       uint32_t* ovf_rows, uint8_t* ovf_cm, uint32_t* ovf_count) {
    OffsetsOp<NC> op{};
    op.ovf_rows = ovf_rows; op.ovf_cm = ovf_cm; op.ovf_count = ovf_count;
    op.n = h->n; op.meta = h->meta; op.key_off = h->key_off; op.cnt8 = h->cnt8; op.cntx = h->cntx;
    op.dfr = h->dfr; op.dtx = dtx; op.dtx_count = dtx_count;
    op.lsum_k = h->nk; op.lsum_e = h->ne; op.heavy = heavy;
    for (int k = 0; k < NC; ++k) {
        const int c = cls[k];
        op.o_key_off[k] = h->deps[c].key_off; op.o_ent_off[k] = h->deps[c].ent_off; op.o_k2t_off[k] = h->deps[c].k2t_off;
    }
    scan_any(h, op, h->n);
}
template <int NV>
void launch_offsets(ad_handle* h, bool direct, const int* cls, uint32_t* heavy, uint32_t* dtx, uint32_t* dtx_count,
                    uint32_t* ovf_rows, uint8_t* ovf_cm, uint32_t* ovf_count) {
    if (direct) launch_offsets_nc<2 * NV>(h, cls, heavy, dtx, dtx_count, ovf_rows, ovf_cm, ovf_count);
    else launch_offsets_nc<NV>(h, cls, heavy, dtx, dtx_count, ovf_rows, ovf_cm, ovf_count);
}
template <int NV>
void launch_finish(const TxnArgs& ta, bool direct, hipStream_t st) {
    const unsigned g = (unsigned)ceil_div((long)ta.nrows * (direct ? 2 * NV : NV), 256);
    const bool wide = ta.n >= (1u << 28) - 1;       // ids beyond the 32-bit sort words (TxnId << 4)
    if (direct) {
        if (wide) k_txn_finish<NV, true, true><<<g, 256, 0, st>>>(ta);
        else k_txn_finish<NV, true, false><<<g, 256, 0, st>>>(ta);
    } else {
        if (wide) k_txn_finish<NV, false, true><<<g, 256, 0, st>>>(ta);
        else k_txn_finish<NV, false, false><<<g, 256, 0, st>>>(ta);
    }
    // the overflowed rows (a device-side count: rare, so a small grid — 16K idle workgroups cost 27 us)

}

template <int NV>
void launch_large_sums(const TxnArgs& ta, bool direct, hipStream_t st) {
    const int g = ceil_div((long)ta.n * WAVE, 256);
    if (direct) k_large_sums<2 * NV><<<g, 256, 0, st>>>(ta);
    else k_large_sums<NV><<<g, 256, 0, st>>>(ta);
}
template <int NV>
void launch_large_layout(const TxnArgs& ta, bool direct, hipStream_t st) {
    const int g = ceil_div((long)ta.n * WAVE, 256);
    if (direct) k_large_layout<2 * NV><<<g, 256, 0, st>>>(ta);
    else k_large_layout<NV><<<g, 256, 0, st>>>(ta);
}

template <int NV>
void launch_union(const UnionArgs& ua, bool direct, hipStream_t st) {
    if (direct) k_txn_union<2 * NV><<<ceil_div((long)ua.nrows, 256), 256, 0, st>>>(ua);
    else k_txn_union<NV><<<ceil_div((long)ua.nrows, 256), 256, 0, st>>>(ua);
}

void launch_offsets_nv(ad_handle* h, int nv, bool direct, const int* cls, uint32_t* heavy, uint32_t* dtx, uint32_t* dtx_count,
                       uint32_t* ovf_rows, uint8_t* ovf_cm, uint32_t* ovf_count) {
    NV_DISPATCH(nv, launch_offsets, h, direct, cls, heavy, dtx, dtx_count, ovf_rows, ovf_cm, ovf_count);
}
void launch_finish_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_finish, ta, direct, st); }
// The overflowed rows (a device-side count; each row is a chain of dependent loads — ~27 us of latency for a handful
// of rows on C2 — which is why it runs on the side stream).  Up to 4096 workgroups: C3's hot keys overflow ~10^5 rows,
// which 256 workgroups walked ~6 rows per thread in series (1.6-2.0 ms, on the merge's critical path since the merge
// reads the replies); workgroups past the count exit at once.
template <int NV>
void launch_finish_ovf(const TxnArgs& ta, bool direct, hipStream_t st) {
    const unsigned g = (unsigned)std::min<long>(ceil_div((long)ta.nrows * (direct ? 2 * NV : NV), 256), 4096);
    if (direct) k_txn_finish_ovf<NV, true><<<g, 256, 0, st>>>(ta);
    else k_txn_finish_ovf<NV, false><<<g, 256, 0, st>>>(ta);
}
void launch_finish_ovf_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_finish_ovf, ta, direct, st); }
void launch_large_sums_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_large_sums, ta, direct, st); }
void launch_large_layout_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_large_layout, ta, direct, st); }
void launch_union_nv(int nv, const UnionArgs& ua, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_union, ua, direct, st); }
