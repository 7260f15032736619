// deps_layout.hip — the deps stage's per-txn kernels (offsets scan with the fused KeyDeps layout, large-txn
// sums and layout, TxnId unions), one instantiation per class count; compiled in parallel with deps.hip.
#include "engine_internal.h"

// Offsets of every computed key-class CSR in one scan; with buffers left by an earlier batch, also the
// per-txn layout (fused; *overflow reports rows that did not fit, then k_txn_layout runs after sizing).
// Computed class k is CSR cls[k] (every class, or the keyDeps class of each view when the batch has no
// directKeyDeps).
template <int NC>
void launch_offsets_nc(ad_handle* h, const int* cls, uint32_t* overflow) {
    OffsetsOp<NC> op{};
    op.n = h->n; op.meta = h->meta; op.key_off = h->key_off; op.cnt = h->cnt;
    op.layout = 1;
    op.keys = h->keys; op.dst = h->dst; op.overflow = overflow;
    op.lsum_k = h->nk; op.lsum_e = h->ne; op.heavy = overflow - 1;
    for (int k = 0; k < NC; ++k) {
        const int c = cls[k];
        op.o_key_off[k] = h->deps[c].key_off; op.o_ent_off[k] = h->deps[c].ent_off; op.o_k2t_off[k] = h->deps[c].k2t_off;
        const size_t base = S_CSR0 + 10 * (size_t)c;
        const size_t ck = csr_cap(h, c, 4, 8), cm = csr_cap(h, c, 5, 4);
        op.out_keys[k] = ck ? (uint64_t*)h->bufs[base + 4].p : nullptr;
        op.out_k2t[k] = cm ? (int32_t*)h->bufs[base + 5].p : nullptr;
        op.cap_keys[k] = (uint32_t)std::min<size_t>(ck, 0xFFFFFFFFu);
        op.cap_k2t[k] = (uint32_t)std::min<size_t>(cm, 0xFFFFFFFFu);
    }
    scan_any(h, op, h->n);
}
template <int NV>
void launch_offsets(ad_handle* h, bool direct, const int* cls, uint32_t* overflow) {
    if (direct) launch_offsets_nc<2 * NV>(h, cls, overflow);
    else launch_offsets_nc<NV>(h, cls, overflow);
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
    if (direct) k_txn_union<2 * NV><<<ceil_div((long)ua.n, 256), 256, 0, st>>>(ua);
    else k_txn_union<NV><<<ceil_div((long)ua.n, 256), 256, 0, st>>>(ua);
}

void launch_offsets_nv(ad_handle* h, int nv, bool direct, const int* cls, uint32_t* overflow) {
    NV_DISPATCH(nv, launch_offsets, h, direct, cls, overflow);
}
void launch_large_sums_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_large_sums, ta, direct, st); }
void launch_large_layout_nv(int nv, const TxnArgs& ta, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_large_layout, ta, direct, st); }
void launch_union_nv(int nv, const UnionArgs& ua, bool direct, hipStream_t st) { NV_DISPATCH(nv, launch_union, ua, direct, st); }
