// deps_walk.hip — the deps stage's walk launches (CFK mapReduceActive per entry / virtual item, RangeDeps
// join), one instantiation per replica-view count; a unit of its own so the walks compile in parallel with
// the rest of the deps stage.
#include "engine_internal.h"

template <int NV, bool DIRECT>
void launch_walk_d(const WalkArgs& a, bool fill, bool pairs, hipStream_t st) {
    if (a.P > 0 && pairs) {
        const int g = ceil_div((long)(fill ? a.nitems : a.P), 256);
        KScope ks(fill ? K_WALK_FILL : K_WALK_COUNT, a.P);
        if (fill) k_deps_walk<NV, true, DIRECT><<<g, 256, 0, st>>>(a);
        else k_deps_walk<NV, false, DIRECT><<<g, 256, 0, st>>>(a);
    }
    if (a.V > 0) {
        const int g = ceil_div((long)a.V, 256);
        KScope ks(K_VITEMS);
        if (fill) k_vitem_walk<NV, true, DIRECT><<<g, 256, 0, st>>>(a);
        else k_vitem_walk<NV, false, DIRECT><<<g, 256, 0, st>>>(a);
    }
}
template <int NV>
void launch_walk(const WalkArgs& a, bool fill, bool direct, bool pairs, hipStream_t st) {
    if (direct) launch_walk_d<NV, true>(a, fill, pairs, st);
    else launch_walk_d<NV, false>(a, fill, pairs, st);
}
template <int NV>
void launch_range(const RangeArgs& a, bool fill, hipStream_t st) {
    const int g = ceil_div((long)a.n * WAVE, 256);
    KScope ks(K_RANGE);
    if (fill) k_range_deps<NV, true><<<g, 256, 0, st>>>(a);
    else k_range_deps<NV, false><<<g, 256, 0, st>>>(a);
}
void launch_walk_nv(int nv, const WalkArgs& a, bool fill, bool direct, bool pairs, hipStream_t st) {
    NV_DISPATCH(nv, launch_walk, a, fill, direct, pairs, st);
}
void launch_range_nv(int nv, const RangeArgs& a, bool fill, hipStream_t st) {
    NV_DISPATCH(nv, launch_range, a, fill, st);
}

// k_seg_fuse (seg_fuse_kernels.h): gather + elision state + count walk per tile of key segments
template <int NV>
void launch_seg_fuse(const SegFuseArgs& f, const WalkArgs& w, bool direct, hipStream_t st) {
    if (direct) k_seg_fuse<NV, true><<<(unsigned)f.ntiles, SF_T, 0, st>>>(f, w);
    else k_seg_fuse<NV, false><<<(unsigned)f.ntiles, SF_T, 0, st>>>(f, w);
}
void launch_seg_fuse_nv(int nv, const SegFuseArgs& f, const WalkArgs& w, bool direct, hipStream_t st) {
    NV_DISPATCH(nv, launch_seg_fuse, f, w, direct, st);
}
