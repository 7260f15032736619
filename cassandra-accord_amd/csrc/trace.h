// trace.h — per-kernel HIP-event timing on the handle's stream (the "--trace" mode of SURVEY §5).
//
// A KScope brackets one kernel launch (or one multi-launch device_scan) with a pair of events on the
// stream the kernel is launched on, when that kernel id is enabled in the active tracer's mask.  The
// pairs are resolved after the pipeline's final synchronisation, so tracing adds no host syncs.
// bench.py enables only the dominant kernel inside its timed region (roofline.achieved) and every
// kernel in a separate, untimed breakdown pass.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

namespace ad {

enum KernelId : int {
    K_MINMAX, K_PACK, K_RADIX_HIST, K_RADIX_SCATTER, K_SCAN_RADIX, K_GATHER, K_SCAN_ELIDE, K_WALK_COUNT,
    K_TXN_COUNTS, K_SCAN_OFFSETS, K_TXN_LAYOUT, K_WALK_FILL, K_TXN_UNION, K_MERGE_COUNT, K_MERGE_WRITE,
    K_CHAIN_PREP, K_SCAN_CHAIN, K_ORDER, K_RANGE, K_VITEMS, K_UNION_LDS, K_LEVEL_EDGES, K_KAHN, K_MERGE_HEAVY_COUNT, K_MERGE_HEAVY_WRITE, K_MAX_CONFLICTS, K_MERGE_OFFSETS, K_CSR_OFFSETS, K_BLOCK_LEVELS, K_RECOVER, K_SEG_FUSE, K_SEG_KEYS, K_MERGE_CAP, K_COUNT
};

inline const char* kernel_name(int k) {
    static const char* names[K_COUNT] = {
        "k_minmax", "k_pack", "k_radix_hist", "k_radix_scatter", "scan_radix", "k_gather_entries", "scan_elide",
        "k_deps_walk<count>", "k_txn_counts", "scan_offsets", "k_txn_finish", "k_deps_walk<fill>", "k_txn_union",
        "k_merge<count>", "k_merge<write>", "chain_prep", "scan_chain", "order_sort", "k_range_deps", "vitems",
        "k_union_lds", "level_edges", "kahn_levels", "k_merge_heavy<count>", "k_merge_heavy<write>",
        "max_conflicts", "merge_offsets", "csr_offsets", "block_levels", "recover", "k_seg_fuse", "seg_keys", "k_merge_ref"};
    return (k >= 0 && k < K_COUNT) ? names[k] : "?";
}

struct Tracer {
    hipStream_t st = nullptr;
    uint64_t mask = 0;
    struct Rec { int kid; hipEvent_t a, b; uint64_t units; };
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    std::vector<Rec> recs;
    double total_ms[K_COUNT] = {};
    uint64_t calls[K_COUNT] = {};
    uint64_t units[K_COUNT] = {};      // elements processed (the kernel's algorithmic unit), summed

    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            hipEventCreate(&e);
            pool.push_back(e);
        }
        return pool[used++];
    }
    void reset_counts() {
        for (int k = 0; k < K_COUNT; ++k) { total_ms[k] = 0; calls[k] = 0; units[k] = 0; }
    }
    // After the stream has been synchronised: fold the recorded pairs into the totals.
    void resolve() {
        for (const Rec& r : recs) {
            float ms = 0;
            if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
                total_ms[r.kid] += ms;
                calls[r.kid] += 1;
                units[r.kid] += r.units;
            }
        }
        recs.clear();
        used = 0;
    }
    ~Tracer() {
        for (hipEvent_t e : pool) hipEventDestroy(e);
    }
};

inline thread_local Tracer* g_tracer = nullptr;

struct KScope {
    Tracer* t;
    int kid;
    hipEvent_t b = nullptr;
    explicit KScope(int k, uint64_t units = 0) : t(g_tracer), kid(k) {
        if (t && (t->mask >> k & 1ull)) {
            hipEvent_t a = t->get();
            b = t->get();
            hipEventRecord(a, t->st);
            t->recs.push_back(Tracer::Rec{k, a, b, units});
        } else {
            t = nullptr;
        }
    }
    ~KScope() {
        if (t) hipEventRecord(b, t->st);
    }
};

}  // namespace ad
