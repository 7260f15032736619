// conflict_kernels.h — the replica's witnessedAt proposal (MaxConflicts) for a key batch (gfx950).
//
// CommandStore.preaccept (local/CommandStore.java:322-347) answers witnessedAt = TxnId when
// TxnId >= maxConflicts.get(keys), else a fresh HLC above it.  MaxConflicts (local/MaxConflicts.java:46-59)
// is a per-key running max of the executeAt of every globally visible txn the store has recorded
// (CommandStore.updateMaxConflicts :282-291, SafeCommandStore.updateMaxConflicts :210-222).  For a batch
// that arrives in TxnId order this is, per (txn i, key) and replica view v, the max executeAt over the
// key's CommandsForKey entries j < i the view holds: out-of-window entries whose final status is recorded
// (category != CAT_SKIP) plus in-flight ones the view did not drop — the same entry set the deps walk
// visits (deps_kernels.h walk_query), without the witness/elision filters.
//
//   MaxConflictOp scan   segmented inclusive prefix max of (executeAt+1, rank) over recorded entries; its
//                        store also inverts the sort permutation (pair -> sorted position)
//   k_mc_txns<NV>        one thread per txn: per pair, the in-flight window walk per view from the pair's
//                        sorted position, then the prefix max of the entry just below the window; max over
//                        the txn's pairs per view, fast-path test (no per-pair intermediate in HBM)
#pragma once
#include "deps_kernels.h"

namespace ad {

// (executeAt+1, rank) pairs: executeAt+1 = packed ts64 + 1 (0 = Timestamp.NONE), rank = batch row of the txn
// holding it; ordered lexicographically, so equal executeAts go to the larger rank
__device__ inline bool mc_less(uint64_t ae, uint32_t ar, uint64_t be, uint32_t br) {
    return ae < be || (ae == be && ar < br);
}

struct MaxConflictOp {
    struct S {
        uint64_t e;
        uint32_t r;
        uint32_t head;
    };
    const int32_t* seg_start;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const uint32_t* e_txn;
    const uint32_t* sval;      // sorted position -> pair index
    uint64_t* pm_e;
    uint32_t* pm_r;
    uint32_t* inv;             // pair index -> sorted position

    __device__ S load(size_t i) const {
        const uint32_t m = e_meta[i];
        const bool rec = category(m) != CAT_SKIP;
        return S{rec ? e_exec1[i] : 0ull, rec ? e_txn[i] : 0u, seg_start[i] == (int32_t)i ? 1u : 0u};
    }
    __device__ S identity() const { return S{0ull, 0u, 0u}; }
    __device__ S combine(const S& a, const S& b) const {
        if (b.head) return S{b.e, b.r, 1u};
        const bool lt = mc_less(a.e, a.r, b.e, b.r);
        return S{lt ? b.e : a.e, lt ? b.r : a.r, a.head};
    }
    __device__ void store(size_t i, const S&, const S& inc, const S&) const {
        pm_e[i] = inc.e;
        pm_r[i] = inc.r;
        inv[sval[i]] = (uint32_t)i;
    }
};

struct McArgs {
    size_t n, P;
    const uint32_t* e_txn;
    const uint8_t* e_meta;
    const uint64_t* e_exec1;
    const int32_t* seg_start;
    const uint32_t* inv;       // pair index -> sorted position
    const uint32_t* gid;       // sharded batches: local row -> global arrival rank (nullable)
    const uint64_t* pm_e;
    const uint32_t* pm_r;
    uint32_t window, thresh;
    uint64_t seed;
    const uint32_t* key_off;
    const uint64_t* tx_ts;
    uint32_t* max_rank;        // [v * n + t]
    uint8_t* fast;             // [v * n + t]
};

template <int NV>
__global__ __launch_bounds__(256) void k_mc_txns(McArgs a) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t gi = a.gid ? a.gid[t] : (uint32_t)t;
    const uint32_t lo = a.window == 0 ? gi : (gi > a.window ? gi - a.window : 0u);
    uint64_t be[NV];
    uint32_t br[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) { be[v] = 0; br[v] = 0; }
    for (uint32_t p = a.key_off[t]; p < a.key_off[t + 1]; ++p) {
        const int s = (int)a.inv[p];
        const int seg0 = a.seg_start[s];
        // in-flight window [i - W, i): recorded as PreAccepted by every view that did not drop it
        int q = s - 1;
        for (; q >= seg0; --q) {
            const uint32_t j = a.e_txn[q];
            const uint32_t gj = a.gid ? a.gid[j] : j;
            if (gj < lo) break;
            if (!manages(a.e_meta[q])) continue;
            const uint64_t e = a.e_exec1[q];
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (!(a.thresh && drop_hash(a.seed, (uint32_t)v, gi, gj) < a.thresh) && mc_less(be[v], br[v], e, j)) {
                    be[v] = e; br[v] = j;
                }
        }
        // recorded prefix [seg0, q]: one segmented-scan value, identical for every view
        if (q >= seg0) {
            const uint64_t e = a.pm_e[q];
            const uint32_t r = a.pm_r[q];
#pragma unroll
            for (int v = 0; v < NV; ++v)
                if (mc_less(be[v], br[v], e, r)) { be[v] = e; br[v] = r; }
        }
    }
    const uint64_t t1 = a.tx_ts[t] + 1;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        // sharded stores answer in global arrival ranks (ascending with local rows: the tie rule is kept)
        a.max_rank[(size_t)v * a.n + t] = be[v] ? (a.gid ? a.gid[br[v]] : br[v]) : AD_RANK_NONE;
        a.fast[(size_t)v * a.n + t] = (be[v] == 0 || t1 >= be[v]) ? 1 : 0;   // TxnId.compareTo(max) >= 0
    }
}

}  // namespace ad
