// common.h — device-side encodings and helpers shared by the gfx950 kernels.
//
// Timestamps are compared through a packed 64-bit order key ("ts64") built per batch:
//   ts64 = (msb - msb_min) << (HB+4+NB) | (lowHlc - hlc_min) << (4+NB) | ((lsb>>1)&0xF) << NB | (node - node_min)
// which orders exactly as Timestamp.compareTo (Timestamp.java:208-217: msb unsigned, lsb>>>16,
// lsb & 0x1E, node signed) whenever MB+HB+4+NB <= 64 (checked per batch; AD_ERR_UNSUPPORTED otherwise).
// Equality of ts64 is Timestamp.equals (IDENTITY_LSB = hlc bits | 0x1E, Timestamp.java:41,244-249).
#pragma once
#include <initializer_list>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/accord_deps.h"
#include "trace.h"

namespace ad {

constexpr int WAVE = 64;
constexpr uint64_t TS_NONE = 0xFFFFFFFFFFFFFFFFull;   // "no timestamp" sentinel (never a packed value: widths < 64)

// Per-txn metadata byte: bits 0-2 kind, bit 3 domain, bits 4-6 final InternalStatus.
__host__ __device__ inline uint32_t meta_kind(uint32_t m) { return m & 7u; }
__host__ __device__ inline uint32_t meta_domain(uint32_t m) { return (m >> 3) & 1u; }
__host__ __device__ inline uint32_t meta_status(uint32_t m) { return (m >> 4) & 7u; }

// Txn.Kind.witnesses (primitives/Txn.java:221-245, Kinds.test :140-152)
//   Read/EphemeralRead -> Ws; Write/SyncPoint -> RsOrWs; ExclusiveSyncPoint -> AnyGloballyVisible.
__host__ __device__ inline bool witnesses(uint32_t q, uint32_t d) {
    switch (q) {
        case AD_KIND_READ:
        case AD_KIND_EPHEMERAL_READ: return d == AD_KIND_WRITE;
        case AD_KIND_WRITE:
        case AD_KIND_SYNC_POINT: return d == AD_KIND_READ || d == AD_KIND_WRITE;
        case AD_KIND_EXCLUSIVE_SYNC_POINT:
            return d == AD_KIND_READ || d == AD_KIND_WRITE || d == AD_KIND_SYNC_POINT || d == AD_KIND_EXCLUSIVE_SYNC_POINT;
        default: return false;
    }
}
// CommandsForKey.manages (key domain, globally visible) — CommandsForKey.java:185-188
__host__ __device__ inline bool manages(uint32_t m) {
    uint32_t k = meta_kind(m);
    return meta_domain(m) == AD_DOMAIN_KEY && (k == AD_KIND_READ || k == AD_KIND_WRITE || k == AD_KIND_SYNC_POINT ||
                                               k == AD_KIND_EXCLUSIVE_SYNC_POINT);
}
// CommandsForKey.managesExecution (key Read/Write) — CommandsForKey.java:196-199
__host__ __device__ inline bool manages_execution(uint32_t m) {
    uint32_t k = meta_kind(m);
    return meta_domain(m) == AD_DOMAIN_KEY && (k == AD_KIND_READ || k == AD_KIND_WRITE);
}
// Entry categories for an out-of-window CFK entry (CommandsForKey.mapReduceActive :951-962)
enum : uint32_t { CAT_SKIP = 0, CAT_ALWAYS = 1, CAT_ELIDABLE = 2 };
__host__ __device__ inline uint32_t category(uint32_t m) {
    uint32_t st = meta_status(m);
    if (!manages(m)) return CAT_SKIP;                      // not in CommandsForKey.byId at all
    if (st == AD_ST_TRANSITIVELY_KNOWN || st == AD_ST_INVALID) return CAT_SKIP;
    bool committed = st == AD_ST_COMMITTED || st == AD_ST_STABLE || st == AD_ST_APPLIED;
    if (committed && witnesses(AD_KIND_WRITE, meta_kind(m))) return CAT_ELIDABLE;
    return CAT_ALWAYS;                                     // undecided, or committed sync point
}

struct TsPack {            // per-batch packing parameters (device + host)
    uint64_t msb_min, hlc_min;
    int64_t node_min;
    uint32_t sh_msb, sh_hlc, sh_flags;   // shifts
    uint32_t total_bits;                 // width of the packed key
};

__host__ __device__ inline uint64_t ts_pack(const TsPack& p, uint64_t msb, uint64_t lsb, int32_t node) {
    return ((msb - p.msb_min) << p.sh_msb) | (((lsb >> 16) - p.hlc_min) << p.sh_hlc) |
           (((lsb >> 1) & 0xFull) << p.sh_flags) | (uint64_t)((int64_t)node - p.node_min);
}

// Device twin of ad_drop_hash (include/accord_deps.h) — must stay bit-identical (tests check it).
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint32_t drop_hash(uint64_t seed, uint32_t view, uint32_t i, uint32_t j) {
    return (uint32_t)(mix64(seed ^ mix64(((uint64_t)view << 56) ^ ((uint64_t)i << 28) ^ (uint64_t)j)) >> 32);
}

__device__ inline uint32_t lane_id() { return __lane_id(); }

template <class T>
__device__ inline T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { T u = __shfl_xor(v, o); v = u > v ? u : v; }
    return v;
}
template <class T>
__device__ inline T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// One batched per-txn CSR on the device (one Deps class of one replica view, or merged):
//   key_off[n+1], keys[nkeys], k2t_off[n+1], k2t[nk2t] (exact KeyDeps.keysToTxnIds per txn),
//   ent_off[n+1] txn-rank capacity offsets (= entry counts), tcnt[n] unique TxnIds, txns[ncap].
struct DevCsr {
    uint32_t *key_off = nullptr, *k2t_off = nullptr, *ent_off = nullptr, *tcnt = nullptr, *txns = nullptr;
    uint64_t* keys = nullptr;
    int32_t* k2t = nullptr;
    size_t nkeys = 0, nk2t = 0, ncap = 0;
};

inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }

// Raise a 0/1 "something happened" flag from one lane of every wave that saw the event.  Thousands of
// waves doing atomicOr on one address serialise at the memory side (measured: 150+ us in one launch), so
// a lane first reads the flag and only stores if it is still clear; every writer stores the same value.
__device__ inline void wave_set_flag(bool event, uint32_t* flag) {
    if (__ballot(event) && __lane_id() == 0 && *(volatile uint32_t*)flag == 0u) *(volatile uint32_t*)flag = 1u;
}

// Several buffer fills in one launch (each hipMemsetAsync is a dispatch of its own: ~16 per C2 step cost
// ~80 us of mostly launch time).  Segments are 4-byte aligned, their byte value replicated into words.
constexpr int FILL_SEGS = 16;
// Sub-segments of 4-byte words (vec = 0) or 16-byte vectors (vec = 1): a fill's 16-byte-aligned body is written with
// one dwordx4 store per lane, its unaligned head and tail with dword stores (dword stores alone ran a 36 MB fill at
// ~2.2 TB/s).
struct FillList {
    uint32_t* p[FILL_SEGS];
    uint64_t end[FILL_SEGS];     // inclusive prefix of the sub-segments' unit counts
    uint32_t v[FILL_SEGS];
    uint8_t vec[FILL_SEGS];
    int n;
};
static __global__ __launch_bounds__(256) void k_fill_multi(FillList f) {
    const uint64_t total = f.n ? f.end[f.n - 1] : 0;
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (uint64_t)gridDim.x * blockDim.x) {
        int k = 0;
#pragma unroll
        for (int q = 0; q < FILL_SEGS - 1; ++q) k += (q < f.n - 1 && x >= f.end[q]) ? 1 : 0;
        const uint64_t b = k ? f.end[k - 1] : 0;
        const uint32_t v = f.v[k];
        if (f.vec[k]) reinterpret_cast<uint4*>(f.p[k])[x - b] = make_uint4(v, v, v, v);
        else f.p[k][x - b] = v;
    }
}

// One launch for several fills (k_fill_multi): {pointer, bytes, byte value}; 4-byte aligned pointers and sizes
// (else that segment falls back to hipMemsetAsync).
struct FillSeg { void* p; size_t bytes; uint8_t v; };
inline void fill_multi(hipStream_t st, std::initializer_list<FillSeg> segs) {
    FillList f{};
    uint64_t acc = 0;
    auto add = [&](uint32_t* p, uint64_t units, uint32_t v, bool vec) {
        if (!units) return;
        acc += units;
        f.p[f.n] = p; f.end[f.n] = acc; f.v[f.n] = v; f.vec[f.n] = vec ? 1 : 0; ++f.n;
    };
    for (const FillSeg& g : segs) {
        if (!g.p || g.bytes == 0) continue;
        if (((uintptr_t)g.p & 3) || (g.bytes & 3) || f.n + 3 > FILL_SEGS) { hipMemsetAsync(g.p, g.v, g.bytes, st); continue; }
        const uint32_t v = 0x01010101u * g.v;
        uint32_t* p = (uint32_t*)g.p;
        const uint64_t words = g.bytes / 4;
        const uint64_t head = std::min<uint64_t>(words, ((16 - ((uintptr_t)p & 15)) & 15) / 4);
        const uint64_t vecs = (words - head) / 4;
        add(p, head, v, false);
        add(p + head, vecs, v, true);
        add(p + head + 4 * vecs, words - head - 4 * vecs, v, false);
    }
    if (!f.n) return;
    const uint64_t blocks = (acc + 255) / 256 < 4096 ? (acc + 255) / 256 : 4096;
    k_fill_multi<<<(unsigned)blocks, 256, 0, st>>>(f);
}

// Appends `v` for every lane with `event` to list[*count ...]: one atomic per wave (rare events: deferred txns,
// overflowing pairs), slots in lane order.
__device__ inline void wave_append(bool event, uint32_t v, uint32_t* list, uint32_t* count) {
    const uint64_t m = __ballot(event);
    if (!m) return;
    const int lane = __lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (event) list[base + __popcll(m & ((1ull << lane) - 1ull))] = v;
}

}  // namespace ad
