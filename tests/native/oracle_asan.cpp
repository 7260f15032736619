// The CPU oracle (oracle/oracle.cpp) under -fsanitize=address,undefined (tests/test_native_sanitizers.py): seeded
// batches of every shape the tests use — key Reads/Writes, ephemeral reads, sync points, all statuses, in-flight
// windows with drops, range txns — through oracle_run (deps, merge, levels; 1 and 3 threads; fast-path mask),
// the MaxConflicts entries with a carried map chained over batches, and every fetch.  Exit 0 with no sanitizer
// report is the pass.
#include "../../oracle/oracle.cpp"

#include <cstdio>
#include <random>

struct HostBatch {
    std::vector<uint64_t> tm, tl, em, el, keys, rs, re;
    std::vector<int32_t> tn, en;
    std::vector<uint8_t> st;
    std::vector<uint32_t> ko, ro;
    ad_batch view() {
        return ad_batch{tm.size(), tm.data(), tl.data(), tn.data(), em.data(), el.data(), en.data(), st.data(), ko.data(),
                        keys.data(), ro.data(), rs.data(), re.data()};
    }
};

static HostBatch make(std::mt19937& g, size_t n, uint64_t keyspace, bool ranges, bool mixed, uint64_t hlc0) {
    HostBatch b;
    b.ko = {0}; b.ro = {0};
    uint64_t hlc = hlc0;
    for (size_t i = 0; i < n; ++i) {
        hlc += 1 + g() % 8;
        const bool rng = ranges && g() % 10 == 0;
        int kind = g() % 2 ? AD_KIND_WRITE : AD_KIND_READ;
        if (mixed && g() % 5 == 0) kind = (int)(g() % 5);
        const uint64_t flags = ((uint64_t)kind << 1) | (rng ? 1u : 0u);
        const uint64_t msb = (1ull << 15) | (hlc >> 48), lsb = (hlc << 16) | flags;
        b.tm.push_back(msb); b.tl.push_back(lsb); b.tn.push_back(1 + (int32_t)(g() % 8));
        const bool slow = g() % 10 == 0;
        const uint64_t eh = slow ? hlc + 1 + g() % 16 : hlc;
        b.em.push_back((1ull << 15) | (eh >> 48)); b.el.push_back((eh << 16) | flags);
        b.en.push_back(slow ? 101 + (int32_t)(g() % 3) : b.tn.back());
        b.st.push_back(mixed ? (uint8_t)(g() % 8) : (uint8_t)AD_ST_APPLIED);
        if (rng) {
            uint64_t s = g() % keyspace;
            const int nr = 1 + (int)(g() % 2);
            for (int r = 0; r < nr; ++r) {
                const uint64_t w = 1 + g() % 50;
                b.rs.push_back(s); b.re.push_back(s + w);
                s += w + 1 + g() % 20;
            }
        } else {
            std::vector<uint64_t> ks;
            const int k = 1 + (int)(g() % 4);
            while ((int)ks.size() < k) {
                const uint64_t key = g() % keyspace;
                if (std::find(ks.begin(), ks.end(), key) == ks.end()) ks.push_back(key);
            }
            std::sort(ks.begin(), ks.end());
            b.keys.insert(b.keys.end(), ks.begin(), ks.end());
        }
        b.ko.push_back((uint32_t)b.keys.size());
        b.ro.push_back((uint32_t)b.rs.size());
    }
    if (b.rs.empty()) { b.rs.push_back(0); b.re.push_back(0); }     // keep data() non-null for the view
    if (b.keys.empty()) b.keys.push_back(0);
    return b;
}

static size_t fetch_all(oracle_result* r, uint32_t replicas) {
    size_t total = 0;
    for (int stage = 0; stage < 2; ++stage)
        for (uint32_t v = 0; v < (stage ? 1u : replicas); ++v)
            for (uint32_t c = 0; c < AD_NUM_CLASSES; ++c) {
                ad_csr_sizes s;
                if (oracle_sizes(r, stage, v, c, &s) != AD_OK) continue;
                std::vector<uint32_t> ko(s.n + 1), mo(s.n + 1), to(s.n + 1), tx(s.txns + 1);
                std::vector<uint64_t> ks(2 * s.keys + 1);
                std::vector<int32_t> m(s.k2t + 1);
                ad_csr_out o{ko.data(), ks.data(), mo.data(), m.data(), to.data(), tx.data()};
                oracle_fetch(r, stage, v, c, &o);
                total += s.txns;
            }
    return total;
}

int main() {
    std::mt19937 g(0xACC0D);
    size_t work = 0;
    std::vector<uint64_t> ck, cm, cl;
    std::vector<int32_t> cn;
    for (int round = 0; round < 24; ++round) {
        const bool ranges = round % 3 == 1, mixed = round % 4 == 3;
        HostBatch b = make(g, 300 + g() % 900, round % 2 ? 60 : 5000, ranges, mixed, 1000000 + 20000ull * round);
        ad_batch bv = b.view();
        if (!ranges) bv.range_off = nullptr;
        oracle_config cfg{(uint32_t)(round % 3 ? 8 : 0), 3, round % 2 ? 0.2f : 0.0f, 0, (uint64_t)round};
        for (uint32_t threads : {1u, 3u}) {
            if (threads > 1 && ranges) continue;
            const uint32_t flags = (mixed ? 0u : 4u) | 2u | (threads > 1 ? 1u : 0u);
            oracle_result* r = oracle_run(&bv, &cfg, flags, threads);
            if (const char* e = oracle_error(r)) { std::fprintf(stderr, "round %d: %s\n", round, e); return 1; }
            work += fetch_all(r, cfg.replicas);
            if (flags & 4) {
                std::vector<uint32_t> lv(bv.n), od(bv.n);
                oracle_levels(r, lv.data(), od.data());
            }
            oracle_free(r);
        }
        if (!ranges) {
            const size_t n = bv.n;
            std::vector<uint32_t> rank(3 * n);
            std::vector<uint8_t> fast(3 * n);
            if (oracle_max_conflicts(&bv, &cfg, rank.data(), fast.data()) != AD_OK) return 1;
            std::vector<uint64_t> om(3 * n), ol(3 * n);
            std::vector<int32_t> on(3 * n);
            if (oracle_max_conflicts_ts(&bv, &cfg, ck.size(), ck.data(), cm.data(), cl.data(), cn.data(), om.data(), ol.data(),
                                        on.data(), fast.data()) != AD_OK) return 1;
            oracle_result* r = oracle_run_masked(&bv, &cfg, 2u, 1, fast.data());
            work += fetch_all(r, cfg.replicas);
            oracle_free(r);
            size_t m = 0;
            oracle_max_conflicts_export(&bv, ck.size(), ck.data(), cm.data(), cl.data(), cn.data(), &m, nullptr, nullptr, nullptr,
                                        nullptr);
            std::vector<uint64_t> nk(m + 1), nm(m + 1), nl(m + 1);
            std::vector<int32_t> nn(m + 1);
            oracle_max_conflicts_export(&bv, ck.size(), ck.data(), cm.data(), cl.data(), cn.data(), &m, nk.data(), nm.data(),
                                        nl.data(), nn.data());
            nk.resize(m); nm.resize(m); nl.resize(m); nn.resize(m);
            ck.swap(nk); cm.swap(nm); cl.swap(nl); cn.swap(nn);
        }
    }
    std::printf("oracle under ASan/UBSan: 24 batches, %zu dependency TxnIds fetched, carried map %zu keys\n", work, ck.size());
    return 0;
}
