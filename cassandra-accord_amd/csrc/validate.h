// validate.h — host-side validation of caller-supplied CSRs (ad_merge_host), shared with the native host test
// (tests/native/test_validate.cpp, built with -fsanitize=address,undefined).  Plain C++: no HIP.
//
// A reply from the network must never reach a kernel as an out-of-range index: every offset array monotone from
// 0, keys strictly ascending (Range::compare for ranges), per txn sorted unique dependency ranks < n, and a
// canonical keysToTxnIds (KeyDeps.java:153-172: nKeys strictly increasing end offsets starting past the header,
// then per key strictly ascending indices into the txn's TxnId list).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>

#include "../../include/accord_deps.h"

namespace {

// Validates one caller-supplied canonical CSR over n txns (host side: a malformed reply must never reach a
// kernel as an out-of-range index).  Returns the three lengths via *keys/*k2t/*txns.
inline bool valid_part(const ad_csr_in& c, size_t n, int kw, size_t* nkeys, size_t* nk2t, size_t* ntx, std::string& why) {
    if (!c.key_off || !c.k2t_off || !c.txn_off) { why = "null offsets"; return false; }
    if (c.key_off[0] != 0 || c.k2t_off[0] != 0 || c.txn_off[0] != 0) { why = "offsets must start at 0"; return false; }
    for (size_t i = 0; i < n; ++i) {
        const uint32_t k0 = c.key_off[i], k1 = c.key_off[i + 1], m0 = c.k2t_off[i], m1 = c.k2t_off[i + 1];
        const uint32_t t0 = c.txn_off[i], t1 = c.txn_off[i + 1];
        if (k1 < k0 || m1 < m0 || t1 < t0) { why = "offsets not monotone at txn " + std::to_string(i); return false; }
        const uint32_t nk = k1 - k0, len = m1 - m0, nt = t1 - t0;
        if ((nk == 0) != (len == 0) || (nk == 0) != (nt == 0) || len < nk) { why = "inconsistent CSR at txn " + std::to_string(i); return false; }
        // keys strictly ascending (Range::compare for ranges)
        for (uint32_t k = k0 + 1; k < k1; ++k) {
            const uint64_t* a = c.keys + (size_t)kw * (k - 1);
            const uint64_t* b = c.keys + (size_t)kw * k;
            const bool lt = kw == 1 ? a[0] < b[0] : (a[0] < b[0] || (a[0] == b[0] && a[1] < b[1]));
            if (!lt) { why = "keys not strictly ascending at txn " + std::to_string(i); return false; }
        }
        for (uint32_t x = t0; x < t1; ++x)
            if (c.txns[x] >= n || (x > t0 && c.txns[x] <= c.txns[x - 1])) { why = "TxnIds not sorted unique ranks at txn " + std::to_string(i); return false; }
        uint32_t prev = nk;
        for (uint32_t k = 0; k < nk; ++k) {
            const uint32_t end = (uint32_t)c.k2t[m0 + k];
            if (end < prev || end > len || (end == prev)) { why = "keysToTxnIds header invalid at txn " + std::to_string(i); return false; }
            for (uint32_t x = prev; x < end; ++x) {
                const int32_t ix = c.k2t[m0 + x];
                if (ix < 0 || (uint32_t)ix >= nt || (x > prev && ix <= c.k2t[m0 + x - 1])) { why = "keysToTxnIds index invalid at txn " + std::to_string(i); return false; }
            }
            prev = end;
        }
        if (prev != len) { why = "keysToTxnIds length mismatch at txn " + std::to_string(i); return false; }
    }
    *nkeys = c.key_off[n]; *nk2t = c.k2t_off[n]; *ntx = c.txn_off[n];
    return true;
}

}  // namespace
