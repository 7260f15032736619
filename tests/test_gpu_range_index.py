"""The interval index over range commands (range_index.h, the device form of SearchableRangeList /
CheckpointIntervalArray, utils/SearchableRangeList.java:33-131): layouts that defeat a fixed query window.

* one very wide range among narrow ones — every query's candidate window used to span the widest range;
* RangeDepsTest.generateNemesisRanges (test/primitives/RangeDepsTest.java:220-237): staircases of ranges
  [i, i + width) shared round-robin by a few "nemesis" txns, with and without one narrow [i, i + 1) per
  nemesis entry (testNemesisRanges / testHalfNemesisRanges);
* at 1M txns with whole-keyspace ranges mixed in, exact prefix parity against the oracle and a time bound
  that the old window scan (every query walking all Q entries) misses by orders of magnitude.
Every class of the deps, the merged Deps and (where cheap) levels bit-exact vs the oracle; the same layouts
also run the index from ad_max_conflicts and ad_recover.
"""
import time

import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload
from test_gpu_parity import check

pytestmark = pytest.mark.gpu


def with_ranges(b, starts, ends, owners):
    """Replace batch b's range footprints: txns `owners` (ascending, with repeats for several ranges) become
    range-domain Reads with the given (start, end] ranges (sorted, disjoint per txn)."""
    n = b["n"]
    owners = np.asarray(owners, np.int64)
    is_range = np.zeros(n, bool)
    is_range[owners] = True
    kind = np.where(is_range, abi.KIND_READ, (b["txn_lsb"].astype(np.uint64) >> np.uint64(1)) & np.uint64(7))
    flags = (kind.astype(np.uint64) << np.uint64(1)) | is_range.astype(np.uint64)
    b["txn_lsb"] = (b["txn_lsb"].astype(np.uint64) & ~np.uint64(0xF)) | flags
    b["exec_lsb"] = (b["exec_lsb"].astype(np.uint64) & ~np.uint64(0xF)) | flags
    ko = b["key_off"].astype(np.int64)
    b["keys"] = np.ascontiguousarray(b["keys"][np.repeat(~is_range, np.diff(ko))])
    b["key_off"] = np.concatenate([[0], np.cumsum(np.where(is_range, 0, np.diff(ko)))]).astype(np.uint32)
    cnt = np.bincount(owners, minlength=n)
    b["range_off"] = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    b["range_start"] = np.asarray(starts, np.uint64)
    b["range_end"] = np.asarray(ends, np.uint64)
    return b


def wide_among_narrow(n, keyspace, frac, n_wide, seed):
    rng = np.random.default_rng(seed)
    b = workload.generate(n, 3, keyspace, "uniform", seed=seed)
    owners = np.sort(rng.choice(n, size=int(n * frac), replace=False))
    s = rng.integers(0, keyspace - 20, size=len(owners)).astype(np.int64)
    e = s + rng.integers(1, 16, size=len(owners))
    wide = np.zeros(len(owners), bool)                       # whole-keyspace ranges, early and throughout
    wide[np.linspace(0, len(owners) - 1, n_wide).astype(np.int64)] = True
    s[wide], e[wide] = 0, keyspace + 1
    return with_ranges(b, s, e, owners)


def nemesis(width, nemesis_txns, range_count, non_nemesis_per, n_key_txns, seed):
    """generateNemesisRanges' layout as range-domain Reads, interleaved with key txns over the same domain."""
    non = nemesis_txns * non_nemesis_per
    rc = range_count // (1 + non_nemesis_per)
    build = {}
    for i in range(rc):
        build.setdefault(i % nemesis_txns, []).append((i, i + width))
        for _ in range(non_nemesis_per):
            build.setdefault(nemesis_txns + (i % non), []).append((i, i + 1))
    domain = rc + width
    n_range = nemesis_txns + non
    n = n_range + n_key_txns
    rng = np.random.default_rng(seed)
    b = workload.generate(n, 2, domain + 2, "uniform", seed=seed)
    owners_txn = np.sort(rng.choice(n, size=n_range, replace=False))
    starts, ends, owners = [], [], []
    for t, rows in zip(owners_txn, (build[k] for k in range(n_range))):
        # Ranges.of: sorted, overlapping/adjacent ranges merged ((start, end] semantics: touching ranges merge)
        rows = sorted(rows)
        merged = [list(rows[0])]
        for s, e in rows[1:]:
            if s <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], e)
            else:
                merged.append([s, e])
        for s, e in merged:
            starts.append(s)
            ends.append(e)
            owners.append(t)
    return with_ranges(b, starts, ends, owners)


@pytest.mark.parametrize("seed", [1, 2])
def test_one_wide_range_among_narrow(engine_factory, seed):
    check(engine_factory, wide_among_narrow(12000, 60000, 0.2, 5, seed), window=16)


@pytest.mark.parametrize("width,ntx,non", [(64, 8, 0), (64, 8, 1), (7, 3, 1), (300, 1, 0)])
def test_rangedeps_nemesis_layouts(engine_factory, width, ntx, non):
    check(engine_factory, nemesis(width, ntx, 1000, non, 3000, seed=width + ntx), window=8)


def test_index_serves_max_conflicts_and_recovery(engine_factory):
    b = wide_among_narrow(6000, 30000, 0.2, 4, 7)
    eng = engine_factory(window=16, replicas=3, drop_p=0.1, seed=0xC0DE)
    eng.load(b)
    eng.preaccept_deps()
    rank, fast = eng.max_conflicts()
    orank, ofast = O.max_conflicts(b, abi.make_config(16, 3, 0.1, 0xC0DE))
    assert np.array_equal(rank, orank) and np.array_equal(fast, ofast)
    # BeginRecovery over a mixed-status batch whose single ranges are widened to the whole key space
    from test_oracle_recovery import _mixed
    from test_gpu_recovery import _same
    b = _mixed(900, 200, 0.2, 5)
    ro = b["range_off"].astype(np.int64)
    one = np.nonzero(np.diff(ro) == 1)[0]
    for t in one[::4]:
        b["range_start"][ro[t]], b["range_end"][ro[t]] = 0, 201
    eng = engine_factory(window=16, replicas=1, drop_p=0.2, seed=5)
    eng.load(b)
    eng.accept_deps()
    eng.merge()
    merged = [eng.fetch_merged(c) for c in range(3)]
    rows = [i for i in range(b["n"]) if b["status"][i] < abi.ST_COMMITTED]
    _same(eng.recover(rows), O.recover(b, merged, rows), rows)


def test_full_size_wide_ranges_prefix_and_time(engine_factory):
    # 1M txns, 5% range txns (Q ~ 52k), four of them spanning the whole key space: the old windowed join walked
    # every entry that starts below the query key (~26k on average) for each of the 1M queries, in both passes
    n = 1 << 20
    b = wide_among_narrow(n, 10_000_000, 0.05, 4, 11)
    eng = engine_factory(window=32, replicas=3, drop_p=0.1, seed=0xACC0D1)
    eng.load(b)
    eng.preaccept_deps()                       # warm (allocations)
    eng.load(b)
    t0 = time.perf_counter()
    eng.preaccept_deps()
    dt = time.perf_counter() - t0
    print("deps at 1M with whole-keyspace ranges: %.1f ms" % (dt * 1e3))
    assert dt < 2.0, "range join took %.2f s" % dt
    k = 6000
    ref = O.OracleResult(workload.slice_batch(b, 0, k), abi.make_config(32, 3, 0.1, 0xACC0D1), 0)
    from test_gpu_fullsize import prefix
    for v in range(3):
        for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY, abi.CLASS_RANGE):
            assert prefix(eng.fetch_deps(v, c), k).equal(ref.deps(v, c)), "view %d class %d prefix differs" % (v, c)
