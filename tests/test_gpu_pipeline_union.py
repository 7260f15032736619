"""ad_run_pipeline's merged Deps — by default k_merge_ref over the R replies' CSRs (merge.hip merge_cap: references to an
identical reply, the other txns merged in the same pass, compacted by merged_ready for the fetch), or, with ad_set_pipeline_union, the deps stage's union
view (deps.hip stage_deps): the replies, the merged Deps (per class, ad_fetch_merged and ad_fetch_merged_all) and the
levels equal the oracle's Deps.merge (RelationMultiMap.LinearMerger, utils/RelationMultiMap.java:284-406) on batches
that take every branch of the deps stage: the fused tile kernel, the three-kernel path (hot keys), direct classes
(sync points), txns with more than four keys (fill walk + k_txn_union), inline-id overflow re-walks, 1, 2, 4 and 7
replica views (k_merge_ref's register path for <= 4 views, its serial loops above and for long lists)."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload

pytestmark = pytest.mark.gpu


def _mixed(n, seed):
    rng = np.random.default_rng(seed)
    kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_EPHEMERAL_READ, abi.KIND_SYNC_POINT,
                        abi.KIND_EXCLUSIVE_SYNC_POINT], p=[0.4, 0.4, 0.1, 0.05, 0.05], size=n)
    status = rng.integers(0, 8, size=n).astype(np.uint8)
    return workload.generate(n, keys_per_txn=3, keyspace=5000, seed=seed, kinds=kinds, status=status)


CASES = {
    "c2": (lambda: workload.config("C2", n=50000, seed=9), (32, 3, 0.1)),
    "mixed_direct": (lambda: _mixed(20000, 4), (16, 3, 0.2)),
    "hot_keys": (lambda: workload.generate(20000, keys_per_txn=2, keyspace=50, seed=5), (32, 3, 0.1)),
    "wide": (lambda: workload.generate(10000, keys_per_txn=6, keyspace=20000, seed=6), (32, 3, 0.1)),
    "one_view": (lambda: workload.config("C2", n=30000, seed=7), (0, 1, 0.0)),
    "seven_views": (lambda: workload.generate(20000, keys_per_txn=4, keyspace=30000, seed=8), (64, 7, 0.3)),
    "c3": (lambda: workload.config("C3", n=20000, seed=10), (32, 3, 0.1)),
    "two_views": (lambda: workload.config("C2", n=30000, seed=11), (48, 2, 0.3)),
    "four_views": (lambda: workload.generate(20000, keys_per_txn=4, keyspace=3000, seed=12), (40, 4, 0.25)),
}


@pytest.mark.parametrize("union", [False, True], ids=["merge", "union_view"])
@pytest.mark.parametrize("name", list(CASES))
def test_pipeline_union_equals_oracle(engine_factory, name, union):
    make, (w, r, d) = CASES[name]
    b = make()
    eng = engine_factory(window=w, replicas=r, drop_p=d, seed=0x5EED)
    eng.set_pipeline_union(union)
    eng.load(b)
    eng.run_pipeline()
    ref = O.OracleResult(b, abi.make_config(w, r, d, 0x5EED), O.FLAG_MERGE | O.FLAG_LEVELS)
    for v in range(r):
        for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY):
            got, want = eng.fetch_rows(v, c, 0, b["n"]), ref.deps(v, c)
            assert got.equal(want), "%s view %d class %d differs at txn %s" % (name, v, c, got.first_difference(want))
    merged = [eng.fetch_rows(r, c, 0, b["n"]) for c in range(abi.NUM_CLASSES)]   # view == replicas: the merged Deps
    for c in range(abi.NUM_CLASSES):
        want = ref.merged(c)
        assert merged[c].equal(want), "%s merged class %d differs at txn %s" % (name, c, merged[c].first_difference(want))
    allm = eng.fetch_merged_all()
    for c in range(abi.NUM_CLASSES):
        assert allm[c].equal(merged[c]), "%s: ad_fetch_merged_all class %d" % (name, c)
    s = eng.merged_sizes()
    for c in range(abi.NUM_CLASSES):
        assert s[c].txns == s[c].txn_cap == len(merged[c].txns)
    if not union:      # the merged entries k_merge_ref counted (per-workgroup sums) == the merged Deps' entries
        want_e = sum(len(merged[c].k2t) - len(merged[c].keys) for c in range(abi.NUM_CLASSES))
        assert eng.last_times()["merged_entries"] == want_e
    lv, order = eng.fetch_levels()
    rlv, rorder = ref.levels()
    assert np.array_equal(lv, rlv) and np.array_equal(order, rorder)
    # the staged calls after the pipeline: ad_merge_deps on the pipeline's deps, then a plain preaccept + merge
    eng.merge()
    assert all(eng.fetch_merged(c).equal(merged[c]) for c in range(abi.NUM_CLASSES))
    eng.preaccept_deps()
    eng.merge()
    assert all(eng.fetch_merged(c).equal(merged[c]) for c in range(abi.NUM_CLASSES))
    assert eng.merged_sizes()[abi.CLASS_KEY].txns == s[abi.CLASS_KEY].txns


@pytest.mark.parametrize("name", ["c2", "one_view"])
def test_gather_items_counts_multi_entry_segments(engine_factory, name):
    """ad_stage_times.gather_items (k_seg_fuse's gathered records, the byte model's G) == the entries whose key holds
    more than one entry of the batch; walk_items == those entries minus one per such key."""
    make, (w, r, d) = CASES[name]
    b = make()
    eng = engine_factory(window=w, replicas=r, drop_p=d, seed=0x5EED)
    eng.load(b)
    eng.run_pipeline()
    st = eng.last_times()
    _, cnt = np.unique(np.asarray(b["keys"]), return_counts=True)
    multi = cnt[cnt > 1]
    assert st["gather_items"] == int(multi.sum())
    assert st["walk_items"] == int(multi.sum()) - len(multi)


def test_speculative_key_sort_across_key_spreads(engine_factory):
    """stage_prepare sorts the keys right behind k_pack with the previous batch's key spread, before reading this
    batch's Params: a wider spread (more 8-bit passes) must redo the sort, a narrower one keeps it (an extra pass
    over an all-zero digit).  One handle, batches of 10-, 24-, 10- and 17-bit key spreads, each == the oracle."""
    eng = engine_factory(window=16, replicas=3, drop_p=0.1, seed=0x5EED)
    for i, keyspace in enumerate((1000, 10_000_000, 1000, 100_000)):
        b = workload.generate(20000, keys_per_txn=3, keyspace=keyspace, seed=40 + i)
        eng.load(b)
        eng.run_pipeline()
        ref = O.OracleResult(b, abi.make_config(16, 3, 0.1, 0x5EED), O.FLAG_MERGE | O.FLAG_LEVELS)
        for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY):
            got = eng.fetch_rows(3, c, 0, b["n"])
            assert got.equal(ref.merged(c)), "batch %d (keyspace %d) merged class %d" % (i, keyspace, c)
        lv, order = eng.fetch_levels()
        rlv, rorder = ref.levels()
        assert np.array_equal(lv, rlv) and np.array_equal(order, rorder), "batch %d levels" % i
