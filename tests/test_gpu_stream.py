"""The batch stream through the C-ABI (SURVEY §8d end-to-end): ad_load_batch_async uploads the next batch on the
copy stream while the loaded one runs, ad_load_batch_commit swaps it in, ad_fetch_merged_all pages out the three
merged classes in one call, all from / into pinned host memory (ad_host_alloc).  Checked bit-exact against the
oracle, and against the synchronous path (ad_load_batch + ad_fetch_merged) on the same batches."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, engine, workload

pytestmark = pytest.mark.gpu


def _mixed(n, seed):
    return workload.generate(n, keys_per_txn=3, keyspace=5000, range_frac=0.1, range_width_max=300, seed=seed)


def _same(a, b):
    for f in ("key_off", "keys", "k2t_off", "k2t", "txn_off", "txns"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


@pytest.mark.parametrize("ranges", [False, True])
def test_async_stream_matches_oracle(engine_factory, ranges):
    cfg = abi.make_config(32, 3, 0.1, 0xACC0D1)
    batches = [(_mixed(6000 + 500 * k, seed=k) if ranges else workload.generate(8000 + 700 * k, keys_per_txn=4,
                                                                                  keyspace=20000, seed=k))
               for k in range(4)]
    arena = engine.PinnedArena()
    try:
        pinned = [arena.batch(b) for b in batches]
        eng = engine_factory(window=32, replicas=3, drop_p=0.1, seed=0xACC0D1)
        eng.load_async(pinned[0])
        eng.load_commit()
        for k, b in enumerate(batches):
            if k + 1 < len(batches):
                eng.load_async(pinned[k + 1])      # staged while batch k runs and is paged out
            eng.run_pipeline()
            ref = O.OracleResult(b, cfg, O.FLAG_MERGE | O.FLAG_LEVELS)
            s = eng.merged_sizes()
            outs = [arena.csr(s[c], is_range=(c == abi.CLASS_RANGE)) for c in range(abi.NUM_CLASSES)]
            eng.fetch_merged_all(outs)
            for c in range(abi.NUM_CLASSES):
                assert s[c].txns == s[c].txn_cap
                assert outs[c].equal(ref.merged(c)), "batch %d merged %s" % (k, abi.CLASS_NAMES[c])
            lv, order = eng.fetch_levels((arena.empty(b["n"], np.uint32), arena.empty(b["n"], np.uint32)))
            rlv, rord = ref.levels()
            assert np.array_equal(lv, rlv) and np.array_equal(order, rord), "batch %d levels" % k
            if k + 1 < len(batches):
                eng.load_commit()
    finally:
        arena.close()


@pytest.mark.parametrize("ranges", [False, True])
def test_async_page_out_matches_the_synchronous_fetch(engine_factory, ranges):
    # ad_fetch_results_async: batch k's merged Deps + levels paged out on the copy stream while batch k + 1 is committed
    # and runs; after ad_fetch_wait the host buffers equal what the synchronous fetches returned for batch k
    batches = [(_mixed(5000 + 400 * k, seed=20 + k) if ranges else workload.generate(7000 + 600 * k, keys_per_txn=4,
                                                                                       keyspace=20000, seed=20 + k))
               for k in range(4)]
    arena = engine.PinnedArena()
    try:
        pinned = [arena.batch(b) for b in batches]
        eng = engine_factory(window=32, replicas=3, drop_p=0.1, seed=0xACC0D1)
        sync = engine_factory(window=32, replicas=3, drop_p=0.1, seed=0xACC0D1)
        eng.load_async(pinned[0])
        eng.load_commit()
        prev = None
        for k, b in enumerate(batches):
            if k + 1 < len(batches):
                eng.load_async(pinned[k + 1])
            eng.run_pipeline()
            if prev is not None:                     # batch k - 1's page-out, overlapped with batch k's pipeline
                eng.fetch_wait()
                pk, outs, lvo = prev
                sync.load(batches[pk])
                sync.run_pipeline()
                for c, want in enumerate(sync.fetch_merged_all()):
                    _same(outs[c], want)
                wl, wo = sync.fetch_levels()
                assert np.array_equal(lvo[0][:len(wl)], wl) and np.array_equal(lvo[1][:len(wo)], wo), "batch %d" % pk
            s = eng.merged_sizes()
            outs = [arena.csr(s[c], is_range=(c == abi.CLASS_RANGE)) for c in range(abi.NUM_CLASSES)]
            lvo = (arena.empty(b["n"], np.uint32), arena.empty(b["n"], np.uint32))
            eng.fetch_results_async(outs, lvo)
            prev = (k, outs, lvo)
            if k + 1 < len(batches):
                eng.load_commit()
        eng.fetch_wait()
        pk, outs, lvo = prev
        sync.load(batches[pk])
        sync.run_pipeline()
        for c, want in enumerate(sync.fetch_merged_all()):
            _same(outs[c], want)
    finally:
        arena.close()


def test_fetch_merged_all_equals_per_class(engine_factory):
    b = _mixed(20000, seed=11)
    eng = engine_factory(window=32, replicas=3, drop_p=0.1)
    eng.load(b)
    eng.preaccept_deps()
    eng.merge()
    allc = eng.fetch_merged_all()
    for c in range(abi.NUM_CLASSES):
        _same(allc[c], eng.fetch_merged(c))
    # key-only batch: the range class comes back empty
    eng.load(workload.generate(5000, keys_per_txn=2, keyspace=3000, seed=2))
    eng.preaccept_deps()
    eng.merge()
    allc = eng.fetch_merged_all()
    assert allc[abi.CLASS_RANGE].txns.size == 0 and not allc[abi.CLASS_RANGE].key_off.any()
    for c in range(abi.NUM_CLASSES):
        _same(allc[c], eng.fetch_merged(c))


def test_async_state_rules(engine_factory):
    b0 = workload.generate(3000, keys_per_txn=3, keyspace=500, seed=5)
    b1 = workload.generate(2000, keys_per_txn=3, keyspace=500, seed=6)
    eng = engine_factory(window=0, replicas=1, drop_p=0.0)
    with pytest.raises(engine.AccordDepsError):
        eng.load_commit()                                   # nothing staged
    eng.load(b0)
    eng.preaccept_deps()
    eng.merge()
    want = eng.fetch_merged(abi.CLASS_KEY)
    eng.load_async(b1)
    with pytest.raises(engine.AccordDepsError):
        eng.load_async(b0)                                  # one staged batch at a time
    _same(eng.fetch_merged(abi.CLASS_KEY), want)            # the loaded batch is untouched until the commit
    eng.load_commit()
    assert eng.n == 2000
    with pytest.raises(engine.AccordDepsError):
        eng.fetch_merged(abi.CLASS_KEY)                     # the new batch has no merged deps yet
    eng.preaccept_deps()
    eng.cfk_retain()
    with pytest.raises(engine.AccordDepsError):
        eng.load_async(b0)                                  # kept CFK rows: ad_load_batch prepends them
    eng.load(b0)
    assert eng.hist_rows > 0
