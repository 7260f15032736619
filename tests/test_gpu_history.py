"""CommandsForKey state across batches on the device (ad_cfk_retain / ad_load_batch with history, csrc/history_kernels.h):
a stream of batches through one handle, each batch's PreAccept deps (every view and class), Deps.merge and MaxConflicts
proposal equal to the oracle resolving the whole stream at once, and the kept rows equal to the restated rule
(tests/test_oracle_history.py: keep_rows)."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, engine, workload
from test_oracle_history import _concat, _mapped, _take, keep_rows

pytestmark = pytest.mark.gpu


def _stream(n_b, nb, keyspace, window, seed, kinds_mix=True):
    rng = np.random.default_rng(seed)
    n = n_b * nb
    kinds = status = None
    if kinds_mix:
        kinds = rng.choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT,
                            abi.KIND_EPHEMERAL_READ], size=n, p=[0.4, 0.4, 0.07, 0.07, 0.06])
        status = rng.choice([abi.ST_APPLIED, abi.ST_COMMITTED, abi.ST_STABLE, abi.ST_PREACCEPTED, abi.ST_ACCEPTED,
                             abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN], size=n,
                            p=[0.55, 0.1, 0.1, 0.08, 0.07, 0.05, 0.05]).astype(np.uint8)
    return workload.generate(n, keys_per_txn=3, keyspace=keyspace, kinds=kinds, status=status, slow_frac=0.3,
                             bump_max=60, seed=seed)


@pytest.mark.parametrize("n_b,nb,keyspace,window,drop,replicas",
                         [(4, 1200, 300, 16, 0.2, 2), (3, 20000, 20000, 32, 0.1, 3), (5, 3000, 60, 0, 0.0, 1)])
def test_history_stream_equals_whole_stream(engine_factory, n_b, nb, keyspace, window, drop, replicas):
    stream = _stream(n_b, nb, keyspace, window, seed=keyspace + nb)
    cfg = abi.make_config(window, replicas, drop, 0x5EED)
    full = O.OracleResult(stream, cfg, O.FLAG_MERGE)
    frank, ffast = O.max_conflicts(stream, cfg)
    ident = np.arange(stream["n"])
    eng = engine_factory(window=window, replicas=replicas, drop_p=drop, seed=0x5EED)
    hist, hgid = None, np.zeros(0, np.uint32)
    for k in range(n_b):
        rows = np.arange(k * nb, (k + 1) * nb)
        new = _take(stream, rows)
        eng.load(new)
        H, gid = eng.cfk_rows()
        assert H == len(hgid) and np.array_equal(gid[:H], hgid) and np.array_equal(gid[H:], rows)
        eng.preaccept_deps()
        for v in range(replicas):
            for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY):
                got, want = eng.fetch_deps(v, c), full.deps(v, c)
                for x in range(nb):
                    assert _mapped(got, H + x, gid) == _mapped(want, k * nb + x, ident), \
                        "batch %d view %d class %d txn %d" % (k, v, c, k * nb + x)
        rank, fast = eng.max_conflicts()              # global ranks (the rows' gid)
        assert np.array_equal(rank[:, H:], frank[:, rows]) and np.array_equal(fast[:, H:], ffast[:, rows])
        eng.merge()
        for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY):
            got, want = eng.fetch_merged(c), full.merged(c)
            for x in range(0, nb, 7):
                assert _mapped(got, H + x, gid) == _mapped(want, k * nb + x, ident)
        # the kept rows: the restated rule over the same combined batch
        comb = new if hist is None else _concat(hist, new)
        keep = keep_rows(comb, gid, window)
        assert eng.cfk_retain() == len(keep)
        hist, hgid = _take(comb, keep), gid[keep]


def test_history_refusals_and_reset(engine_factory):
    stream = _stream(2, 2000, 200, 16, seed=9, kinds_mix=False)
    eng = engine_factory(window=16, replicas=2, drop_p=0.1)
    eng.load(_take(stream, np.arange(2000)))
    eng.preaccept_deps()
    kept = eng.cfk_retain()
    assert kept > 0
    eng.load(_take(stream, np.arange(2000, 4000)))
    assert eng.hist_rows == kept
    eng.preaccept_deps()
    eng.merge()
    eng.exec_levels()                                 # kept rows and new txns in one order (test_gpu_cfk_state.py)
    with pytest.raises(engine.AccordDepsError):
        eng.accept_deps()
    # a batch that does not continue the TxnId order is rejected (the kept rows precede it)
    eng.cfk_retain()
    eng.load(_take(stream, np.arange(0, 2000)))
    with pytest.raises(engine.AccordDepsError):
        eng.preaccept_deps()
    # reset: the next batch is a closed world again
    eng.cfk_reset()
    eng.load(_take(stream, np.arange(2000, 4000)))
    assert eng.hist_rows == 0
    eng.preaccept_deps()
    eng.merge()
    eng.exec_levels()
