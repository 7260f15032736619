"""CommandsForKey state across batches on the oracle: a store's batches continue one TxnId order,
and between batches it keeps only the txns whose CFK entries a later query can still see (csrc/history_kernels.h,
restated below).  The deps of every batch's txns, resolved over [kept rows | new txns] with global arrival ranks
(oracle_run_gid), must equal those of the whole stream resolved at once — the pruning argument of Pruning.java:164-233
(tests/test_oracle_prune.py checks the oracle's own prefix pruning the same way)."""
import numpy as np
import pytest

import oracle as O
from accord_amd import abi, workload

R, W, SP, ESP = abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT, abi.KIND_EXCLUSIVE_SYNC_POINT
COMMITTED = (abi.ST_COMMITTED, abi.ST_STABLE, abi.ST_APPLIED)


def _ts(msb, lsb, node):
    return (int(msb), int(lsb) >> 16, int(lsb) & 0x1E, int(node))


def _take(b, rows):
    """Sub-batch of rows (key CSR rebuilt)."""
    out = {"n": len(rows)}
    for f in ("txn_msb", "txn_lsb", "txn_node", "exec_msb", "exec_lsb", "exec_node", "status"):
        out[f] = np.ascontiguousarray(b[f][rows])
    ko = b["key_off"].astype(np.int64)
    cnt = (ko[1:] - ko[:-1])[rows]
    out["key_off"] = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    out["keys"] = np.concatenate([b["keys"][ko[r]:ko[r + 1]] for r in rows]).astype(np.uint64) if len(rows) else np.zeros(0, np.uint64)
    out["range_off"] = out["range_start"] = out["range_end"] = None
    return out


def _concat(a, b):
    out = {"n": a["n"] + b["n"]}
    for f in ("txn_msb", "txn_lsb", "txn_node", "exec_msb", "exec_lsb", "exec_node", "status", "keys"):
        out[f] = np.concatenate([a[f], b[f]])
    out["key_off"] = np.concatenate([a["key_off"][:-1], b["key_off"] + a["key_off"][-1]]).astype(np.uint32)
    out["range_off"] = out["range_start"] = out["range_end"] = None
    return out


def keep_rows(b, gid, window):
    """history_kernels.h k_hist_seg_wmax + k_hist_keep: rows a later query or the execution order can still need
    (statuses are current: only INVALID rows and APPLIED rows no later mapReduceActive sees are dropped)."""
    n = b["n"]
    kind = (b["txn_lsb"] >> np.uint64(1)) & np.uint64(7)
    ex = [_ts(b["exec_msb"][i], b["exec_lsb"][i], b["exec_node"][i]) for i in range(n)]
    last = _ts(b["txn_msb"][n - 1], b["txn_lsb"][n - 1], b["txn_node"][n - 1])
    nxt = int(gid[n - 1]) + 1
    wlo = nxt - window if window else nxt
    ko = b["key_off"]
    mk = {}
    for i in range(n):
        if kind[i] == W and b["status"][i] in COMMITTED and ex[i] <= last:
            for k in b["keys"][ko[i]:ko[i + 1]]:
                k = int(k)
                if k not in mk or ex[i] > mk[k]:
                    mk[k] = ex[i]
    keep = []
    for i in range(n):
        if int(gid[i]) >= wlo:
            keep.append(i)
            continue
        managed = kind[i] in (R, W, SP, ESP)
        st = b["status"][i]
        for k in b["keys"][ko[i]:ko[i + 1]]:
            k = int(k)
            prunable = st == abi.ST_INVALID or (
                st == abi.ST_APPLIED and (not managed or (kind[i] in (R, W) and k in mk and ex[i] < mk[k])))
            if not prunable:
                keep.append(i)
                break
    return np.array(keep, np.int64)


def _mapped(csr, i, gid):
    ks, txns, k2t = csr.txn(i)
    return ks.tolist(), [int(gid[t]) for t in txns], k2t.tolist()


@pytest.mark.parametrize("window,drop,keyspace", [(16, 0.2, 300), (0, 0.0, 120), (32, 0.1, 3000)])
def test_history_batches_equal_whole_stream(window, drop, keyspace):
    rng = np.random.default_rng(keyspace + window)
    n_b, nb = 4, 1200
    kinds = rng.choice([R, W, SP, ESP, abi.KIND_EPHEMERAL_READ], size=n_b * nb, p=[0.4, 0.4, 0.07, 0.07, 0.06])
    status = rng.choice([abi.ST_APPLIED, abi.ST_COMMITTED, abi.ST_STABLE, abi.ST_PREACCEPTED, abi.ST_ACCEPTED,
                         abi.ST_INVALID, abi.ST_TRANSITIVELY_KNOWN], size=n_b * nb,
                        p=[0.55, 0.1, 0.1, 0.08, 0.07, 0.05, 0.05]).astype(np.uint8)
    stream = workload.generate(n_b * nb, keys_per_txn=3, keyspace=keyspace, kinds=kinds, status=status,
                               slow_frac=0.3, bump_max=60, seed=keyspace)
    cfg = abi.make_config(window, 2, drop, 0x5EED)
    full = O.OracleResult(stream, cfg, O.FLAG_MERGE)
    hist, hgid = None, np.zeros(0, np.uint32)
    kept_sizes = []
    for k in range(n_b):
        rows = np.arange(k * nb, (k + 1) * nb)
        new = _take(stream, rows)
        comb = new if hist is None else _concat(hist, new)
        gid = np.concatenate([hgid, rows.astype(np.uint32)])
        res = O.OracleResult(comb, cfg, O.FLAG_MERGE, gid=gid)
        H = len(hgid)
        for v in range(2):
            for c in (abi.CLASS_KEY, abi.CLASS_DIRECT_KEY):
                got, want = res.deps(v, c), full.deps(v, c)
                for x in range(nb):
                    assert _mapped(got, H + x, gid) == _mapped(want, k * nb + x, np.arange(n_b * nb)), \
                        "batch %d view %d class %d txn %d" % (k, v, c, k * nb + x)
        keep = keep_rows(comb, gid, window)
        hist, hgid = _take(comb, keep), gid[keep]
        done = np.isin(comb["status"][keep], (abi.ST_APPLIED, abi.ST_INVALID))
        kept_sizes.append(int(done.sum()))
        # every row that still executes or may still be preaccepted stays (statuses are current between batches)
        live = ~np.isin(comb["status"], (abi.ST_APPLIED, abi.ST_INVALID))
        assert np.isin(np.nonzero(live)[0], keep).all()
    # the applied rows kept are what a later query can still see (in flight, each key's last applied Write and
    # what executes after it): bounded on dense keyspaces; on a sparse one every once-touched key keeps its
    # entry, as a live CommandsForKey does until a committed Write there lets Pruning drop it
    assert all(s < (k + 1) * nb for k, s in enumerate(kept_sizes))
    if keyspace <= 300:
        assert max(kept_sizes) < 2 * nb
