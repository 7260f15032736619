"""Deps wire formats (accord_amd/wire.py): the Maelstrom JSON form of Json.DEPS_ADAPTER
(accord-maelstrom/.../Json.java:316-428) written from the per-txn CSR rows and read back through Builder semantics.

CPU: a hand-written known answer (the adapter's shape, node ids, signed longs, order), refusals, and a round trip of
every row of every class of oracle deps (keys and ranges).  GPU: replies rebuilt from their JSON go through
ad_merge_host and equal the device's own merge of the same replies."""
import json

import numpy as np
import pytest

import oracle as O
from accord_amd import abi, wire, workload


def _small_batch():
    # three txns; TxnId = (msb, lsb, node); lsb carries the kind in bits 1..3 (Write = 1)
    b = {"n": 3,
         "txn_msb": np.array([10, 10, 11], np.uint64), "txn_lsb": np.array([2, 0x10002, 2], np.uint64),
         "txn_node": np.array([1, 2, 0], np.int32)}
    return b


def test_node_and_timestamp_encoding():
    assert wire.node_to_json(0) is None and wire.node_to_json(5) == "n5" and wire.node_to_json(-3) == "c-3"
    assert wire.node_from_json(None) == 0 and wire.node_from_json("n17") == 17 and wire.node_from_json("c4") == 4
    with pytest.raises(ValueError):
        wire.node_from_json("x1")
    big = (1 << 63) + 5                                   # a u64 with the top bit set is a negative Java long
    assert wire.ts_to_json(big, 7, 2) == [-(1 << 63) + 5, 7, "n2"]
    assert wire.ts_from_json([-(1 << 63) + 5, 7, "n2"]) == (big, 7, 2)


def test_known_answer_key_deps():
    t = wire.TxnTable(_small_batch())
    # txn 2's deps: key 5 -> {0, 1}, key 9 -> {1}; ranges: (0, 100] -> {0}
    key = abi.Csr(np.array([0, 0, 0, 2], np.uint32), np.array([5, 9], np.uint64), np.array([0, 0, 0, 5], np.uint32),
                  np.array([4, 5, 0, 1, 1], np.int32), np.array([0, 0, 0, 2], np.uint32), np.array([0, 1], np.uint32))
    empty = abi.Csr(np.zeros(4, np.uint32), np.zeros(0, np.uint64), np.zeros(4, np.uint32), np.zeros(0, np.int32),
                    np.zeros(4, np.uint32), np.zeros(0, np.uint32))
    rng = abi.Csr(np.array([0, 0, 0, 1], np.uint32), np.array([0, 100], np.uint64), np.array([0, 0, 0, 2], np.uint32),
                  np.array([2, 0], np.int32), np.array([0, 0, 0, 1], np.uint32), np.array([0], np.uint32), True)
    js = wire.to_json(t, key, empty, rng, 2)
    assert js == {"keyDeps": [[5, [10, 2, "n1"]], [5, [10, 0x10002, "n2"]], [9, [10, 0x10002, "n2"]]],
                  "rangeDeps": [[0, 100, [10, 2, "n1"]]], "directKeyDeps": []}
    s = wire.dumps(js)
    assert s.startswith('{"keyDeps":[[5,[10,2,"n1"]]')
    # read back from a shuffled, duplicated entry list (KeyDeps.Builder semantics)
    obj = json.loads(s)
    obj["keyDeps"] = [obj["keyDeps"][2], obj["keyDeps"][0], obj["keyDeps"][1], obj["keyDeps"][0]]
    rels = wire.from_json(obj, t)
    assert rels["key"] == ([5, 9], [0, 1], [4, 5, 0, 1, 1])
    assert rels["range"] == ([(0, 100)], [0], [2, 0])
    assert rels["direct"] == ([], [], [])


def test_refusals():
    t = wire.TxnTable(_small_batch())
    with pytest.raises(ValueError):
        wire.from_json({"keyDeps": [[1, [99, 0, None]]]}, t)      # a TxnId outside the batch
    with pytest.raises(ValueError):
        wire.from_json({"other": []}, t)                          # Json.java:420 'Unknown name'


@pytest.mark.parametrize("range_frac", [0.0, 0.2])
def test_round_trip_oracle_deps(range_frac):
    kinds = np.random.default_rng(1).choice([abi.KIND_READ, abi.KIND_WRITE, abi.KIND_SYNC_POINT,
                                             abi.KIND_EXCLUSIVE_SYNC_POINT, abi.KIND_EPHEMERAL_READ],
                                            size=1500, p=[0.4, 0.4, 0.07, 0.07, 0.06])  # direct deps need sync kinds
    b = workload.generate(1500, keys_per_txn=3, keyspace=500, kinds=kinds, range_frac=range_frac,
                          range_width_max=64, seed=77)
    res = O.OracleResult(b, abi.make_config(16, 2, 0.1, 3), O.FLAG_MERGE)
    t = wire.TxnTable(b)
    classes = [abi.CLASS_KEY, abi.CLASS_DIRECT_KEY] + ([abi.CLASS_RANGE] if range_frac else [])
    for v in range(2):
        csr = {c: res.deps(v, c) for c in classes}
        assert all(csr[c].entries() > 0 for c in classes)
        back = {c: [] for c in classes}
        for i in range(b["n"]):
            js = json.loads(wire.dumps(wire.to_json(t, csr[abi.CLASS_KEY], csr[abi.CLASS_DIRECT_KEY],
                                                    csr.get(abi.CLASS_RANGE), i)))
            rels = wire.from_json(js, t)
            back[abi.CLASS_KEY].append(rels["key"])
            back[abi.CLASS_DIRECT_KEY].append(rels["direct"])
            if abi.CLASS_RANGE in csr:
                back[abi.CLASS_RANGE].append(rels["range"])
        for c in classes:
            rebuilt = wire.relations_to_csr(back[c], is_range=(c == abi.CLASS_RANGE))
            assert rebuilt.first_difference(csr[c]) is None, "view %d class %d" % (v, c)


@pytest.mark.gpu
def test_gpu_merge_of_json_replies(engine_factory):
    """Replies that crossed the wire as JSON merge on the device (ad_merge_host) exactly as the device's own."""
    b = workload.generate(3000, keys_per_txn=3, keyspace=800, range_frac=0.1, range_width_max=64, seed=5)
    eng = engine_factory(window=16, replicas=3, drop_p=0.2, seed=11)
    eng.load(b)
    eng.preaccept_deps()
    replies = [[eng.fetch_deps(v, c) for c in range(abi.NUM_CLASSES)] for v in range(3)]
    eng.merge()
    want = [eng.fetch_merged(c) for c in range(abi.NUM_CLASSES)]
    t = wire.TxnTable(b)
    decoded = []
    for v in range(3):
        rows = {"key": [], "direct": [], "range": []}
        for i in range(b["n"]):
            js = json.loads(wire.dumps(wire.to_json(t, replies[v][abi.CLASS_KEY], replies[v][abi.CLASS_DIRECT_KEY],
                                                    replies[v][abi.CLASS_RANGE], i)))
            rels = wire.from_json(js, t)
            for name in rows:
                rows[name].append(rels[name])
        rep = [None] * abi.NUM_CLASSES
        rep[abi.CLASS_KEY] = wire.relations_to_csr(rows["key"])
        rep[abi.CLASS_DIRECT_KEY] = wire.relations_to_csr(rows["direct"])
        rep[abi.CLASS_RANGE] = wire.relations_to_csr(rows["range"], is_range=True)
        decoded.append(rep)
    eng.merge_host(decoded)
    for c in range(abi.NUM_CLASSES):
        assert eng.fetch_merged(c).first_difference(want[c]) is None, "class %d" % c
