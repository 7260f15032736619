"""bench.py's N > 1 transport choice on CPU (gloo, world 2): when RCCL cannot serve the group, every rank falls back to
the host transport together — ranks sharing one GPU, rank 0 without a unique id, or an ncclCommInitRank failure on one
rank (the rank whose init succeeded drops its communicator) — and with RCCL usable the RCCL transport is kept
(bench.pick_transport over accord_amd.sharding.RcclTransport, with a stand-in store: no GPU here)."""
import os
import socket
import sys

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Eng:
    def __init__(self, device):
        self.device = device


class _Store:
    """The two calls RcclTransport makes on a store, recorded (no device)."""

    def __init__(self, device, fail_init):
        self.eng = _Eng(device)
        self.fail_init = fail_init
        self.inits = self.destroys = 0

    def comm_init(self, world, rank, uid):
        from accord_amd import engine
        self.inits += 1
        if self.fail_init:
            raise engine.AccordDepsError(-6, "ncclCommInitRank failed (stand-in)")

    def comm_destroy(self):
        self.destroys += 1


def _worker(rank, world, port, case, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "cassandra-accord_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from accord_amd import sharding
        device = 0 if case == "shared_gpu" else rank
        store = _Store(device, fail_init=(case == "init_fails" and rank == 1))
        if case == "no_uid" or case == "init_fails" or case == "ok":
            # ncclGetUniqueId needs the library on a GPU node: a stand-in id (None on rank 0 = unavailable)
            sharding.unique_id = (lambda: None) if case == "no_uid" else (lambda: b"\x01" * 128)
        if case == "shared_gpu":
            sharding.unique_id = lambda: b"\x01" * 128
        tr = bench.pick_transport("rccl", dist, store, rank, world)
        q.put((rank, tr.name, store.inits, store.destroys))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,want", [("shared_gpu", "host"), ("no_uid", "host"), ("init_fails", "host"), ("ok", "rccl")])
def test_transport_falls_back_together(case, want):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0, "rank exited with %s" % p.exitcode
    got = sorted(q.get(timeout=5) for _ in range(world))
    names = {g[1] for g in got}
    assert names == {"host(gloo)" if want == "host" else "rccl"}, got
    if case == "init_fails":                   # rank 0's init succeeded: it dropped its communicator
        assert got[0][2:] == (1, 1) and got[1][2:] == (1, 0), got
    if case == "shared_gpu":                   # decided before any init
        assert all(g[2] == 0 for g in got), got
