"""CPU, world_size 2 (gloo): the multi-GPU sharding / gather / timing logic of the
data-parallel path, with the oracle standing in for each rank's GPU shard."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import firedancer_amd.ed25519 as fe
        from firedancer_amd.dist import aggregate_throughput, gather_codes
        from firedancer_amd.shard import shard_range
        from golden_io import read_sigs
        recs = read_sigs("vectors_ref.bin")
        arena, desc, sz = fe.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
        n = len(desc)
        a, b = shard_range(n, rank, world)
        orc = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle_ed25519.so"))
        orc.fdo_verify_descs.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
        local = np.zeros(b - a, np.int8)
        d = np.ascontiguousarray(desc[a:b])
        orc.fdo_verify_descs(arena.ctypes.data_as(ctypes.c_void_p), d.ctypes.data_as(ctypes.c_void_p), b - a,
                             local.ctypes.data_as(ctypes.c_void_p), 0)
        full = gather_codes(local, n)
        items, secs = aggregate_throughput(b - a, 1.0 + rank)
        q.put((rank, full.tolist(), items, secs, [r["code"] for r in recs]))
    finally:
        dist.destroy_process_group()


def test_two_rank_shard_gather_and_timing():
    import subprocess
    if not os.path.exists(os.path.join(REPO, "oracle", "liboracle_ed25519.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle")])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, full, items, secs, golden in res:
        assert full == golden                 # gathered shards == reference codes, in order
        assert items == len(golden)           # SUM over ranks covers every descriptor once
        assert secs == 2.0                    # MAX over ranks
