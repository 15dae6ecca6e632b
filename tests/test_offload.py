"""The shared-memory link of include/fd_verify_offload.h (SURVEY.md §8(f)
next-1: verify tile <-> GPU offload process).  CPU tests drive the client
API against a stand-in server written with the server primitives (no GPU):
ordering, byte integrity through the FIFO frag area and its wrap, flow
control, result-slot reuse, and a client in a separate process.  The GPU
form (fd_verify_offload_serve behind the same link) is in
tests/test_verify_stage.py."""
import multiprocessing as mp
import os

import numpy as np
import pytest

import firedancer_amd as fa

NAME = "/fdvo_test_%d" % os.getpid()


@pytest.fixture
def link():
    srv = fa.OffloadLink.create(NAME, depth=16, dcache_sz=4096)
    cli = fa.OffloadLink.join(NAME)
    yield srv, cli
    cli.close()
    srv.close()


def fake_serve(srv, fn, max_take=None):
    """Take every available frag (in ring-contiguous runs), read its bytes
    from the frag area, and complete it with result fn(bytes)."""
    out = []
    while True:
        first, n = srv.avail()
        if not n:
            return out
        if max_take:
            n = min(n, max_take)
        fr = srv.frags(first, n).copy()
        dc = srv.dcache_view()
        res = srv.results_view(first, n)
        sig = srv.sigs_view(first, n)
        for i in range(n):
            b = dc[fr[i, 0]:fr[i, 0] + fr[i, 1]].tobytes()
            r, s = fn(b)
            res[i] = r
            sig[i] = s
            out.append((first + i, int(fr[i, 0]), b))
        srv.take(n)
        srv.complete(first + n)


def _frag(i, sz):
    return bytes((i * 7 + j) & 255 for j in range(sz))


def test_roundtrip_in_order(link):
    srv, cli = link
    frags = [_frag(i, 50 + 37 * i) for i in range(10)]
    seqs = [cli.publish(f) for f in frags]
    assert seqs == list(range(10))
    assert cli.result(3) == (0, 0, 0)                    # published, not done
    assert cli.result(10)[0] == fa.offload.ERR_SEQ       # never published
    got = fake_serve(srv, lambda b: (len(b) % 3 - 1, len(b)))
    assert [g[2] for g in got] == frags
    for i, f in enumerate(frags):
        assert cli.result(i) == (1, len(f) % 3 - 1, len(f))
    assert cli.done_seq() == cli.prod_seq() == 10


def test_flow_control_ring_and_frag_area(link):
    srv, cli = link
    # ring: 16 in flight max
    for i in range(16):
        assert cli.publish(_frag(i, 64)) == i
    assert cli.publish(_frag(99, 64)) == fa.offload.ERR_FULL
    fake_serve(srv, lambda b: (0, 1), max_take=4)        # drains all, in runs of 4
    assert cli.done_seq() == 16
    # results of seq s stay until s + depth is published
    assert cli.result(0)[0] == 1
    assert cli.publish(_frag(16, 64)) == 16
    assert cli.result(0)[0] == fa.offload.ERR_SEQ
    assert cli.result(1)[0] == 1
    # frag area: 4096 B; 1000-B frags take 1024 each -> 4 fit, the 5th waits
    fake_serve(srv, lambda b: (0, 0))
    n0 = cli.prod_seq()
    for i in range(4):
        assert cli.publish(_frag(i, 1000)) == n0 + i
    assert cli.publish(_frag(5, 1000)) == fa.offload.ERR_FULL
    assert cli.publish(_frag(5, 64)) == fa.offload.ERR_FULL   # no room at all until a completion
    fake_serve(srv, lambda b: (0, 0), max_take=1)
    assert cli.publish(_frag(5, 1000)) >= 0


def test_frag_area_wrap_keeps_bytes(link):
    """Random sizes through a small frag area with a consumer that lags by a
    random amount: every frag's bytes arrive intact, offsets wrap, and no
    in-flight frag is ever overwritten."""
    srv, cli = link
    rng = np.random.default_rng(1)
    sent = {}
    wrapped = False
    last_off = -1
    for k in range(3000):
        sz = int(rng.integers(1, 1500))
        f = rng.bytes(sz)
        s = cli.publish(f)
        if s == fa.offload.ERR_FULL:
            got = fake_serve(srv, lambda b: (0, 0), max_take=int(rng.integers(1, 6)))
            for seq, off, b in got:
                assert b == sent.pop(seq), seq
                wrapped |= off < last_off
                last_off = off
            continue
        assert s >= 0
        sent[s] = f
    for seq, off, b in fake_serve(srv, lambda b: (0, 0)):
        assert b == sent.pop(seq)
    assert not sent and wrapped


def _client_proc(name, n, q):
    import firedancer_amd as fa2
    cli = fa2.OffloadLink.join(name)
    seq = 0
    while seq < n:
        s = cli.publish(_frag(seq, 100 + seq % 200))
        if s == fa2.offload.ERR_FULL:
            continue
        seq += 1
    res = []
    for s in range(max(0, n - 16), n):
        while True:
            st, r, g = cli.result(s)
            if st == 1:
                break
        res.append((s, r, g))
    cli.halt()
    cli.close()
    q.put(res)


def test_client_in_another_process():
    srv = fa.OffloadLink.create(NAME + "_p", depth=16, dcache_sz=8192)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_client_proc, args=(NAME + "_p", 500, q))
    p.start()
    import time
    t0 = time.time()
    seen = 0
    while time.time() - t0 < 60:
        got = fake_serve(srv, lambda b: (len(b) & 1, len(b)))
        for seq, off, b in got:
            assert b == _frag(seq, 100 + seq % 200)
            seen += 1
        if not got and srv.lib.fd_verify_offload_halted(srv.h):
            break
    res = q.get(timeout=30)
    p.join(30)
    srv.close()
    assert seen == 500
    assert res == [(s, (100 + s % 200) & 1, 100 + s % 200) for s in range(484, 500)]


def test_burst_publish_and_results(link):
    srv, cli = link
    arena = np.frombuffer(b"".join(_frag(i, 200) for i in range(40)), np.uint8).copy()
    fr = np.zeros(40, fa.FRAG_DTYPE)
    fr["off"] = np.arange(40) * 200
    fr["sz"] = 200
    n = cli.publish_burst(arena, fr)
    assert n == 16                      # ring depth; (16 x 256 B chunks = 4096 B also exactly fit)
    res = np.zeros(40, np.int8); sig = np.zeros(40, np.uint64)
    assert cli.results(0, res[:16], sig[:16]) == 0
    fake_serve(srv, lambda b: (b[0] & 1, b[1]), max_take=5)
    assert cli.results(0, res[:40], sig[:40]) == 16
    assert list(sig[:16]) == [_frag(i, 200)[1] for i in range(16)]
    assert cli.publish_burst(arena, fr[16:]) == 16


# Header layout of fd_verify_offload.cpp (struct hdr): the geometry words,
# then one 64-B line per cursor.
_H_DEPTH, _H_DSZ, _H_FOOT, _H_FRAG, _H_RES, _H_SIG, _H_DC = 8, 16, 24, 32, 40, 48, 56
_H_PROD, _H_CURSOR, _H_CONS, _H_DONE = 64, 72, 128, 192


def _shm_u64(name):
    """Writable u64 view of the link's first page, as another process (a
    buggy or hostile client) would map it."""
    import mmap
    fd = os.open("/dev/shm" + name, os.O_RDWR)
    m = mmap.mmap(fd, 4096)
    os.close(fd)
    return m


def _put(m, off, v):
    m[off:off + 8] = int(v).to_bytes(8, "little")


def test_corrupt_header_cannot_move_server_out_of_bounds():
    """the server must not take the ring geometry or its own
    consumer cursor from the shared header after create.  A client that
    rewrites depth / region offsets / cons_seq / prod_seq leaves the server
    indexing inside its own validated ring."""
    name = NAME + "_c"
    srv = fa.OffloadLink.create(name, depth=16, dcache_sz=4096)
    cli = fa.OffloadLink.join(name)
    try:
        for i in range(5):
            assert cli.publish(_frag(i, 100)) == i
        m = _shm_u64(name)
        _put(m, _H_DEPTH, 1 << 40)            # geometry rewritten behind the server's back
        _put(m, _H_DSZ, 1 << 40)
        _put(m, _H_FRAG, 1 << 50)
        _put(m, _H_RES, 1 << 50)
        _put(m, _H_SIG, 1 << 50)
        _put(m, _H_DC, 1 << 50)
        _put(m, _H_CONS, 12345678)            # the server's cursor is private: this is ignored
        assert srv.depth == 16 and srv.dcache_sz == 4096
        first, n = srv.avail()
        assert (first, n) == (0, 5)
        got = fake_serve(srv, lambda b: (0, len(b)))
        assert [g[2] for g in got] == [_frag(i, 100) for i in range(5)]
        assert int.from_bytes(m[_H_CONS:_H_CONS + 8], "little") == 5   # published one way
        # a client claiming far more in flight than the ring holds: capped at depth, ring-contiguous
        _put(m, _H_PROD, 5 + (1 << 33))
        first, n = srv.avail()
        assert first == 5 and 0 < n <= 16 - (5 % 16)
        _put(m, _H_PROD, 3)                    # prod behind cons: nothing available
        assert srv.avail() == (5, 0)
        # the client's own handle also keeps its validated geometry
        assert cli.depth == 16 and cli.dcache_sz == 4096
        m.close()
    finally:
        cli.close()
        srv.close()


@pytest.mark.parametrize("field,value", [
    (_H_DEPTH, 24),                # not a power of two
    (_H_DEPTH, 1 << 30),           # rings past the mapping
    (_H_DSZ, 100),                 # not a multiple of 64
    (_H_DSZ, 1 << 30),             # frag area past the mapping
    (_H_FRAG, 1 << 40),
    (_H_RES, 1 << 62),
    (_H_SIG, 7),                   # misaligned / inside the header
    (_H_DC, (1 << 64) - 64),       # offset + size wraps around
])
def test_join_refuses_bad_geometry(field, value):
    name = NAME + "_g"
    srv = fa.OffloadLink.create(name, depth=16, dcache_sz=4096)
    try:
        m = _shm_u64(name)
        _put(m, field, value)
        m.close()
        with pytest.raises(fa.GpuError):
            fa.OffloadLink.join(name)
        assert srv.depth == 16         # the creator is unaffected
    finally:
        srv.close()
