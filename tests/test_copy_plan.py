"""CPU: the submit paths' copy plan.  A multi-slot
context copies each slot's shard to HBM as the 4 KB page runs its fields
touch (fd_ed25519_gpu_host.cpp cp_plan), not as one [min, max) span: on a
wrapped dcache ring (frag order != arena order) the old span of the slot
holding the wrap was nearly the whole ring, 8 slots could send 8x the bytes.
Checked through the host-only hook fd_ed25519_gpu_test_copy_plan: per-slot
bytes against the shard's own bytes, and the device image a slot would get
(runs at their packed offsets, offsets rebased as the submit paths rebase
them) byte-equal to the host arena at every field, with each offset's low
12 bits kept (the frag parse's align_up( addr, 2 ) depends on them)."""
import ctypes as C

import numpy as np
import pytest

import firedancer_amd as fa

PAGE = 4096
GAP = 16 * PAGE          # FD_CP_GAP pages bridged
FRAG = np.dtype([("off", "<u4"), ("sz", "<u4")])


def _lib():
    lib = fa.load_lib()
    vp = C.c_void_p
    lib.fd_ed25519_gpu_test_copy_plan.argtypes = [C.c_int, vp, C.c_uint64, vp, C.c_uint64, C.c_int, vp, vp,
                                                  vp, C.c_uint64, vp]
    return lib


def _plan(kind, items, arena, nslot, image_cap=None):
    lib = _lib()
    b = np.zeros(nslot, np.uint64); r = np.zeros(nslot, np.uint64)
    img = None if image_cap is None else np.zeros(nslot * image_cap, np.uint8)
    reb = np.zeros_like(items)
    p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
    rc = lib.fd_ed25519_gpu_test_copy_plan(kind, p(items), len(items), p(arena), len(arena), nslot, p(b), p(r),
                                           p(img), image_cap or 0, p(reb) if img is not None else None)
    assert rc == 0, rc
    return b, r, img, reb


def _ring(rng, n, ring_sz, start, chunk=64):
    """n frags of 200..1300 B in a dcache-like ring: consecutive chunks from
    `start`, a frag that would cross the ring's end starts again at 0"""
    arena = rng.integers(0, 256, ring_sz, dtype=np.uint8)
    fr = np.zeros(n, FRAG)
    pos = start
    for i in range(n):
        sz = int(rng.integers(200, 1301))
        if pos + sz > ring_sz:
            pos = 0
        fr[i] = (pos, sz)
        pos += (sz + chunk - 1) // chunk * chunk
    return arena, fr


def _shard_bounds(n, nslot):
    return [(n * i // nslot, n * (i + 1) // nslot) for i in range(nslot)]


@pytest.mark.parametrize("nslot", [1, 3, 8])
def test_wrapped_ring_copies_each_shard_once(nslot):
    rng = np.random.default_rng(11)
    ring = 8 << 20
    arena, fr = _ring(rng, 6000, ring, ring - (2 << 20))      # ~4.5 MB of frags, wrapping 2 MB in
    b, r, img, reb = _plan(1, fr, arena, nslot, image_cap=ring)
    for i, (lo, hi) in enumerate(_shard_bounds(len(fr), nslot)):
        own = int(fr["sz"][lo:hi].sum())
        old_span = int((fr["off"][lo:hi] + fr["sz"][lo:hi]).max() - fr["off"][lo:hi].min())
        wraps = bool((np.diff(fr["off"][lo:hi].astype(np.int64)) < 0).any())
        assert r[i] == (2 if wraps else 1), (i, r[i])
        # what the shard occupies (64-B chunks) plus a page at each end of each run
        assert own <= b[i] <= own * 1.06 + 2 * r[i] * PAGE, (i, b[i], own)
        if wraps:
            assert old_span > ring // 2 and b[i] < old_span - (1 << 20)   # the [min, max) span took the unused ring too
    assert b.sum() <= fr["sz"].sum() * 1.06 + 2 * r.sum() * PAGE
    # the device images: every frag byte-equal at its rebased offset, low 12 bits kept
    for i, (lo, hi) in enumerate(_shard_bounds(len(fr), nslot)):
        base = i * ring
        for j in range(lo, hi):
            o, z, o2 = int(fr["off"][j]), int(fr["sz"][j]), int(reb["off"][j])
            assert o2 % PAGE == o % PAGE and reb["sz"][j] == z
            assert np.array_equal(img[base + o2:base + o2 + z], arena[o:o + z]), j


def test_frags_outside_the_arena_get_an_offset_past_the_span():
    rng = np.random.default_rng(3)
    arena = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    fr = np.array([(0, 300), (1 << 20, 8), ((1 << 20) - 4, 8), (500, 1), (4096, 0), (8192, 700)], FRAG)
    b, r, img, reb = _plan(1, fr, arena, 1, image_cap=1 << 20)
    assert list(reb["off"][1:5]) == [0xFFFFFFFF] * 4            # out of bounds or shorter than 2 B: BAD_FRAG
    assert r[0] == 1 and b[0] == 8192 + 700                     # pages 0..2 (gap of one page bridged)
    for j in (0, 5):
        o, z, o2 = int(fr["off"][j]), int(fr["sz"][j]), int(reb["off"][j])
        assert np.array_equal(img[o2:o2 + z], arena[o:o + z])


def test_scattered_descriptors_image_and_far_fields():
    """descriptors whose sig / key / message sit in different places, some
    keys far away (a key table elsewhere in the workspace), empty messages"""
    rng = np.random.default_rng(5)
    asz = 64 << 20
    arena = rng.integers(0, 256, asz, dtype=np.uint8)
    n = 3000
    d = np.zeros(n, fa.DESC_DTYPE)
    d["sig_off"] = rng.integers(0, 2 << 20, n)
    d["pub_off"] = np.where(rng.random(n) < 0.2, rng.integers(40 << 20, (40 << 20) + 65536, n), rng.integers(0, 2 << 20, n))
    d["msg_sz"] = np.where(rng.random(n) < 0.05, 0, rng.integers(1, 1233, n))
    d["msg_off"] = rng.integers(0, 3 << 20, n)
    d["txn_idx"] = np.arange(n) & 0xffff
    for nslot in (1, 4):
        b, r, img, reb = _plan(0, d, arena, nslot, image_cap=8 << 20)
        # far keys: a second run per slot instead of a 38 MB span
        assert (r >= 2).all() and (b < (6 << 20)).all(), (b, r)
        for i, (lo, hi) in enumerate(_shard_bounds(n, nslot)):
            base = i * (8 << 20)
            for j in range(lo, hi):
                x, y = d[j], reb[j]
                for f, ln in (("sig_off", 64), ("pub_off", 32), ("msg_off", int(x["msg_sz"]))):
                    o, o2 = int(x[f]), int(y[f])
                    if ln:
                        assert o2 % PAGE == o % PAGE
                        assert np.array_equal(img[base + o2:base + o2 + ln], arena[o:o + ln]), (j, f)
                assert y["msg_sz"] == x["msg_sz"] and y["txn_idx"] == x["txn_idx"]


def test_one_contiguous_batch_is_one_run():
    rng = np.random.default_rng(9)
    arena, fr = _ring(rng, 2000, 16 << 20, 0)
    b, r, _, _ = _plan(1, fr, arena, 1)
    span = int(fr["off"][-1]) + int(fr["sz"][-1])
    assert r[0] == 1 and b[0] == span
