"""GPU: the in-process multi-device path (VERDICT r01 missing #2) on one GPU.

fd_ed25519_gpu_new_devs maps shard slots to devices with repeats allowed, so
a context with three slots on device 0 runs exactly the code a three-GPU
context runs: batch sharding in fd_ed25519_gpu_submit (contiguous thirds,
each slot with its own stream, tables and staging), frag sharding in
fd_ed25519_gpu_frags_submit / _poll, the hot-key cache on every slot.  Also
the scratch-ordering rule of the device-pointer entry: two
batches launched back to back on two different streams of one slot must not
overwrite each other's tables."""
import ctypes as C

import numpy as np
import pytest

import firedancer_amd as fa
from golden_io import read_sigs, read_txns

pytestmark = pytest.mark.gpu

SLOTS = [0, 0, 0]


@pytest.fixture(scope="module")
def mgpu():
    g = fa.Ed25519Gpu(devices=SLOTS, max_batch=1 << 14)
    assert g.device_cnt() == len(SLOTS)
    yield g
    g.close()


def _golden():
    return read_sigs("vectors_ref.bin") + read_sigs("synthetic.bin")


@pytest.mark.parametrize("flavour,key", [(fa.CODES_AVX512, "code"), (fa.CODES_REF, "code_ref")])
def test_sharded_golden_parity(mgpu, flavour, key):
    recs = _golden()
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    mgpu.set_codes(flavour)
    try:
        out = mgpu.verify_batch(arena, sz, desc)
    finally:
        mgpu.set_codes(fa.CODES_AVX512)
    assert np.array_equal(out, np.array([r[key] for r in recs], np.int8))


@pytest.mark.parametrize("n", [1, 2, 3, 4, 7])
def test_sharded_small_batches(mgpu, n):
    """fewer descriptors than slots: empty shards are skipped"""
    recs = _golden()[:n]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    assert np.array_equal(mgpu.verify_batch(arena, sz, desc), np.array([r["code"] for r in recs], np.int8))


def test_sharded_txn_reduce(mgpu):
    txns = [t for t in read_txns() if 1 <= t["n"] <= 16] + [t for t in read_txns("cctv_batches.bin")]
    recs = []
    for ti, t in enumerate(txns):
        for j in range(t["n"]):
            recs.append((t["msg"], t["sigs"][j], t["pubs"][j], ti & 0xffff))
    arena, desc, sz = fa.pack_batch(recs)
    codes = mgpu.verify_batch(arena, sz, desc)
    assert np.array_equal(fa.txn_reduce(codes, desc), np.array([t["code"] for t in txns], np.int8))


def test_sharded_async_submit_poll(mgpu):
    recs = _golden()[:999]
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    out = np.zeros(len(desc), np.int8)
    mgpu.submit(arena, sz, desc, out)
    import time
    t0 = time.time()
    while not mgpu.poll():
        assert time.time() - t0 < 60
        time.sleep(0.001)
    assert np.array_equal(out, np.array([r["code"] for r in recs], np.int8))


def _ring_relayout(arena, frags, ring_sz, start, chunk=64):
    """The same frags laid out in a dcache-like ring of ring_sz bytes from
    `start`: a frag that would cross the ring's end starts again at 0, so
    the batch wraps (frag order != arena order).  fd_txn_t offsets are
    payload-relative and chunks stay 64-B aligned, so every frag parses the
    same."""
    out = np.zeros(ring_sz, np.uint8)
    fr = frags.copy()
    pos = start
    for i in range(len(frags)):
        o, z = int(frags["off"][i]), int(frags["sz"][i])
        if pos + z > ring_sz:
            pos = 0
        out[pos:pos + z] = arena[o:o + z]
        fr["off"][i] = pos
        pos += (z + chunk - 1) // chunk * chunk
    assert pos < start
    return out, fr


@pytest.mark.parametrize("layout", ["packed", "wrapped_ring"])
def test_sharded_device_parse_stage_vs_reference_tile(mgpu, layout):
    """The async verify stage with the frags parsed on the GPU, its frag batches
    sharded over the three slots (fd_ed25519_gpu_frags_submit), against the
    sequential reference tile -- also with the frags in a wrapped dcache ring,
    where each slot copies the page runs its shard occupies (cp_plan: two of
    them for the slot holding the wrap) and parses rebased frag records."""
    import os
    import test_verify_stage as tvs
    if not os.path.exists(tvs.REF_SO):
        pytest.skip("oracle/_ref not built")
    ref = C.CDLL(tvs.REF_SO)
    ref.fdref_verify_frags_seq.argtypes = [C.c_void_p, C.c_void_p, C.c_ulong, C.c_ulong, C.c_ulong,
                                           C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(303)
    arena, frags = tvs._random_frag_stream(rng, 600, 1500)
    if layout == "wrapped_ring":
        arena, frags = _ring_relayout(arena, frags, len(arena) + (1 << 20), len(arena) // 2 + (1 << 20))
    exp_res, exp_tag = tvs.ref_seq(ref, arena, frags)
    lib = fa.load_lib()
    vp = C.c_void_p
    lib.fd_ed25519_gpu_stage_new.restype = vp
    lib.fd_ed25519_gpu_stage_new.argtypes = [vp, vp, C.c_uint64, C.c_int]
    lib.fd_ed25519_gpu_stage_submit.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp, vp]
    lib.fd_ed25519_gpu_stage_poll.argtypes = [vp, C.c_int]
    lib.fd_ed25519_gpu_stage_pending.argtypes = [vp]
    lib.fd_ed25519_gpu_stage_delete.argtypes = [vp]
    lib.fd_ed25519_gpu_stage_set_device_parse.argtypes = [vp, C.c_int]
    tc = fa.TCache()
    st = lib.fd_ed25519_gpu_stage_new(mgpu.ctx, tc.tc, 1024, 4)
    assert st
    assert lib.fd_ed25519_gpu_stage_set_device_parse(st, 1) == 0
    res = np.zeros(len(frags), np.int8)
    sig = np.zeros(len(frags), np.uint64)
    fr = np.ascontiguousarray(frags)
    i = 0
    for b in [1, 2, 3, 500, 1024, 10 ** 9]:
        if i >= len(frags):
            break
        b = min(b, len(frags) - i)
        while True:
            r = lib.fd_ed25519_gpu_stage_submit(st, arena.ctypes.data, len(arena), fr[i:].ctypes.data, b,
                                                res[i:].ctypes.data, sig[i:].ctypes.data)
            if r != -104:
                break
            assert lib.fd_ed25519_gpu_stage_poll(st, 1) == 0
        assert r == 0, r
        i += b
    while lib.fd_ed25519_gpu_stage_pending(st):
        assert lib.fd_ed25519_gpu_stage_poll(st, 1) == 0
    lib.fd_ed25519_gpu_stage_delete(st)
    bad = np.nonzero((res != exp_res) | (sig != exp_tag))[0]
    assert len(bad) == 0, [(int(j), int(res[j]), int(exp_res[j])) for j in bad[:10]]


def test_sharded_far_fields_copy_runs(mgpu):
    """fd_ed25519_gpu_submit over three slots with every public key in a key
    area 48 MB past the signatures and messages: each slot copies its two
    page runs (cp_plan), not a 48 MB span, and the rebased descriptors give
    the golden codes."""
    recs = _golden()
    arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
    far = 48 << 20
    big = np.zeros(far + 32 * len(recs) + 64, np.uint8)
    big[:sz] = arena[:sz]
    d = desc.copy()
    for j, r in enumerate(recs):
        big[far + 32 * j:far + 32 * j + 32] = np.frombuffer(r["pub"], np.uint8)
        d["pub_off"][j] = far + 32 * j
    mgpu.host_stats(reset=True)
    out = np.full(len(recs), 99, np.int8)
    mgpu.submit(big, len(big), d, out)
    assert mgpu.poll(block=True)
    assert np.array_equal(out, np.array([r["code"] for r in recs], np.int8))
    sent = mgpu.host_stats()["h2d_bytes"]
    assert sent < sz + 32 * len(recs) + 16 * len(recs) + 3 * 4 * 2 * 4096 * 17, sent


def test_sharded_keycache(mgpu):
    recs = _golden()
    keys = sorted({r["pub"] for r in recs})
    mgpu.keycache_reserve(len(keys))
    try:
        assert mgpu.keycache_add(keys[::2]) == len(keys[::2])
        arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in recs])
        assert np.array_equal(mgpu.verify_batch(arena, sz, desc), np.array([r["code"] for r in recs], np.int8))
    finally:
        mgpu.keycache_clear()


def test_dev_entry_two_streams_back_to_back(gpu):
    """Two different batches on two streams with no host sync between the
    launches: each launch waits for the slot's previous one (scratch event),
    so both keep their own tables and both are bit-exact."""
    import torch
    recs = _golden()
    a_recs, b_recs = recs[:2000], recs[-2000:][::-1]
    outs = []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = []
    for rs, st in zip((a_recs, b_recs), streams):
        arena, desc, sz = fa.pack_batch([(r["msg"], r["sig"], r["pub"]) for r in rs])
        d_arena = torch.from_numpy(arena.copy()).to("cuda:0")
        d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to("cuda:0")
        d_out = torch.full((len(desc),), 99, dtype=torch.int8, device="cuda:0")
        bufs.append((d_arena, d_desc, d_out, sz, len(desc), st))
    torch.cuda.synchronize()
    for _ in range(3):
        for d_arena, d_desc, d_out, sz, n, st in bufs:
            gpu.verify_batch_dev(d_arena.data_ptr(), sz, d_desc.data_ptr(), n, d_out.data_ptr(), stream=st.cuda_stream)
    torch.cuda.synchronize()
    for (d_arena, d_desc, d_out, sz, n, st), rs in zip(bufs, (a_recs, b_recs)):
        assert np.array_equal(d_out.cpu().numpy(), np.array([r["code"] for r in rs], np.int8))
